# PMC passes on fixed-N panel solves (N = 1 and N = 41, 4096 instances): instruction-cache and
# translation counters per dispatch, to locate the per-launch fixed cost.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for N in 1 41; do
  for P in "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_IFETCH" "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum" "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA"; do
    tag=$(echo $P | cut -d' ' -f1)
    rm -rf gpurun_out/pmcl_${N}_$tag
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmcl_${N}_$tag -o run -- python3 tools/nsolve.py --N $N > /dev/null 2>&1 || { echo "pass $P N=$N failed"; exit 1; }
    echo "== N=$N $P"; python3 tools/pmc_dispatch.py gpurun_out/pmcl_${N}_$tag --last 3
  done
done
