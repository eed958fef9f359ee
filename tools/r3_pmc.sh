set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 bash tools/pmc_panel.sh a
python3 - <<'PY'
import csv,glob,collections,os
for d in sorted(glob.glob('gpurun_out/pmc_panel_a/*_*/')):
    fs=glob.glob(d+'**/*counter_collection.csv',recursive=True)
    if not fs: print(d,'no csv'); continue
    agg=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
    for f in fs:
        for r in csv.DictReader(open(f)):
            k=r['Kernel_Name'][:40]
            if 'panel2' not in k: continue
            agg[r['Counter_Name']][r['Dispatch_Id']]+=float(r['Counter_Value'])
    print(d, {c: sum(v.values())/max(1,len(v)) for c,v in agg.items()}, {c: len(v) for c,v in agg.items()})
PY
# tail probe: 10-iteration phases, no plan, finisher thresholds 0 (panels only) and 512
for ft in 0 512; do
  GPAD_PANEL_NOPLAN=1 GPAD_PANEL_PHASE=10 GPAD_FINISH_THRESH=$ft TAG=r3p_ft$ft timeout -k 10 320 bash tools/tl_run.sh > /dev/null
  echo "== finisher threshold $ft"; tail -45 gpurun_out/r3p_ft${ft}_timeline.txt
done
