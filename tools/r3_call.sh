# round-3 call: quad schedule-table variants, single-workgroup rates
set -e
cd $GRAFT_REPO_ROOT
for v in qa qb; do echo "$v $(GPAD_LIB=$PWD/tools/abl/$v.so timeout -k 10 200 python3 tools/quad_solo.py)"; done
