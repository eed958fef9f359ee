import json, sys
sys.path.insert(0, "tools")
import microbench
for b in (8192, 4096):
    for nm in (200, 192, 208, 184):
        print(json.dumps(microbench.case("panel", nm, nm, b, 100, reps=5)), flush=True)
