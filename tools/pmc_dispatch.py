"""Per-dispatch PMC counters of a rocprofv3 --pmc run (tools only): prints, in dispatch order, each
gpad kernel's counters (e.g. GRBM_GUI_ACTIVE = GPU clocks the dispatch spanned, SQ_WAVES, MFMA and
VALU instruction counts) so phases of one solve can be compared.
  python3 tools/pmc_dispatch.py <rocprof output dir> [--last N]"""
import argparse
import collections
import csv
import glob
import os

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--last", type=int, default=30)
args = ap.parse_args()
files = glob.glob(os.path.join(args.dir, "**", "*counter_collection.csv"), recursive=True)
rows = collections.OrderedDict()
names = []
for f in files:
    for r in csv.DictReader(open(f)):
        if "gpad" not in r["Kernel_Name"]:
            continue
        key = int(r["Dispatch_Id"])
        d = rows.setdefault(key, {"kernel": r["Kernel_Name"].split("(")[0][-40:], "grid": r.get("Grid_Size", "")})
        c = r["Counter_Name"]
        d[c] = d.get(c, 0.0) + float(r["Counter_Value"])
        if c not in names:
            names.append(c)
keys = sorted(rows)[-args.last:]
print(f"{'dispatch':>8} {'kernel':<40} " + " ".join(f"{n[:18]:>18}" for n in names))
for k in keys:
    d = rows[k]
    print(f"{k:>8} {d['kernel']:<40} " + " ".join(f"{d.get(n, 0):>18.0f}" for n in names))
