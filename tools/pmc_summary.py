"""Summarise a tools/profile.sh run: per-kernel average duration (kernel trace) and per-launch
PMC values, with the gfx950 corrections of MI355X_MICROARCH.md §HBM:
  * FETCH_SIZE (KiB) counts exactly half of a wide coalesced streaming read -> x2;
  * WRITE_SIZE (KiB) is exact for 16-B-per-lane stores;
  * effective clock = GRBM_GUI_ACTIVE / 8 (summed over 8 XCDs) / kernel duration.
Usage: python tools/pmc_summary.py gpurun_out/prof_<tag>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def main(d):
    out = {"kernels": {}}
    ks = glob.glob(os.path.join(d, "kt", "*kernel_stats.csv"))
    if ks:
        for r in csv.DictReader(open(ks[0])):
            out["kernels"][short(r["Name"])] = {
                "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                "total_ns": float(r["TotalDurationNs"]), "percent": float(r["Percentage"])}
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for sub in ("fetch", "write", "sq", "grbm"):
        for f in glob.glob(os.path.join(d, sub, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                if sub == "grbm" and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                    dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    pmc = {}
    for k, cs in vals.items():
        e = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in e:
            e["hbm_read_bytes_corrected"] = 2.0 * e["FETCH_SIZE"] * 1024.0
        if "WRITE_SIZE" in e:
            e["hbm_write_bytes"] = e["WRITE_SIZE"] * 1024.0
        if "hbm_read_bytes_corrected" in e and "hbm_write_bytes" in e:
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes_corrected"] + e["hbm_write_bytes"]
        if "GRBM_GUI_ACTIVE" in e and dur.get(k):
            ns = sum(dur[k]) / len(dur[k])
            e["effective_clock_ghz"] = e["GRBM_GUI_ACTIVE"] / 8.0 / ns
        if "SQ_INSTS_MFMA" in e and "SQ_INSTS_VALU" in e and e["SQ_INSTS_MFMA"] > 0:
            e["valu_non_mfma_per_mfma"] = (e["SQ_INSTS_VALU"] - e["SQ_INSTS_MFMA"]) / e["SQ_INSTS_MFMA"]
        # totals over the profiled run (per-launch averages mix phases of very different length)
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            e["launches"] = len(cs["FETCH_SIZE"])
            e["hbm_bytes_total"] = 2.0 * sum(cs["FETCH_SIZE"]) * 1024.0 + sum(cs["WRITE_SIZE"]) * 1024.0
        pmc[k] = e
    out["pmc_per_launch"] = pmc
    out["bench_args"] = os.environ.get("PROFILE_ARGS", "")
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
