"""Effective shader clock of each kernel from a rocprofv3 GRBM pass (MI355X_MICROARCH.md 'DVFS
give-back': clock ~= GRBM_GUI_ACTIVE / 8 / kernel wall time, rocprofv3 summing the 8 XCDs; within
~3 % of the in-kernel s_memtime clock on dispatches of >= 10 ms). Joins counter_collection.csv
(GRBM_GUI_ACTIVE per dispatch) with kernel_trace.csv (start/end ns per dispatch) of the same run.
Usage: grbm_clock.py <rocprofv3 output dir>  -> JSON per kernel (median MHz, dispatches, ms)."""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc:
        sys.exit(f"no counter_collection.csv under {d}")
    gui = {}
    names = {}
    times = {}
    for r in csv.DictReader(open(cc[0])):
        did = r.get("Dispatch_Id")
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            gui[did] = gui.get(did, 0.0) + float(r["Counter_Value"])
            names[did] = r.get("Kernel_Name", "?")
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                times[did] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    if kt:
        for r in csv.DictReader(open(kt[0])):
            did = r.get("Dispatch_Id")
            if did in gui:
                times[did] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    per = collections.defaultdict(list)
    for did, g in gui.items():
        if did not in times:
            continue
        ns = times[did][1] - times[did][0]
        if ns <= 0:
            continue
        per[names[did]].append((g / 8.0 / (ns * 1e-9) / 1e6, ns * 1e-6))
    out = {}
    for k, v in per.items():
        mhz = [x for x, _ in v]
        ms = [y for _, y in v]
        out[k[:100]] = {"grbm_clock_mhz_median": round(statistics.median(mhz), 1),
                        "grbm_clock_mhz_min_max": [round(min(mhz), 1), round(max(mhz), 1)],
                        "dispatches": len(v), "ms_median": round(statistics.median(ms), 4)}
    print(json.dumps(dict(sorted(out.items(), key=lambda kv: -kv[1]["ms_median"] * kv[1]["dispatches"])),
                     indent=1))


if __name__ == "__main__":
    main()
