"""Summarise a rocprofv3 counter_collection.csv per kernel: mean of each counter per dispatch,
and (for SQ counters) the derived utilisation fractions. Usage: pmc_summary.py file.csv"""
import collections
import csv
import json
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k = r.get("Kernel_Name", r.get("Kernel-Name", "?"))
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = dict(m)
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC"):
                if c in m:
                    d[c + "_frac"] = round(m[c] / wc, 4)
        if "SQ_BUSY_CYCLES" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            d["mfma_busy_per_busy_cycle"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / m["SQ_BUSY_CYCLES"], 4)
        out[k[:90]] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
