"""Copy the rocprofv3 summaries of a gpurun session from gpurun_out/ into profiles/<tag>/ and
derive the per-launch HBM traffic of the gate kernel (MI355X_MICROARCH.md §HBM: FETCH_SIZE
counts half the bytes of wide coalesced reads on gfx950, so it is doubled; WRITE_SIZE is exact
for 16-B-per-lane stores; both in KiB).

Usage: python scripts/save_profiles.py r01
"""
import csv
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")


def main(tag):
    dst = os.path.join(REPO, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    ks = os.path.join(OUT, f"kernel_stats_{tag}.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(dst, "kernel_stats.csv"))
    for src, name in ((f"kernel_stats_cfg5_{tag}.csv", "kernel_stats_cfg5.csv"),
                      (f"pmc_sq_summary_{tag}.json", "pmc_sq_summary.json")):
        if os.path.exists(os.path.join(OUT, src)):
            shutil.copy(os.path.join(OUT, src), os.path.join(dst, name))
    for name in ("bench.log", "rocprof.log", "probe.log", "stamps.log", "ab.log", "bench_cfg5.log",
                 "bench_cfg4.log", "bench_dist1.log", "rocprof_cfg5.log",
                 "probe_image.log", "pytest_gpu.log", "smoke.log", "determinism.log"):
        p = os.path.join(OUT, name)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, name))
    traffic = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        p = os.path.join(OUT, f"pmc_{tag}_{ctr}.csv")
        if not os.path.exists(p):
            continue
        rows = [r for r in csv.DictReader(open(p)) if "gate_" in r["Kernel_Name"]]
        with open(os.path.join(dst, f"pmc_{ctr}.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
        traffic[ctr + "_KiB"] = statistics.median(float(r["Counter_Value"]) for r in rows)
        traffic["kernel"] = rows[0]["Kernel_Name"]
    if traffic:
        traffic["hbm_bytes_per_launch"] = int(
            (2 * traffic.get("FETCH_SIZE_KiB", 0) + traffic.get("WRITE_SIZE_KiB", 0)) * 1024)
        traffic["correction"] = "2 x FETCH_SIZE (gfx950 half-counting of wide reads) + WRITE_SIZE"
        traffic["command"] = ("rocprofv3 --pmc <CTR> --kernel-trace -- python bench.py --steps 3 "
                              "--warmup 1 --no-cpu-baseline (bench defaults: 16 bags x N=2048, "
                              "T=100, bf16, separate attention)")
        traffic["config"] = {"bags": 16, "N": 2048, "T": 100, "dtype": "bf16", "shared": 0}
        json.dump(traffic, open(os.path.join(dst, "gate_traffic.json"), "w"), indent=1)
    print(sorted(os.listdir(dst)))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
