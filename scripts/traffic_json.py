"""Per-launch HBM traffic of the gate kernel from a FETCH_SIZE and a WRITE_SIZE pass of
scripts/pmc_passes.sh (their pmc_summary.py JSONs: mean counter value per dispatch of each kernel),
corrected as MI355X_MICROARCH.md's HBM section prescribes for gfx950 (FETCH_SIZE counts half the
bytes of wide coalesced reads: doubled; WRITE_SIZE exact; both KiB), written as the
profiles/<round>/gate_traffic*.json record bench.py's roofline.traffic reads.
Usage: traffic_json.py <pmc dir> <out.json> <workload: cfg3|cfg4> <command string>"""
import json
import os
import sys

import numpy as np


def main():
    d, out, workload, command = sys.argv[1:5]
    fetch = json.load(open(os.path.join(d, "fetch.json")))
    write = json.load(open(os.path.join(d, "write.json")))
    name = next(k for k in fetch if "gate_fused_kernel" in k or "gate_pipe_kernel" in k)
    f_kib, w_kib = fetch[name]["FETCH_SIZE"], write[name]["WRITE_SIZE"]
    T, L, C = 100, 512, 2
    if workload == "cfg3":
        sizes = [2048] * 512
        config = {"bags": 512, "N": 2048, "T": T, "dtype": "bf16", "shared": 0}
    else:
        sizes = np.random.default_rng(0).integers(256, 2049, 4096).tolist()   # bench.py cfg4
        config = {"bags": 4096, "N": "U(256,2048)", "T": T, "dtype": "bf16", "shared": 0}
    rows = sum(sizes)
    fused = "fused" in name
    # fused: H once + A once + Y; two-kernel gate only: H once + logits and z written (fp32 [T*rows, C] each)
    alg = rows * L * 2 + (T * C * rows * 4 if fused else 2 * T * rows * C * 4) + (len(sizes) * T * C * 4 if fused else 0)
    rec = {"path": "fused" if fused else "pipe", "kernel": name, "FETCH_SIZE_KiB": f_kib, "WRITE_SIZE_KiB": w_kib,
           "hbm_bytes_per_launch": int((2 * f_kib + w_kib) * 1024),
           "correction": "2 x FETCH_SIZE (gfx950 half-counting of wide reads) + WRITE_SIZE, per launch "
                         "(mean of the profiled launches)",
           "command": command, "config": config, "algorithmic_bytes_per_launch": alg,
           "algorithmic": ("H once (bf16) + A written once (fp32 [T, C, N] per bag) + Y" if fused else
                           "H once (bf16) + the fp32 logits and z workspace written ([T x rows, C] each); "
                           "softmax_pool_kernel reads them back in its own launch"),
           "ratio_to_algorithmic": round((2 * f_kib + w_kib) * 1024 / alg, 3)}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
