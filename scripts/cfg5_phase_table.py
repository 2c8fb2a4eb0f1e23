"""Per-phase time of one config-5 image's bf16 `features` stage, from a rocprofv3 kernel trace of
`bench.py --workload cfg5` (scripts/gpu_round6.sh step profcfg5).

The last complete image of the trace is cut at its stem dispatch; its convolution dispatches are
numbered in launch order (ResNet-18: layer 1 = 4, layers 2-4 = 5 each: downsample, conv1, conv2,
conv1, conv2), and every other dispatch joins the phase of the convolution before it (BatchNorm
statistics, residual / ReLU passes), the stem's until the first convolution. The stage ends at the
global average pool (the first non-backbone kernel after layer 4).
Usage: python scripts/cfg5_phase_table.py kernel_trace_cfg5.csv [out.json]"""
import csv
import json
import sys

CONV = ("conv3x3c64", "conv_dma_kernel", "conv3x3_halo_kernel", "conv1x1_kernel")
BACKBONE = CONV + ("stem_", "bn_", "_bn")
LAYER_CONVS = [4, 5, 5, 5]


def short(name):
    n = name.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda x: int(x["Start_Timestamp"]))
    stems = [i for i, x in enumerate(rows) if "stem_conv_kernel" in x["Kernel_Name"]]
    if len(stems) < 2:
        sys.exit("need at least two images in the trace")
    start = stems[-2]          # the last image whose layers all ran before the next image began
    if start > 0 and "stem_prep" in rows[start - 1]["Kernel_Name"]:
        start -= 1
    seq, nconv = [], 0
    bounds = [sum(LAYER_CONVS[:k + 1]) for k in range(4)]
    for x in rows[start:]:
        name = x["Kernel_Name"]
        is_conv = any(c in name for c in CONV)
        if nconv == bounds[-1] and not is_conv and not any(b in name for b in BACKBONE):
            break              # past layer 4's last BatchNorm pass: the head begins
        if is_conv:
            nconv += 1
        phase = "stem" if nconv == 0 else "layer%d" % (1 + sum(nconv > b for b in bounds[:-1]))
        kind = "conv" if is_conv else ("stem" if "stem_" in name else "bn")
        seq.append((phase, kind, short(name), int(x["Start_Timestamp"]), int(x["End_Timestamp"])))
    if nconv != bounds[-1]:
        sys.exit("trace image incomplete: %d convolutions" % nconv)
    wall = (seq[-1][4] - seq[0][3]) / 1e6
    table = {}
    for phase, kind, _, t0, t1 in seq:
        d = table.setdefault(phase, {"conv_ms": 0.0, "bn_ms": 0.0, "stem_ms": 0.0, "dispatches": 0})
        d[kind + "_ms"] += (t1 - t0) / 1e6
        d["dispatches"] += 1
    busy = sum((t1 - t0) for *_, t0, t1 in seq) / 1e6
    out = {"trace": sys.argv[1], "image_dispatches": len(seq), "wall_ms": round(wall, 4),
           "kernel_ms": round(busy, 4), "gaps_ms": round(wall - busy, 4),
           "phases": {k: {kk: round(vv, 4) if isinstance(vv, float) else vv for kk, vv in v.items()}
                      for k, v in table.items()},
           "dispatches": [{"phase": p, "kernel": n, "us": round((t1 - t0) / 1e3, 1)}
                          for p, _, n, t0, t1 in seq]}
    print("| phase | MFMA kernels (ms) | BN / stem passes (ms) | dispatches |")
    print("|---|---|---|---|")
    for k, v in table.items():
        print("| %s | %.3f | %.3f | %d |" % (k, v["conv_ms"] + v["stem_ms"], v["bn_ms"], v["dispatches"]))
    print("| all (wall %.3f ms, kernels %.3f, gaps %.3f) | | | %d |" % (wall, busy, wall - busy, len(seq)))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
