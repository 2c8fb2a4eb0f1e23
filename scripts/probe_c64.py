"""A/B of the ResNet layer-1 convolution (3x3 / stride 1 / 64 -> 64, conv3x3c64_kernel) across
variant builds of the library (MCGMIL_PROBE_LIBS=a.so,b.so; scripts/build_variants.sh), at a
config-5 bag (PROBE_K instances, default 1,507, of 56 x 56), interleaved in one process: plain,
with the BatchNorm statistics epilogue, and with statistics + input BatchNorm. One JSON line per
(library, variant): median ms, TFLOP/s, and whether y (and the statistics) are bitwise equal to
the first library's."""
import ctypes
import json
import os
import statistics
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "montecarlo-gated-mil_amd"))


def main():
    from mcgmil import _lib
    from mcgmil.features import _conv_args, packed_conv_weight
    dev = torch.device("cuda", 0)
    paths = [p for p in os.environ.get("MCGMIL_PROBE_LIBS", "").split(",") if p]
    libs = {os.path.basename(p): _lib.bind(p) for p in paths} or {"libmcgmil.so": _lib.load()}
    K = int(os.environ.get("PROBE_K", "1507"))
    rounds = int(os.environ.get("PROBE_ROUNDS", "5"))
    torch.manual_seed(0)
    conv = nn.Conv2d(64, 64, 3, 1, 1, bias=False).to(dev).eval()
    x = torch.randn(K, 64, 56, 56, device=dev).relu_().bfloat16().contiguous(memory_format=torch.channels_last)
    ab = torch.stack([torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev)]).contiguous()
    flops = 2.0 * K * 56 * 56 * 64 * 64 * 9
    with torch.no_grad():
        w = packed_conv_weight(conv, x)
    y = torch.empty_like(x)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def run(L, stats, inbn):
        a = _conv_args(conv, x)
        a.x, a.w, a.y = (ctypes.c_void_p(t.data_ptr()) for t in (x, w, y))
        part = None
        if inbn:
            a.in_ab, a.in_relu = ctypes.c_void_p(ab.data_ptr()), 1
        if stats:
            n = ctypes.c_int32()
            _lib.check(L.mcgmil_conv_stats_parts(ctypes.byref(a), ctypes.byref(n)), "parts")
            part = torch.empty((n.value, 3, 64), dtype=torch.float32, device=dev)
            a.stats = ctypes.c_void_p(part.data_ptr())
        _lib.check(L.mcgmil_conv2d(ctypes.byref(a), stream), "mcgmil_conv2d")
        return part

    variants = [(name, st, ib) for name in libs for (st, ib) in ((False, False), (True, False), (True, True))]
    ref, equal = {}, {}
    for name, st, ib in variants:
        part = run(libs[name], st, ib)
        torch.cuda.synchronize()
        out = (y.clone(), None if part is None else part.clone())
        key = (st, ib)
        if key not in ref:
            ref[key] = out
        # the statistics blocks depend on the grid (workgroups per CU), so compare their combination
        same = torch.equal(out[0], ref[key][0])
        if st:
            def comb(p):
                p = p.double()
                n = p[:, 0].sum(0)
                m = (p[:, 0] * p[:, 1]).sum(0) / n
                return m, (p[:, 2] + p[:, 0] * (p[:, 1] - m) ** 2).sum(0) / n
            m1, v1 = comb(out[1])
            m0, v0 = comb(ref[key][1])
            same = same and float((m1 - m0).abs().max()) < 1e-5 and float(((v1 - v0).abs() / v0).max()) < 1e-5
        equal[(name, st, ib)] = same
    times = {v: [] for v in variants}
    for _ in range(rounds):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(libs[v[0]], v[1], v[2])
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1))
    for v in variants:
        ms = statistics.median(times[v])
        print(json.dumps({"lib": v[0], "stats": v[1], "in_bn": v[2], "ms": round(ms, 4),
                          "tflops": round(flops / (ms * 1e-3) / 1e12, 1), "same": equal[v],
                          "all_ms": [round(t, 4) for t in times[v]]}), flush=True)


if __name__ == "__main__":
    main()
