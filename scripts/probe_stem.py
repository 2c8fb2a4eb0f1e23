"""Time the fused ResNet stem (mcgmil_stem_forward) on one config-5 bag (916 instances of
3 x 224 x 224 bf16) against the torch layers it replaces (conv1 under autocast on channels-last
input + the fused BN/ReLU/max-pool), with HIP events. Prints one JSON line."""
import json
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "montecarlo-gated-mil_amd"))
from mcgmil.features import stem, bn_act  # noqa: E402
from mcgmil.resnet import deactivate_batchnorm  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    from mcgmil import _lib
    libs = [p for p in os.environ.get("MCGMIL_PROBE_LIBS", "").split(",") if p]
    if libs:     # A/B variant builds in one process: time the stem of each
        for path in libs:
            _lib._lib = None
            _lib.lib_path = lambda path=path: path
            _lib.load()
            run(os.path.basename(path))
        return
    run("tree")


def run(tag):
    dev = torch.device("cuda", 0)
    N = int(os.environ.get("STEM_N", "916"))
    torch.manual_seed(0)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(dev).eval()
    bn = nn.BatchNorm2d(64).to(dev).eval()
    deactivate_batchnorm(bn)
    pool = nn.MaxPool2d(3, 2, 1)
    x = torch.randn(N, 3, 224, 224, device=dev).bfloat16()
    xcl = x.contiguous(memory_format=torch.channels_last)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        own = timeit(lambda: stem(conv, bn, True, pool, x))
        ref = timeit(lambda: bn_act(bn, conv(xcl), True, pool=pool))
        y1 = stem(conv, bn, True, pool, x)
        y2 = bn_act(bn, conv(xcl), True, pool=pool)
    act_bytes = N * 112 * 112 * 64 * 2
    print(json.dumps({"lib": tag, "N": N, "own_ms": round(own, 4), "torch_layers_ms": round(ref, 4),
                      "max_abs_diff": float((y1.float() - y2.float()).abs().max()),
                      "own_GBps_min_traffic": round((x.numel() * 2 + 2 * act_bytes + y1.numel() * 2) / own / 1e6, 1)}))


if __name__ == "__main__":
    main()
