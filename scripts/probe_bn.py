"""Time the fused BN apply pass (batch statistics, + residual + ReLU) on a config-5 layer-1
activation (916 x 64 x 56 x 56 bf16, channels-last) for each library in MCGMIL_PROBE_LIBS."""
import json
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "montecarlo-gated-mil_amd"))


def run(tag):
    from mcgmil.features import batchnorm_act
    from mcgmil.resnet import deactivate_batchnorm
    dev = torch.device("cuda", 0)
    bn = nn.BatchNorm2d(64).to(dev).eval()
    deactivate_batchnorm(bn)
    x = torch.randn(916, 64, 56, 56, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x)
    out = {}
    for name, res in (("apply", None), ("apply_res", r)):
        with torch.no_grad():
            for _ in range(3):
                batchnorm_act(x, bn, True, res)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                batchnorm_act(x, bn, True, res)
            b.record()
            torch.cuda.synchronize()
            out[name + "_ms"] = round(a.elapsed_time(b) / 10, 4)
    print(json.dumps({"lib": tag, **out}))


def main():
    from mcgmil import _lib
    for path in [p for p in os.environ.get("MCGMIL_PROBE_LIBS", "").split(",") if p] or [None]:
        if path:
            _lib._lib = None
            _lib.lib_path = lambda path=path: path
            _lib.load()
        run(os.path.basename(path) if path else "tree")


if __name__ == "__main__":
    main()
