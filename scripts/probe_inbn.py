"""Time the input BatchNorm fused into the halo convolutions (conv2d(..., in_ab=...)) against the
plain convolution and the unfused pair (batchnorm_act + conv2d) on ResNet-18's 3x3 / stride 1
block shapes at a config-5 bag (k = 916 instances); one JSON line per shape, one process."""
import json
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "montecarlo-gated-mil_amd"))
from mcgmil.features import batchnorm_act, batchnorm_coefficients, conv2d, conv_input_bn  # noqa: E402
from mcgmil.resnet import deactivate_batchnorm  # noqa: E402

K = int(os.environ.get("PROBE_K", "916"))
LAYERS = [(64, 56, 64), (128, 28, 128)]      # (C, H, Cout): layer 1, layer 2


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dev = torch.device("cuda", 0)
    for c, h, cout in LAYERS:
        conv = nn.Conv2d(c, cout, 3, 1, 1, bias=False).to(dev).eval()
        bn = nn.BatchNorm2d(c)
        deactivate_batchnorm(bn)
        bn = bn.to(dev).eval()
        x = torch.randn(K, c, h, h, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        flop = 2.0 * K * h * h * cout * c * 9
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            assert conv_input_bn(conv, x)
            ab = batchnorm_coefficients(x, bn)
            plain = timed(lambda: conv2d(conv, x, stats=True))
            fused = timed(lambda: conv2d(conv, x, stats=True, in_ab=ab))
            apply = timed(lambda: batchnorm_act(x, bn, True))
        print(json.dumps({"cin": c, "hw": h, "cout": cout, "conv_ms": round(plain, 4),
                          "conv_with_input_bn_ms": round(fused, 4), "bn_apply_ms": round(apply, 4),
                          "unfused_pair_ms": round(plain + apply, 4),
                          "conv_tflops": round(flop / plain / 1e9, 1),
                          "conv_with_input_bn_tflops": round(flop / fused / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
