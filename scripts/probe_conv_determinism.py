"""Run-to-run bitwise determinism of the convolution kernels (one process, repeated launches on
the same inputs), per plan shape; prints mismatch counts and the worst deviation from fp64."""
import json
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "montecarlo-gated-mil_amd"))
from mcgmil.features import conv2d  # noqa: E402

dev = torch.device("cuda", 0)
SHAPES = [(2, 64, 12, 12, 128, 3, 1, 1), (3, 64, 56, 56, 64, 3, 1, 1), (2, 128, 28, 28, 256, 3, 1, 1),
          (2, 256, 14, 14, 512, 3, 2, 1), (4, 128, 25, 20, 128, 3, 1, 1), (2, 64, 56, 56, 128, 3, 2, 1)]
for N, cin, H, W, cout, k, s, p in SHAPES:
    torch.manual_seed(N + cin + H)
    conv = nn.Conv2d(cin, cout, k, s, p, bias=False).to(dev).bfloat16()
    x = torch.randn(N, cin, H, W, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y0 = conv2d(conv, x)
        ref = F.conv2d(x.double(), conv.weight.double(), None, s, p)
        bad = 0
        for _ in range(40):
            y = conv2d(conv, x)
            bad += int((y != y0).sum())
        err = float(((y0.double() - ref).abs() - 2.0 ** -8 * ref.abs()).max())
    print(json.dumps({"shape": [N, cin, H, W, cout, k, s, p], "mismatched_elements_over_40_runs": bad,
                      "max_excess_over_half_ulp": err}), flush=True)

# the sequence of tests/test_gpu_conv.py::test_conv2d_bf16_weights_and_repack, with other kernels
# (an fp64 convolution, the weight repack) between the launches, repeated
fails = 0
for it in range(300):
    torch.manual_seed(it)
    conv = nn.Conv2d(64, 128, 3, 1, 1, bias=False).to(dev).bfloat16()
    x = torch.randn(2, 64, 12, 12, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y1 = conv2d(conv, x)
        ref1 = F.conv2d(x.double(), conv.weight.double(), None, 1, 1)
        conv.weight.mul_(-2.0)
        y2 = conv2d(conv, x)
        y2b = conv2d(conv, x)
        conv.weight.mul_(-0.5)
        y1b = conv2d(conv, x)
    want = (-2.0 * y1.float()).bfloat16()
    bad = (y2 != want).nonzero()
    if bad.shape[0]:
        fails += 1
        i = tuple(bad[0])
        print(json.dumps({"iter": it, "n_bad": int(bad.shape[0]), "first": bad[:6].tolist(),
                          "y2": y2[i].item(), "want": want[i].item(), "fp64": -2.0 * ref1[i].item(),
                          "y2_repeat_equal": bool(torch.equal(y2, y2b)),
                          "y1_repeat_equal": bool(torch.equal(y1, y1b))}),
              flush=True)
print(json.dumps({"repack_sequence_failures_of_300": fails}), flush=True)

# the same with a positive power-of-two scale (no sign flip)
fails = 0
for it in range(300):
    torch.manual_seed(it)
    conv = nn.Conv2d(64, 128, 3, 1, 1, bias=False).to(dev).bfloat16()
    x = torch.randn(2, 64, 12, 12, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y1 = conv2d(conv, x)
        conv.weight.mul_(2.0)
        y2 = conv2d(conv, x)
        conv.weight.mul_(-1.0)
        y3 = conv2d(conv, x)
    fails += int(not torch.equal(y2, (2.0 * y1.float()).bfloat16()))
    if it < 300 and not torch.equal(y3, -y2):
        print(json.dumps({"iter": it, "negation_not_exact": int((y3 != -y2).sum())}), flush=True)
print(json.dumps({"scale_by_2_failures_of_300": fails}), flush=True)
