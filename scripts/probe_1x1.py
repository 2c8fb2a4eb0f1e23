"""Check the 1x1 / stride-2 streaming convolution on one shape: y against an fp64 convolution and
its statistics rows (Chan-combined) against the statistics of y itself."""
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "montecarlo-gated-mil_amd"))
from mcgmil.features import conv2d  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for (N, Cin, H, W, Cout, off) in [(3, 128, 13, 11, 256, 4.0), (3, 128, 13, 11, 256, 0.0), (2, 64, 28, 28, 128, 0.0)]:
        torch.manual_seed(0)
        conv = nn.Conv2d(Cin, Cout, 1, 2, 0, bias=False).to(dev).eval()
        x = (torch.randn(N, Cin, H, W, device=dev).relu_() + off).bfloat16().contiguous(memory_format=torch.channels_last)
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            y, part = conv2d(conv, x, stats=True)
        wb = conv.weight.detach().bfloat16().double()
        ref = F.conv2d(x.double(), wb, None, 2, 0)
        rel = ((y.double() - ref).abs() / (ref.abs() + 1e-3)).max().item()
        yd = y.double()
        mean_t = yd.mean(dim=(0, 2, 3))
        var_t = yd.var(dim=(0, 2, 3), unbiased=False)
        p = part.double()
        n = p[:, 0, :]
        tot = n.sum(0)
        mean_p = (p[:, 1, :] * n).sum(0) / tot
        m2 = p[:, 2, :].sum(0) + (n * (p[:, 1, :] - mean_p[None]) ** 2).sum(0)
        var_p = m2 / tot
        print(dict(shape=(N, Cin, H, W, Cout, off), parts=part.shape[0], count=(tot.min().item(), tot.max().item(), N * ((H + 1) // 2) * ((W + 1) // 2)),
                   y_rel=rel, mean_err=(mean_p - mean_t).abs().max().item(), std=var_t.sqrt().mean().item(),
                   var_rel=((var_p - var_t).abs() / (var_t + 1e-12)).max().item()), flush=True)


main()
