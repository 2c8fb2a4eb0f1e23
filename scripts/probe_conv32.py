"""Time the fp32 backbone convolution (mcgmil_conv2d_f32) against MIOpen's fp32 convolution (the
torch layer, channels-last) on ResNet-18's convolution shapes at a config-5 bag (k instances,
default 1,507), interleaved in one process; also the native one with its BatchNorm statistics
epilogue (stats) and with an input BatchNorm too (stats_inbn). Prints one JSON line per shape:
ms and TFLOP/s of each, and the max |diff| / max |ref| between native and MIOpen."""
import json
import os
import statistics
import sys

import torch
import torch.nn as nn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))

# (Cin, H, W, Cout, k, stride, pad) of ResNet-18's convolutions, per 224-px instance (the stem first)
SHAPES = [(3, 224, 224, 64, 7, 2, 3), (64, 56, 56, 64, 3, 1, 1), (64, 56, 56, 128, 3, 2, 1), (64, 56, 56, 128, 1, 2, 0),
          (128, 28, 28, 128, 3, 1, 1), (128, 28, 28, 256, 3, 2, 1), (128, 28, 28, 256, 1, 2, 0),
          (256, 14, 14, 256, 3, 1, 1), (256, 14, 14, 512, 3, 2, 1), (256, 14, 14, 512, 1, 2, 0),
          (512, 7, 7, 512, 3, 1, 1)]


def main():
    from mcgmil.features import conv2d_f32, torch_conv
    dev = torch.device("cuda", 0)
    N = int(os.environ.get("PROBE_N", "1507"))
    rounds = int(os.environ.get("PROBE_ROUNDS", "5"))
    for (cin, h, w, cout, k, s, p) in SHAPES:
        torch.manual_seed(0)
        conv = nn.Conv2d(cin, cout, k, s, p, bias=False).to(dev).eval()
        x = torch.randn(N, cin, h, w, device=dev).contiguous(memory_format=torch.channels_last)
        oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        flops = 2.0 * N * oh * ow * cout * cin * k * k
        times = {"native": [], "miopen": [], "stats": [], "stats_inbn": []}
        ab = torch.stack([torch.rand(cin, device=dev) + 0.5, torch.randn(cin, device=dev)]).contiguous()
        fns = {"native": lambda: conv2d_f32(conv, x), "miopen": lambda: torch_conv(conv, x),
               "stats": lambda: conv2d_f32(conv, x, stats=True),
               "stats_inbn": lambda: conv2d_f32(conv, x, stats=True, in_ab=ab)}
        if cin % 16:
            del fns["stats_inbn"], times["stats_inbn"]
        with torch.no_grad():
            a = conv2d_f32(conv, x)
            b = torch_conv(conv, x)
            torch.cuda.synchronize()
            diff = float((a - b).abs().max() / b.abs().max())
            for _ in range(rounds):
                for name, fn in fns.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    fn()
                    e1.record()
                    torch.cuda.synchronize()
                    times[name].append(e0.elapsed_time(e1))
        out = {"shape": [N, cin, h, w, cout, k, s, p], "nrel_native_vs_miopen": diff}
        for name, t in times.items():
            ms = statistics.median(t)
            out[name + "_ms"] = round(ms, 4)
            out[name + "_tflops"] = round(flops / (ms * 1e-3) / 1e12, 1)
        print(json.dumps(out), flush=True)
        del x, a, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
