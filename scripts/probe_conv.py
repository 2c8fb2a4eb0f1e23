"""Time the implicit-GEMM convolution (mcgmil.features.conv2d) against torch's bf16 autocast
convolution (MIOpen) on ResNet-18's block convolutions at a config-5 bag (k = 916 instances of
224 x 224); one JSON line per layer shape, interleaved in one process."""
import json
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "montecarlo-gated-mil_amd"))
from mcgmil.features import conv2d  # noqa: E402

K = int(os.environ.get("PROBE_K", "916"))
# (Cin, H, Cout, k, stride, pad, count in ResNet-18)
LAYERS = [(64, 56, 64, 3, 1, 1, 4), (64, 56, 128, 3, 2, 1, 1), (64, 56, 128, 1, 2, 0, 1),
          (128, 28, 128, 3, 1, 1, 3), (128, 28, 256, 3, 2, 1, 1), (128, 28, 256, 1, 2, 0, 1),
          (256, 14, 256, 3, 1, 1, 3), (256, 14, 512, 3, 2, 1, 1), (256, 14, 512, 1, 2, 0, 1),
          (512, 7, 512, 3, 1, 1, 3)]


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
    tot_own = tot_torch = 0.0
    for cin, h, cout, k, s, p, count in LAYERS:
        conv = nn.Conv2d(cin, cout, k, s, p, bias=False).to(dev).eval()
        x = torch.randn(K, cin, h, h, device=dev).relu_().bfloat16().contiguous(
            memory_format=torch.channels_last)
        conv = conv.to(memory_format=torch.channels_last)
        oh = (h + 2 * p - k) // s + 1
        flop = 2.0 * K * oh * oh * cout * cin * k * k
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            tiles = {}
            for tile in [t for t in os.environ.get("PROBE_TILES", "").split(",") if t]:
                os.environ["MCGMIL_CONV_TILE"] = tile
                tiles[tile] = round(flop / timed(lambda: conv2d(conv, x)) / 1e9, 1)
            os.environ.pop("MCGMIL_CONV_TILE", None)
            own = timed(lambda: conv2d(conv, x))
            ref = timed(lambda: conv(x))
            y, yr = conv2d(conv, x), conv(x)
            dev_rel = float((y.float() - yr.float()).abs().max() / yr.float().abs().max())
        tot_own += own * count
        tot_torch += ref * count
        print(json.dumps({"cin": cin, "hw": h, "cout": cout, "k": k, "stride": s, "count": count,
                          "own_ms": round(own, 4), "torch_ms": round(ref, 4),
                          "own_tflops": round(flop / own / 1e9, 1),
                          "torch_tflops": round(flop / ref / 1e9, 1), "nrel_vs_torch": dev_rel,
                          "forced_tile_tflops": tiles}),
              flush=True)
    print(json.dumps({"resnet18_block_convs_ms": {"own": round(tot_own, 3), "torch": round(tot_torch, 3)}}))


if __name__ == "__main__":
    main()
