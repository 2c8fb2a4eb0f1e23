"""Time the ResNet-18 feature extractor on a config-5 bag (k instances of 3x224x224) under
several layouts / precisions / MIOpen search modes; one JSON line per variant."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "montecarlo-gated-mil_amd"))
from mcgmil import MultiHeadGatedAttentionMIL, deactivate_batchnorm  # noqa: E402

K = int(os.environ.get("PROBE_K", "916"))


def timed(fn, reps=5):
    fn()
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
    x32 = torch.randn(K, 3, 224, 224, device=dev)
    for bench in (False, True):
        torch.backends.cudnn.benchmark = bench
        for layout in ("nchw", "nhwc"):
            for prec in ("autocast", "bf16"):
                torch.manual_seed(0)
                m = MultiHeadGatedAttentionMIL(pretrained=False)
                m.apply(deactivate_batchnorm)
                fe = m.feature_extractor.to(dev).eval()
                mf = torch.channels_last if layout == "nhwc" else torch.contiguous_format
                fe.to(memory_format=mf)
                x = x32.to(torch.bfloat16).contiguous(memory_format=mf)
                if prec == "bf16":
                    fe.to(torch.bfloat16)

                def run():
                    with torch.no_grad():
                        if prec == "autocast":
                            with torch.autocast("cuda", dtype=torch.bfloat16):
                                return fe(x)
                        return fe(x)
                ms = timed(run)
                print(json.dumps({"benchmark": bench, "layout": layout, "prec": prec, "ms": ms,
                                  "TFLOPs": K * 3.64 / ms}), flush=True)


if __name__ == "__main__":
    main()
