"""Config-5 fp32 feature extractor (the reference precision): ResNet-18 over one bag of k = 1,507
224-px instances with BatchNorm on the bag's statistics (infer.py:105-109,154), timed under the
layout / MIOpen-search choices the fp32 line could make. One JSON line per variant; the features
of every variant are compared with the first (max |diff| / max |ref|)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))

import torch  # noqa: E402


def main():
    from mcgmil import MultiHeadGatedAttentionMIL, deactivate_batchnorm
    dev = torch.device("cuda", 0)
    k = int(os.environ.get("PROBE_K", "1507"))
    torch.manual_seed(0)
    model = MultiHeadGatedAttentionMIL(pretrained=False, shared_attention=False)
    model.apply(deactivate_batchnorm)
    model.to(dev).eval()
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(1, k, 3, 224, 224, device=dev, generator=g)
    ref = None
    variants = [("weights channels_last (bench default)", True, False),
                ("weights NCHW", False, False),
                ("weights channels_last, MIOpen search", True, True),
                ("weights NCHW, MIOpen search", False, True)]
    for name, cl, bench in variants:
        torch.backends.cudnn.benchmark = bench
        model.feature_extractor.to(memory_format=torch.channels_last if cl else torch.contiguous_format)
        with torch.no_grad():
            for _ in range(2):
                H = model.extract_features(x)
            torch.cuda.synchronize()
            reps = 3
            t0 = time.perf_counter()
            for _ in range(reps):
                H = model.extract_features(x)
            torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / reps
        if ref is None:
            ref = H.clone()
        diff = float((H - ref).abs().max() / ref.abs().max())
        print(json.dumps({"variant": name, "k": k, "ms": round(ms, 2),
                          "tflops": round(k * 3.64 / ms, 1), "nrel_vs_first": diff}), flush=True)


if __name__ == "__main__":
    main()
