"""Config-5 bf16-vs-fp32 drift, step by step: which pipeline moves between runs?

Runs the bench's model/image/seed through bf16 and fp32 twice each (in the order given on the
command line, default "bf16 fp32 fp32 bf16") and prints the feature / A_mean / A_var drift of
every run against the first fp32 and the first bf16 run."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench_cfg5 as C5  # noqa: E402
from mcgmil import MultiHeadGatedAttentionMIL, deactivate_batchnorm  # noqa: E402
from mcgmil.infer import mc_predict_image  # noqa: E402
from mcgmil.patcher import ImagePatcher  # noqa: E402


def main():
    order = sys.argv[1:] or ["bf16", "fp32", "fp32", "bf16"]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = MultiHeadGatedAttentionMIL(pretrained=False, shared_attention=False)
    model.apply(deactivate_batchnorm)
    model.to(dev).eval()
    model.feature_extractor.to(memory_format=torch.channels_last)
    patcher = ImagePatcher(patch_size=C5.PS, overlap=C5.OVERLAP, empty_thresh=C5.THRESH)
    patcher.get_tiles(C5.H_IMG, C5.W_IMG)
    img = C5.synthetic_mammogram(dev, seed=5)
    runs = []
    for mode in order:
        model.compute_dtype = torch.bfloat16 if mode == "bf16" else torch.float32
        o = mc_predict_image(model, patcher, img, T=100, seed=6,
                             features_dtype=torch.bfloat16 if mode == "bf16" else None)
        torch.cuda.synchronize()
        f = o["features"].double()
        print(f"{mode}: k={len(o['tiles_indices'])} features |max| {f.abs().max():.4g} "
              f"mean {f.mean():.4g} finite {bool(torch.isfinite(f).all())}", flush=True)
        runs.append((mode, o))

    def nr(x, y):
        x, y = x.double(), y.double()
        return float((x - y).abs().max() / y.abs().max())

    for ref_mode in ("fp32", "bf16"):
        ref = next((o for m, o in runs if m == ref_mode), None)
        if ref is None:
            continue
        for i, (m, o) in enumerate(runs):
            print(f"run {i} ({m}) vs first {ref_mode}: features {nr(o['features'], ref['features']):.3g} "
                  f"A_mean {nr(o['A_mean'], ref['A_mean']):.3g} A_var {nr(o['A_var'], ref['A_var']):.3g} "
                  f"Y {float((o['Y'] - ref['Y']).abs().max()):.3g}", flush=True)


if __name__ == "__main__":
    main()
