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
        # fp32torch: the fp32 pipeline with this build's BatchNorm kernels off (torch/MIOpen only)
        os.environ["MCGMIL_FUSED_BN"] = "0" if mode == "fp32torch" else "1"
        # fp32nochunk: the fp32 convolutions unsplit (features.torch_conv)
        os.environ["MCGMIL_FP32_CONV_CHUNK"] = "0" if mode == "fp32nochunk" else "1"
        model.compute_dtype = torch.bfloat16 if mode == "bf16" else torch.float32
        o = mc_predict_image(model, patcher, img, T=100, seed=6,
                             features_dtype=torch.bfloat16 if mode == "bf16" else None)
        os.environ["MCGMIL_FUSED_BN"] = "1"
        torch.cuda.synchronize()
        f = o["features"].double()
        print(f"{mode}: k={len(o['tiles_indices'])} features |max| {f.abs().max():.4g} "
              f"mean {f.mean():.4g} finite {bool(torch.isfinite(f).all())}", flush=True)
        runs.append((mode, o))

    def nr(x, y):
        x, y = x.double(), y.double()
        return float((x - y).abs().max() / y.abs().max())

    if os.environ.get("PROBE_CPU") == "1":   # the same instances through the ResNet on the host
        from mcgmil.infer import IMAGENET_MEAN, IMAGENET_STD
        inst, ids, _ = patcher.convert_img_to_bag(img, seed=6, out_dtype=torch.float32,
                                                  normalize=(IMAGENET_MEAN, IMAGENET_STD))
        torch.manual_seed(0)
        cpu_model = MultiHeadGatedAttentionMIL(pretrained=False, shared_attention=False)
        cpu_model.apply(deactivate_batchnorm)
        cpu_model.load_state_dict({k: v.cpu() for k, v in model.state_dict().items()})
        cpu_model.eval()
        with torch.no_grad():
            f_cpu = cpu_model.extract_features(inst.cpu()[None])[0]
        print(f"cpu fp32: features |max| {f_cpu.abs().max():.4g} mean {f_cpu.mean():.4g}", flush=True)
        for i, (m, o) in enumerate(runs):
            print(f"run {i} ({m}) vs CPU fp32 features: nrel {nr(o['features'].cpu(), f_cpu):.3g}", flush=True)

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
