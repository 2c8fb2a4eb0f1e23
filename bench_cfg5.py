"""BASELINE config 5 (bench.py --workload cfg5): end-to-end per-image MCDO inference on one
MI355X per rank -- on-GPU ImagePatcher (7036 x 2800 synthetic mammogram, 3 channels, 224 px
tiles at the reference's inference settings, overlap_val_test 0.75 and empty_threshold 0.75
(config.yml:31,34): 5,781 tiles, ~1,500 kept, the dataset's ImageNet Normalize fused) ->
ResNet-18 feature extractor (batch-statistics BN over the bag) -> MCDO head kernel (T=100,
separate attention) -> softmax probabilities -> attention-map mean/std over passes on the image
grid (infer.py:187-219 without the plotting).

Two precisions (--features):
  fp32  the reference's precision end to end: fp32 instances, the build's fp32 MFMA convolutions
        (mcgmil_conv2d_f32, conv32_kernel: fp32 operands and accumulation; the 3-channel stem in its
        gather mode, features.py) and fused BN kernels, fp32 head operands;
  bf16  bf16 instances, the build's HIP backbone under autocast, bf16 head operands. The run
        also pushes its last image through the fp32 pipeline (same seed, untimed) and reports
        the drift of prob_mean / A_mean / Y against it.

A step = one image through all of that, the image already resident in HBM. Each rank runs its
own image per step (images are independent: weak scaling, no collective on the data path).
`roofline` prices the dominant stage, the ResNet-18 convolutions (3.64 GFLOP per 224 x 224
instance: 1.82 GMAC, torchvision's published count), against the bf16 dense MFMA peak.
`cpu_baseline` times the same pipeline on the host (oracle/patcher_ref.py, the in-repo ResNet
in fp32 and oracle/mcdo_ref.py with torch's dropout RNG) on a bounded sample, extrapolated to
one image.
"""
import json
import time

import numpy as np
import torch
import torch.distributed as dist

RESNET18_GFLOP = 3.64          # per 3 x 224 x 224 instance (2 x 1.82 GMAC)
# MI355X fp32 peak, vector = matrix (no xf32 on gfx950): 157.3 TFLOP/s spec, MI355X_MICROARCH.md
# spec table. The fp32 line's dominant stage is the ResNet: this build's fp32 MFMA convolutions
# (conv32_kernel, v_mfma_f32_16x16x4_f32) for the blocks and, in gather mode, the 3-channel stem
# (profiles/r03/conv32_bnfold/kernel_stats_cfg5_fp32.csv: no MIOpen kernel in the trace).
PEAK_FP32_TFLOPS = 157.3
H_IMG, W_IMG, PS, OVERLAP, THRESH = 7036, 2800, 224, 0.75, 0.75   # config.yml:31,34
BLOB = (0.30, 0.58)     # semi-axes of the breast region (fractions of H, W): k = 1,507 tiles kept


def synthetic_mammogram(dev, seed=5):
    """A breast-like positive region touching the left border on a zero background, grey
    repeated to 3 channels as the dataset does (dataset.py: unsqueeze(0).repeat(3, 1, 1))."""
    g = torch.Generator(device=dev).manual_seed(seed)
    yy = torch.arange(H_IMG, device=dev, dtype=torch.float32)[:, None]
    xx = torch.arange(W_IMG, device=dev, dtype=torch.float32)[None, :]
    blob = 1 - ((yy - 0.5 * H_IMG) / (BLOB[0] * H_IMG)) ** 2 - (xx / (BLOB[1] * W_IMG)) ** 2
    noise = torch.rand(H_IMG, W_IMG, device=dev, generator=g) * 0.05
    img = torch.where(blob > 0, blob + noise, torch.zeros_like(blob))
    return img[None].repeat(3, 1, 1).contiguous()


def cpu_baseline(k, T, budget_s=20.0):
    """The same pipeline on the host, bounded: the patcher on the whole image, the ResNet on a
    sample of instances, the head and the maps on a few passes -- each scaled to one image."""
    from mcgmil import MultiHeadGatedAttentionMIL, deactivate_batchnorm
    from oracle import mcdo_ref, patcher_ref
    from mcgmil import synthetic
    threads = torch.get_num_threads()
    img = synthetic_mammogram(torch.device("cpu"))
    t0 = time.perf_counter()
    tiles = patcher_ref.tile_grid(H_IMG, W_IMG, PS, OVERLAP)
    px = patcher_ref.nonzero_percent(img, tiles)
    ids = patcher_ref.select(px, THRESH, -1)
    t_patch = time.perf_counter() - t0
    model = MultiHeadGatedAttentionMIL(pretrained=False, shared_attention=False)
    model.apply(deactivate_batchnorm)
    model.eval()
    n_inst = 16
    inst = patcher_ref.crops(img, tiles, ids[:n_inst])
    with torch.no_grad():
        model.extract_features(inst[:2][None])                           # warm-up
        t0 = time.perf_counter()
        model.extract_features(inst[None])
        t_feat = (time.perf_counter() - t0) / n_inst * k
    arrays = synthetic.head_arrays(synthetic.head_state_dict(0, C=2, shared=False), 2, False)
    prm = mcdo_ref.HeadParams(arrays)
    H = synthetic.bag_features(42, k, 512)
    t_pass = 2
    with torch.no_grad():
        t0 = time.perf_counter()
        mcdo_ref.mc_inference_torch_rng(H, prm, t_pass, 0.1, 0.1)
        t_head = (time.perf_counter() - t0) / t_pass * T
    A = torch.softmax(torch.randn(t_pass, 1, 2, k), dim=-1)
    t0 = time.perf_counter()
    maps = patcher_ref.attention_maps(A, tiles, ids[:k], (1, H_IMG, W_IMG))
    patcher_ref.map_stats(maps)
    t_maps = (time.perf_counter() - t0) / t_pass * T
    total = t_patch + t_feat + t_head + t_maps
    return {"value": T / total, "unit": "bag-samples/s", "cores": threads, "kind": "port",
            "sample": f"one 7036x2800 image extrapolated from: patcher on the whole image "
                      f"({t_patch:.2f} s), ResNet-18 fp32 on {n_inst} of {k} instances "
                      f"({t_feat:.1f} s scaled), MCDO head on {t_pass} of {T} passes "
                      f"({t_head:.1f} s scaled), maps+stats on {t_pass} passes ({t_maps:.1f} s "
                      f"scaled); torch {torch.__version__} CPU, {threads} threads"}


def run(args, world, rank, dev, peak_tflops, calib=None):
    from mcgmil import MultiHeadGatedAttentionMIL, deactivate_batchnorm
    from mcgmil.infer import mc_predict_image
    from mcgmil.patcher import ImagePatcher
    T = args.T
    bf16 = args.features == "bf16"
    torch.manual_seed(0)
    model = MultiHeadGatedAttentionMIL(pretrained=False, shared_attention=bool(args.shared))
    model.apply(deactivate_batchnorm)                       # infer.py:154
    model.compute_dtype = torch.bfloat16 if bf16 else torch.float32
    model.to(dev).eval()
    model.feature_extractor.to(memory_format=torch.channels_last)
    patcher = ImagePatcher(patch_size=PS, overlap=OVERLAP, empty_thresh=THRESH)
    patcher.get_tiles(H_IMG, W_IMG)
    img = synthetic_mammogram(dev, seed=5 + rank)
    stream = torch.cuda.current_stream(dev)
    fdt = torch.bfloat16 if bf16 else None

    def step(i, events=None):
        return mc_predict_image(model, patcher, img, T=T, seed=1000 * rank + i, events=events,
                                features_dtype=fdt)

    for i in range(args.warmup):
        out = step(i)
    k = len(out["tiles_indices"])
    stage_ms = {}
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs = []
    for i in range(args.steps):
        ev = []
        step(args.warmup + i, ev)
        evs.append(ev)
    stream.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    for ev in evs:
        for (_, a), (name, b) in zip(ev[:-1], ev[1:]):
            stage_ms[name] = stage_ms.get(name, 0.0) + a.elapsed_time(b) / args.steps
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0])
    feat_tflops = k * RESNET18_GFLOP / stage_ms["features"]         # GFLOP / ms = TFLOP/s
    if rank != 0:
        return None
    drift = None
    if bf16:      # the same image and seed through the fp32 pipeline (untimed)
        seed = 1000 * rank + args.warmup + args.steps - 1
        ob = step(args.warmup + args.steps - 1)
        model.compute_dtype = torch.float32
        of = mc_predict_image(model, patcher, img, T=T, seed=seed, features_dtype=None)
        model.compute_dtype = torch.bfloat16
        am_f, am_b = of["A_mean"].double(), ob["A_mean"].double()
        drift = {"prob_mean_abs": float((ob["prob_mean"] - of["prob_mean"]).abs().max()),
                 "A_mean_nrel": float((am_b - am_f).abs().max() / am_f.abs().max()),
                 "A_var_nrel": float((ob["A_var"].double() - of["A_var"].double()).abs().max()
                                     / of["A_var"].double().abs().max()),
                 "Y_abs": float((ob["Y"] - of["Y"]).abs().max()),
                 "features_nrel": float((ob["features"].double() - of["features"].double()).abs().max()
                                        / of["features"].double().abs().max())}
    cpu = None if args.no_cpu_baseline or world > 1 or rank != 0 else cpu_baseline(k, T)   # rank 0, N=1
    images = world * args.steps
    return {
        "metric": "end-to-end images/sec x MCDO-samples (T=100), config 5", "value": images * T / el,
        "unit": "bag-samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": el * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.features,
        "data": "synthetic 7036x2800 mammogram-like image, random-init ResNet-18 and head",
        "config": {"workload": f"BASELINE config 5: {H_IMG}x{W_IMG} image -> {PS}px tiles "
                               f"(overlap {OVERLAP}, empty_thresh {THRESH}, {len(patcher.tiles)} "
                               f"tiles, k={k} kept) -> ResNet-18 {args.features} -> MCDO head "
                               f"T={T} -> attention map mean/std",
                   "images_per_s": images / el, "instances_per_bag": k, "T": T,
                   "features": ("bf16: HIP backbone (autocast), bf16 head operands" if bf16 else
                                "fp32: fp32 MFMA convolutions incl. the gather-mode stem + fused BN (HIP, conv32_kernel), fp32 head operands"),
                   "drift_vs_fp32_pipeline": drift,
                   "drift_note": (None if drift is None else
                                  "the bf16 line's uncertainty outputs approximate the fp32 (reference-precision) "
                                  "pipeline: A_var ~4% nrel, A_mean ~1%, the same as PyTorch-ROCm's own bf16 autocast "
                                  "pipeline on this bag (tests/test_gpu_pipeline.py bounds this build by 1.25x of it; "
                                  "DESIGN.md §7); the fp32 line (--features fp32) is the reference precision"),
                   "stage_ms": stage_ms, "parallelism": f"one image per GPU per step, {world} GPU(s)"},
        "roofline": {"bound": "mfma", "achieved": feat_tflops,
                     "peak": peak_tflops if bf16 else PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                     "frac": feat_tflops / (peak_tflops if bf16 else PEAK_FP32_TFLOPS), "traffic": None,
                     "kernel": "ResNet-18 feature extractor (the dominant stage): " +
                               ("stem + implicit-GEMM convolutions + fused BN (HIP, bf16)" if bf16 else
                                "fp32 MFMA convolutions (conv32_kernel, the stem in gather mode) + fused BN (HIP, fp32)"),
                     "algorithmic_tflop_per_launch": k * RESNET18_GFLOP / 1e3,
                     **(calib(feat_tflops, "bf16" if bf16 else "f32") if calib else {})},
        "cpu_baseline": cpu,
    }


if __name__ == "__main__":
    raise SystemExit("run through bench.py --workload cfg5")
