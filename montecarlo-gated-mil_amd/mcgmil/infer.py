"""MCDO inference driver -- the build's counterpart of the reference callers of mc_inference
(infer.py:187-219, net_utils.py:195-210), minus neptune, DICOM I/O and plotting.

Runs a whole list of bags (extracted features) through ONE varlen kernel launch and returns,
per bag, what the reference computes from (Y, A):
  probs  = softmax(Y, dim=-1)                          infer.py:195 / net_utils.py:207
  prob_mean, prediction = mean over passes, argmax     net_utils.py:208-210
  positive-class mean/median/std/IQR/min/max           infer.py:47-54
  mean entropy  -sum p log(p + 1e-10)                  infer.py:56-57
  attention mean / unbiased variance over passes       infer.py:216-219 (per instance; the
                                                       reference maps them onto the image)

mc_predict_image is the whole per-image loop of infer.py:187-219 on one GPU (BASELINE config 5):
image -> ImagePatcher bag (+ the dataset's T.Normalize, fused) -> ResNet feature extractor
(PyTorch-ROCm, batch-statistics BN over the bag) -> MCDO head kernel -> softmax probabilities
-> attention maps' mean/std over passes, reconstructed on the image grid.
"""
import contextlib
from typing import List, Optional, Sequence

import torch

from . import ops

IMAGENET_MEAN = (0.485, 0.456, 0.406)   # reference utils.py:50-51 (val/test transforms)
IMAGENET_STD = (0.229, 0.224, 0.225)


def uncertainty_summary(Y: torch.Tensor, prob_mean: Optional[torch.Tensor] = None) -> dict:
    """The per-bag statistics infer.py / net_utils.py derive from the MC logits Y [T, C]:
    softmax over classes per pass (infer.py:195), the mean-probability argmax (net_utils.py:
    207-210), the positive-class mean/median/std (ddof=0)/IQR/min/max over passes
    (infer.py:47-54, numpy's linear percentiles) and the mean entropy with the reference's
    +1e-10 (infer.py:56-57). prob_mean: the kernel's P_mean for this bag, if already computed."""
    probs = torch.softmax(Y, dim=-1)
    pos = probs[:, -1]
    q = torch.quantile(pos, torch.tensor([0.25, 0.5, 0.75], device=pos.device, dtype=pos.dtype))
    ent = -(probs * torch.log(probs + 1e-10)).sum(-1)
    pm = probs.mean(0) if prob_mean is None else prob_mean
    return {
        "probs": probs, "prob_mean": pm, "prediction": int(torch.argmax(pm)),
        "pos_mean": float(pos.mean()), "pos_median": float(q[1]),
        "pos_std": float(pos.std(unbiased=False)), "pos_iqr": float(q[2] - q[0]),
        "pos_min": float(pos.min()), "pos_max": float(pos.max()),
        "mean_entropy": float(ent.mean()),
    }


def mc_predict_bags(model, bags: Sequence[torch.Tensor], T: int = 50, seed: Optional[int] = None,
                    bag_ids: Optional[Sequence[int]] = None) -> List[dict]:
    """bags: list of feature matrices H_b [N_b, L] on one HIP device."""
    device = model._check_device(bags[0].device)
    if seed is None:
        seed = int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())
    sizes = [int(h.shape[0]) for h in bags]
    H = torch.cat([h.reshape(-1, model.L) for h in bags]).to(model.compute_dtype).contiguous()
    offs = ops.bag_offsets_tensor(sizes, device)
    ids = None
    if bag_ids is not None:
        ids = torch.as_tensor(list(bag_ids), dtype=torch.int64).to(torch.int32).to(device)
    head, packed = model.head_tensors(device)
    pf, pa = model.feature_dropout.p, model.attention_dropouts[0].p
    with torch.no_grad():
        out = ops.mcdo_forward(H, offs, head, T, p_feat=pf, p_att=pa, seed=seed, packed=packed,
                               return_stats=True, bag_ids=ids)
    C = model.num_classes
    Am = ops.split_bags(out["A_mean"], sizes, C)
    Av = ops.split_bags(out["A_var"], sizes, C)
    res = []
    for b, n in enumerate(sizes):
        Y = out["Y"][b]                                   # [T, C]
        r = {"Y": Y}
        r.update(uncertainty_summary(Y, out["P_mean"][b]))
        r.update({"A_mean": Am[b].view(C, n), "A_var": Av[b].view(C, n)})
        res.append(r)
    return res


def _stage(events, name, stream):
    if events is not None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream)
        events.append((name, ev))


@torch.no_grad()
def mc_predict_image(model, patcher, image: torch.Tensor, T: int = 100, seed: Optional[int] = None,
                     features_dtype: Optional[torch.dtype] = torch.bfloat16,
                     normalize=(IMAGENET_MEAN, IMAGENET_STD), events: Optional[list] = None) -> dict:
    """One image [c, H, W] on a HIP device (get_tiles(H, W) done) -> dict with the bag's tile
    ids, its features [k, L], Y [T, C], A [T, C, k], probs [T, C], prob_mean [C],
    per-instance A_mean/A_var [C, k], and the
    attention maps' mean/std over passes att_mean/att_std [C, H, W] (infer.py:212-219).

    features_dtype=bfloat16 runs the ResNet under autocast (bf16 convolutions, fp32 BN) on
    bf16 instances; None keeps the reference's fp32. `events` (a list) collects per-stage HIP
    events for timing."""
    device = model._check_device(image.device)
    stream = torch.cuda.current_stream(device)
    if seed is None:
        seed = int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())
    _stage(events, "start", stream)
    inst_dtype = torch.float32 if features_dtype is None else features_dtype
    inst, ids, _ = patcher.convert_img_to_bag(image, seed=seed, out_dtype=inst_dtype,
                                              normalize=normalize)
    _stage(events, "patcher", stream)
    ctx = torch.autocast("cuda", dtype=features_dtype) if features_dtype is not None \
        else contextlib.nullcontext()
    with ctx:
        H = model.extract_features(inst[None])      # NCHW: the stem kernel reads it as written
    _stage(events, "features", stream)
    Y, A, st = model.mc_inference_features(H[0], T=T, seed=seed, return_stats=True)
    _stage(events, "mcdo_head", stream)
    probs = torch.softmax(Y[:, 0], dim=-1)                      # infer.py:195
    att_mean, att_std = patcher.attention_statistics(A, patcher.last_tile_ids, image.shape)
    _stage(events, "attention_maps", stream)
    return {"tiles_indices": ids, "features": H[0], "Y": Y[:, 0], "A": A[:, 0], "probs": probs,
            "prob_mean": st["P_mean"][0], "A_mean": st["A_mean"][0], "A_var": st["A_var"][0],
            "att_mean": att_mean, "att_std": att_std}
