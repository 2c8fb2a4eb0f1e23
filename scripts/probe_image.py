"""Time the image-side entry points at config-5 scale (7036 x 2800, ps 224, overlap 0.5,
T=100, C=2) with HIP events; prints one JSON line per stage."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "montecarlo-gated-mil_amd"))
from mcgmil.patcher import ImagePatcher  # noqa: E402


def timed(fn, reps=20):
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
    h, w, T, C = 7036, 2800, 100, 2
    yy, xx = torch.meshgrid(torch.arange(h, device=dev), torch.arange(w, device=dev), indexing="ij")
    blob = 1 - ((yy - 0.5 * h) / (0.45 * h)) ** 2 - (xx / (0.8 * w)) ** 2
    img = torch.where(blob > 0, blob, torch.zeros_like(blob)).float()[None].expand(3, h, w).contiguous()
    p = ImagePatcher(patch_size=224, overlap=0.5, empty_thresh=0.5)
    p.get_tiles(h, w)
    inst, idx, _ = p.convert_img_to_bag(img, seed=0)
    k = len(idx)
    A = torch.softmax(torch.randn(T, 1, C, k, device=dev), dim=-1)
    res = {"k": k, "tiles": len(p.tiles)}
    res["to_bag_ms"] = timed(lambda: p.convert_img_to_bag(img, seed=0))
    res["stats_ms"] = timed(lambda: p.attention_statistics(A, idx, (1, h, w)))
    res["maps_ms"] = timed(lambda: p.reconstruct_attention_map(A, idx, (1, h, w)), reps=5)
    inst_bytes = k * 3 * 224 * 224 * 4
    res["to_bag_GBps_instances"] = (inst_bytes * 2 + h * w * 4) / res["to_bag_ms"] / 1e6
    res["maps_GBps_written"] = T * C * h * w * 4 / res["maps_ms"] / 1e6
    res["stats_GBps_written"] = 2 * C * h * w * 4 / res["stats_ms"] / 1e6
    print(json.dumps(res))


if __name__ == "__main__":
    main()
