"""Golden fixtures for the image patcher and the attention maps, produced by the REFERENCE
ImagePatcher (image_patcher.py) on synthetic images. Runs only where /root/reference exists.

  patcher_grid.npz   tile grids (get_tiles) for the config sizes and a sweep of shapes
  patcher_case*.npz  per synthetic image: tiles, non-zero percentages, the selected tile SET,
                     and reconstruct_attention_map + infer.py's mean/std for seeded attention

Usage: python tests/golden/make_golden_patcher.py
"""
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def synthetic_image(seed, h, w, c=1):
    """A mammogram-like image: a zero background and a smooth positive blob touching one side."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    cy, cx = rng.uniform(0.3, 0.7) * h, rng.uniform(0.0, 0.3) * w
    ry, rx = rng.uniform(0.3, 0.5) * h, rng.uniform(0.4, 0.8) * w
    blob = 1.0 - ((yy - cy) / ry) ** 2 - ((xx - cx) / rx) ** 2
    img = np.where(blob > 0, blob + 0.05 * rng.random((h, w)), 0.0).astype(np.float32)
    return np.repeat(img[None], c, axis=0)


def main():
    if not os.path.isdir(REF):
        raise SystemExit("needs the reference checkout at /root/reference")
    sys.path.insert(0, REF)
    import image_patcher as ref

    grids = {}
    shapes = [(7036, 2800, 224, 0.5), (7036, 2800, 224, 0.75), (1000, 700, 64, 0.5),
              (513, 300, 32, 0.25), (224, 224, 224, 0.5), (300, 230, 224, 0.5)]
    for h, w, ps, ov in shapes:
        p = ref.ImagePatcher(patch_size=ps, overlap=ov)
        grids[f"{h}x{w}_ps{ps}_ov{ov}"] = p.get_tiles(h, w)
    np.savez_compressed(os.path.join(OUT, "patcher_grid.npz"), **grids)

    cases = [(11, 600, 420, 64, 0.5, 0.75, -1, 1, 6, 2),
             (12, 517, 333, 48, 0.75, 0.5, -1, 3, 5, 2),
             (13, 400, 256, 32, 0.5, 0.3, 20, 1, 3, 2)]
    for seed, h, w, ps, ov, thr, bag, c, T, C in cases:
        img = torch.from_numpy(synthetic_image(seed, h, w, c))
        p = ref.ImagePatcher(patch_size=ps, overlap=ov, bag_size=bag, empty_thresh=thr)
        tiles = p.get_tiles(h, w)
        np.random.seed(seed)  # sklearn.utils.shuffle draws from numpy's global RNG
        inst, ids, cords = p.convert_img_to_bag(img)
        ids = np.asarray(ids)
        px = torch.zeros(len(tiles))
        for i, t in enumerate(tiles):
            px[i] = (img[0, t[0]:t[0] + t[2], t[1]:t[1] + t[3]] > 0).float().mean() * 100
        rng = np.random.default_rng(seed + 100)
        A = torch.from_numpy(rng.dirichlet(np.ones(len(ids)), size=(T, 1, C)).astype(np.float32))
        maps = p.reconstruct_attention_map(A, ids, [1, h, w])
        mean = torch.stack([maps[:, k].mean(dim=0).squeeze() for k in range(C)])
        std = torch.stack([maps[:, k].std(dim=0).squeeze() for k in range(C)])
        np.savez_compressed(
            os.path.join(OUT, f"patcher_case{seed}.npz"), seed=seed, h=h, w=w, c=c, ps=ps,
            overlap=ov, thresh=thr, bag_size=bag, T=T, C=C, tiles=tiles, px=px.numpy(),
            ids=ids, A=A.numpy(), inst_sum=inst.sum(dim=(1, 2, 3)).numpy(),
            map_mean=mean.numpy(), map_std=std.numpy(),
            map_t0=maps[0, :, 0].numpy(), map_tl=maps[-1, :, 0].numpy())
        print(f"case {seed}: {len(tiles)} tiles, {len(ids)} selected, maps {tuple(maps.shape)}")


if __name__ == "__main__":
    main()
