"""TEST INFRASTRUCTURE -- CPU restatement of the reference ImagePatcher (image_patcher.py) and of
the attention statistics infer.py derives from its maps.

Only tests/ and bench.py's cpu_baseline leg may import this, as the checker.

  start_points      image_patcher.py:16-28
  tile_grid         image_patcher.py:30-41   (y, x, ps, ps, i, j) rows
  nonzero_percent   image_patcher.py:51-53   % of pixels > 0 in channel 0, fp32
  select            image_patcher.py:55-59, 115-131: tiles above the threshold, highest first.
                    The reference orders ties with numpy's (unstable) quicksort and then
                    shuffles with sklearn/numpy's global RNG; this restatement uses a stable
                    order (percentage descending, tile index ascending) and no shuffle. The
                    SET of selected tiles is identical; the order differs only among ties, and
                    the MIL head is permutation-equivariant (tests/test_oracle_golden.py).
  reconstruct_image image_patcher.py:62-80   (overlap-averaged patches, float counts)
  attention_maps    image_patcher.py:83-110  (overlap-averaged, per-(pass, class) max-normalised)
  map_stats         infer.py:212-219          mean / unbiased std over passes
Pinned by tests/golden/patcher_*.npz (tests/golden/make_golden_patcher.py runs the reference).
"""
import numpy as np
import torch


def start_points(size, split_size, overlap):
    points = [0]
    stride = int(split_size * (1 - overlap))
    counter = 1
    while True:
        pt = stride * counter
        if pt + split_size >= size:
            points.append(size - split_size)
            break
        points.append(pt)
        counter += 1
    return points


def tile_grid(h, w, ps, overlap):
    xs = start_points(w, ps, overlap)
    ys = start_points(h, ps, overlap)
    tiles = np.zeros((len(ys) * len(xs), 6), dtype=np.int64)
    k = 0
    for i, y in enumerate(ys):
        for j, x in enumerate(xs):
            tiles[k] = (y, x, ps, ps, i, j)
            k += 1
    return tiles


def nonzero_percent(image, tiles):
    image = torch.as_tensor(image)
    out = torch.zeros(len(tiles), dtype=torch.float32)
    for i, (y, x, dh, dw, _, _) in enumerate(tiles):
        out[i] = (image[0, y:y + dh, x:x + dw] > 0).float().mean() * 100
    return out


def select(px, empty_thresh, bag_size=-1):
    px = torch.as_tensor(px)
    order = sorted(range(len(px)), key=lambda i: (-float(px[i]), i))
    k = int((px > empty_thresh * 100).sum())
    if bag_size > 0:
        k = min(k, bag_size)
    elif bag_size != -1:
        raise ValueError("Invalid bag size")
    return np.array(order[:k], dtype=np.int64)


def crops(image, tiles, ids):
    image = torch.as_tensor(image)
    return torch.stack([image[:, y:y + dh, x:x + dw] for (y, x, dh, dw, _, _) in tiles[ids]]) \
        if len(ids) else torch.zeros(0, image.shape[0], tiles[0][2], tiles[0][3])


def reconstruct_image(patches, tiles, ids, image_shape):
    patches = torch.as_tensor(patches)
    c, h, w = image_shape
    rec = torch.zeros(c, h, w, dtype=patches.dtype)
    cnt = torch.zeros(c, h, w, dtype=torch.float32)
    for item in range(len(ids)):
        y, x, dh, dw, _, _ = tiles[ids[item]]
        rec[:, y:y + dh, x:x + dw] += patches[item]
        cnt[:, y:y + dh, x:x + dw] += 1
    cnt = torch.where(cnt == 0, torch.ones_like(cnt), cnt)
    return rec / cnt


def attention_maps(A, tiles, ids, image_shape):
    """A: [T, 1, C, k] -> [T, C, c, H, W] exactly as image_patcher.py:83-110 computes it."""
    A = torch.as_tensor(A)
    T, _, C, k = A.shape
    c, h, w = image_shape
    rec = torch.zeros((T, C, c, h, w), dtype=A.dtype)
    cnt = torch.zeros((T, C, c, h, w), dtype=torch.uint8)
    for item in range(k):
        y, x, dh, dw, _, _ = tiles[ids[item]]
        rec[:, :, :, y:y + dh, x:x + dw] += A[:, :, :, item].view(T, C, 1, 1, 1).expand(T, C, c, dh, dw)
        cnt[:, :, :, y:y + dh, x:x + dw] += 1
    cnt = torch.where(cnt == 0, torch.ones_like(cnt), cnt)
    rec /= cnt
    mx = rec.max(dim=-1)[0].max(dim=-1)[0].max(dim=-1)[0]
    return rec / mx.view(T, C, 1, 1, 1)


def map_stats(maps):
    """infer.py:212-219: per class, mean and (unbiased) std over the passes -> [C, H, W] each."""
    return maps[:, :, 0].mean(dim=0), maps[:, :, 0].std(dim=0)
