"""ImagePatcher on the GPU: drop-in for the reference's image_patcher.ImagePatcher
(image_patcher.py:7-131) over the C ABI in include/mcgmil_image.h.

Same constructor, attributes and methods. Images and results live on the HIP device.

  get_tiles(h, w)                       image_patcher.py:30-41   host C, same int64 [n, 6] array
  convert_img_to_bag(image)             image_patcher.py:43-59, 115-131
  reconstruct_image_from_patches(...)   image_patcher.py:62-80
  reconstruct_attention_map(...)        image_patcher.py:83-110
  attention_statistics(...)             infer.py:212-219 fused: mean/std over passes without
                                        materialising the [T, C, c, H, W] maps

Deliberate differences, all documented in include/mcgmil_image.h:
  * tiles with equal non-zero percentage are ranked by tile index, not by numpy's quicksort;
  * the bag shuffle is a Philox permutation of `seed` instead of sklearn.utils.shuffle. With
    seed=None the seed is drawn from numpy's global RNG, which is where sklearn draws from, so
    np.random.seed(...) still makes a run reproducible.
The selected SET of tiles equals the reference's. The MIL head is permutation-equivariant.
"""
import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .ops import _p, _stream

_IMAGE_DTYPES = {torch.float32: _lib.MCGMIL_F32, torch.bfloat16: _lib.MCGMIL_BF16,
                 torch.uint8: _lib.MCGMIL_U8, torch.uint16: _lib.MCGMIL_U16}
_OUT_DTYPES = {torch.float32: _lib.MCGMIL_F32, torch.bfloat16: _lib.MCGMIL_BF16}


def _workspace(L, a, device):
    n = ctypes.c_size_t()
    _lib.check(L.mcgmil_image_workspace_size(ctypes.byref(a), ctypes.byref(n)),
               "mcgmil_image_workspace_size")
    ws = torch.empty(max(n.value, 1), dtype=torch.uint8, device=device)
    a.workspace, a.workspace_bytes = _p(ws), n.value
    return ws


def _ids_tensor(instances_ids, device) -> torch.Tensor:
    if isinstance(instances_ids, torch.Tensor):
        return instances_ids.to(device=device, dtype=torch.int32).contiguous()
    return torch.as_tensor(np.asarray(instances_ids, dtype=np.int32), device=device)


class ImagePatcher:
    """image_patcher.py:7-14. `self.tiles` is set by get_tiles, which the reference also needs
    before convert_img_to_bag / the reconstruct methods."""

    def __init__(self, patch_size=224, overlap=0.5, bag_size=-1, empty_thresh=0.8):
        self.patch_size = patch_size
        self.overlap = overlap
        self.bag_size = bag_size
        self.empty_thresh = empty_thresh
        self.tiles = None
        self._hw = None
        self.last_px: Optional[torch.Tensor] = None
        self.last_tile_ids: Optional[torch.Tensor] = None

    # -- geometry ------------------------------------------------------------------------
    def _args(self, h: int, w: int, channels: int = 1) -> _lib.ImageArgs:
        a = _lib.ImageArgs()
        a.height, a.width, a.channels = int(h), int(w), int(channels)
        a.patch_size, a.overlap = int(self.patch_size), float(self.overlap)
        a.empty_thresh, a.bag_size = float(self.empty_thresh), int(self.bag_size)
        return a

    def get_tiles(self, h: int, w: int) -> np.ndarray:
        L = _lib.load()
        a = self._args(h, w)
        n = ctypes.c_int32()
        _lib.check(L.mcgmil_tile_grid(ctypes.byref(a), None, ctypes.byref(n), None, None),
                   "mcgmil_tile_grid")
        tiles = np.zeros((n.value, 6), dtype=np.int64)
        _lib.check(L.mcgmil_tile_grid(ctypes.byref(a), tiles.ctypes.data_as(ctypes.c_void_p),
                                      ctypes.byref(n), None, None), "mcgmil_tile_grid")
        self.tiles = tiles
        self._hw = (int(h), int(w))
        return tiles

    def _require_tiles(self, h: int, w: int):
        if self.tiles is None:
            raise RuntimeError("call get_tiles(h, w) first (as with the reference ImagePatcher)")
        if self._hw != (int(h), int(w)):
            raise ValueError(f"tiles were built for {self._hw}, image is {(h, w)}")

    # -- image -> bag --------------------------------------------------------------------
    def convert_img_to_bag(self, image: torch.Tensor, seed: Optional[int] = None,
                           shuffle: bool = True, out_dtype: torch.dtype = torch.float32,
                           normalize: Optional[Tuple[Sequence[float], Sequence[float]]] = None):
        """image [c, H, W] on the HIP device -> (instances [k, c, ps, ps], instances_idx int64
        [k], instances_cords int64 [k, 2]) like image_patcher.py:43-59. One host sync reads k.

        normalize=(mean, std) fuses the dataset's per-instance T.Normalize (reference
        utils.py:50-51, applied in dataset.py:70-71) into the gather: (x - mean) / std in fp32,
        bit-identical to torchvision's sub_/div_."""
        if not isinstance(image, torch.Tensor) or not image.is_cuda or image.dim() != 3:
            raise ValueError("image must be a [c, H, W] HIP tensor")
        if image.dtype not in _IMAGE_DTYPES:
            raise ValueError(f"image dtype {image.dtype} not supported")
        if out_dtype not in _OUT_DTYPES:
            raise ValueError("out_dtype must be float32 or bfloat16")
        c, h, w = image.shape
        self._require_tiles(h, w)
        if image.stride(2) != 1:
            image = image.contiguous()
        L = _lib.load()
        dev = image.device
        a = self._args(h, w, c)
        nt = len(self.tiles)
        cap = nt if self.bag_size <= 0 else min(nt, int(self.bag_size))
        if seed is None and shuffle:
            seed = int(np.random.randint(0, np.iinfo(np.int64).max, dtype=np.int64))
        a.shuffle, a.shuffle_seed = int(bool(shuffle)), int(seed or 0) & (2 ** 64 - 1)
        a.image_dtype, a.out_dtype = _IMAGE_DTYPES[image.dtype], _OUT_DTYPES[out_dtype]
        a.image, a.ld_row, a.ld_channel = _p(image), image.stride(1), image.stride(0)
        if normalize is not None:
            mean, std = (np.asarray(v, dtype=np.float32).reshape(-1) for v in normalize)
            if len(mean) != c or len(std) != c:
                raise ValueError(f"normalize needs {c} means and stds")
            a.normalize = 1
            for i in range(c):
                a.norm_mean[i], a.norm_std[i] = float(mean[i]), float(std[i])
        px = torch.empty(nt, dtype=torch.float32, device=dev)
        # k and the bag's tile ids in one buffer, so one copy (one host sync) brings both back
        sel = torch.empty(nt + 1, dtype=torch.int32, device=dev)
        count, ids = sel[:1], sel[1:]
        inst = torch.empty(cap, c, self.patch_size, self.patch_size, dtype=out_dtype, device=dev)
        a.px, a.tile_ids, a.num_selected = _p(px), _p(ids), _p(count)
        a.instances, a.instance_capacity = _p(inst), cap
        ws = _workspace(L, a, dev)  # noqa: F841  (kept alive until the launch is queued)
        _lib.check(L.mcgmil_image_to_bag(ctypes.byref(a), _stream(dev)), "mcgmil_image_to_bag")
        host = sel.cpu().numpy()
        k = int(host[0])
        self.last_px, self.last_tile_ids = px, ids[:k]
        idx = host[1:1 + k].astype(np.int64)
        return inst[:k], idx, self.tiles[idx, 4:6]

    # -- reconstruction ------------------------------------------------------------------
    def reconstruct_image_from_patches(self, patches: torch.Tensor, instances_ids,
                                       image_shape: Sequence[int]) -> torch.Tensor:
        """patches [k, c, ps, ps] -> [c, H, W] overlap average (image_patcher.py:62-80)."""
        c, h, w = (int(v) for v in image_shape)
        self._require_tiles(h, w)
        dev = patches.device
        patches = patches.to(torch.float32).contiguous()
        k = patches.shape[0]
        if patches.shape[1:] != (c, self.patch_size, self.patch_size):
            raise ValueError(f"patches must be [k, {c}, {self.patch_size}, {self.patch_size}]")
        L = _lib.load()
        a = self._args(h, w, c)
        ids = _ids_tensor(instances_ids, dev)
        if ids.numel() != k:
            raise ValueError("one tile id per patch is required")
        out = torch.empty(c, h, w, dtype=torch.float32, device=dev)
        a.k, a.patches, a.map_tile_ids, a.image_out = k, _p(patches), _p(ids), _p(out)
        ws = _workspace(L, a, dev)  # noqa: F841
        _lib.check(L.mcgmil_reconstruct_image(ctypes.byref(a), _stream(dev)),
                   "mcgmil_reconstruct_image")
        return out

    def _maps(self, attention_weights, instances_ids, image_shape, want_maps, want_stats):
        A = attention_weights
        if not isinstance(A, torch.Tensor) or not A.is_cuda or A.dim() != 4 or A.shape[1] != 1:
            raise ValueError("attention_weights must be a [T, 1, C, k] HIP tensor")
        c, h, w = (int(v) for v in image_shape)
        self._require_tiles(h, w)
        T, _, C, k = A.shape
        dev = A.device
        A = A.to(torch.float32).contiguous()
        ids = _ids_tensor(instances_ids, dev)
        if ids.numel() != k:
            raise ValueError("one tile id per instance is required")
        L = _lib.load()
        a = self._args(h, w, c)
        a.T, a.C, a.k, a.attention, a.map_tile_ids = T, C, k, _p(A), _p(ids)
        maps = stats = None
        if want_maps:
            maps = torch.empty(T, C, h, w, dtype=torch.float32, device=dev)
            a.maps = _p(maps)
        if want_stats:
            stats = torch.empty(2, C, h, w, dtype=torch.float32, device=dev)
            a.map_mean, a.map_std = _p(stats[0]), _p(stats[1])
        ws = _workspace(L, a, dev)  # noqa: F841
        _lib.check(L.mcgmil_attention_maps(ctypes.byref(a), _stream(dev)), "mcgmil_attention_maps")
        return maps, stats

    def reconstruct_attention_map(self, attention_weights: torch.Tensor, instances_ids,
                                  image_shape: Sequence[int]) -> torch.Tensor:
        """[T, 1, C, k] -> [T, C, c, H, W] (image_patcher.py:83-110). The c channels are equal
        in the reference; here they are one stride-0 view of a single [T, C, H, W] map."""
        c = int(image_shape[0])
        maps, _ = self._maps(attention_weights, instances_ids, image_shape, True, False)
        T, C, h, w = maps.shape
        return maps.unsqueeze(2).expand(T, C, c, h, w)

    def attention_statistics(self, attention_weights: torch.Tensor, instances_ids,
                             image_shape: Sequence[int]) -> Tuple[torch.Tensor, torch.Tensor]:
        """Per class mean and unbiased std over the passes of the normalised maps, [C, H, W]
        each (infer.py:212-219), fused: the T maps are never written."""
        _, stats = self._maps(attention_weights, instances_ids, image_shape, False, True)
        return stats[0], stats[1]
