"""Host side of the image C ABI (include/mcgmil_image.h): the tile grid is host C, so it is
checked here against the reference ImagePatcher's grids (tests/golden/patcher_grid.npz); the
device entry points are checked for argument validation only (no launches without a GPU)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _patcher(ps, ov, bag=-1, thr=0.8):
    from mcgmil.patcher import ImagePatcher
    return ImagePatcher(patch_size=ps, overlap=ov, bag_size=bag, empty_thresh=thr)


def test_tile_grid_matches_reference(hip_lib):
    z = np.load(os.path.join(GOLDEN, "patcher_grid.npz"))
    for key in z.files:
        hw, ps, ov = key.split("_")
        h, w = map(int, hw.split("x"))
        got = _patcher(int(ps[2:]), float(ov[2:])).get_tiles(h, w)
        assert got.dtype == np.int64 and np.array_equal(got, z[key]), key


@pytest.mark.parametrize("h,w,ps,ov", [(100, 70, 30, 0.3), (97, 131, 16, 0.75), (64, 64, 64, 0.0),
                                       (1000, 37, 37, 0.5), (250, 250, 100, 0.9)])
def test_tile_grid_matches_oracle(hip_lib, h, w, ps, ov):
    from oracle import patcher_ref
    assert np.array_equal(_patcher(ps, ov).get_tiles(h, w), patcher_ref.tile_grid(h, w, ps, ov))


def _image_args(**kw):
    from mcgmil import _lib
    a = _lib.ImageArgs()
    a.height, a.width, a.channels, a.patch_size, a.overlap = 600, 420, 1, 64, 0.5
    a.empty_thresh, a.bag_size, a.image_dtype, a.out_dtype = 0.75, -1, _lib.MCGMIL_F32, 0
    a.image, a.tile_ids, a.num_selected = [ctypes.c_void_p(0x1000)] * 3
    a.ld_row, a.ld_channel = 420, 600 * 420
    a.workspace, a.workspace_bytes = ctypes.c_void_p(0x10000), 1 << 30
    for k, v in kw.items():
        setattr(a, k, v)
    return a


@pytest.mark.parametrize("field,value,code", [
    ("overlap", 1.0, -1), ("overlap", -0.1, -1), ("patch_size", 0, -1), ("patch_size", 700, -2),
    ("bag_size", 0, -1), ("bag_size", -2, -1), ("image_dtype", 9, -1), ("ld_row", 100, -1),
    ("channels", 0, -1), ("workspace_bytes", 16, -4), ("workspace", ctypes.c_void_p(0x10010), -3),
])
def test_image_to_bag_validation(hip_lib, field, value, code):
    a = _image_args(**{field: value})
    assert hip_lib.mcgmil_image_to_bag(ctypes.byref(a), None) == code
    assert hip_lib.mcgmil_last_error()


def test_zero_stride_is_rejected(hip_lib):
    a = _image_args(patch_size=1, overlap=0.5)            # int(1 * 0.5) == 0 would never end
    assert hip_lib.mcgmil_image_to_bag(ctypes.byref(a), None) == -1
    assert b"stride" in hip_lib.mcgmil_last_error()


def test_attention_maps_validation(hip_lib):
    a = _image_args(T=4, C=2, k=3)                        # no attention / outputs
    assert hip_lib.mcgmil_attention_maps(ctypes.byref(a), None) == -1
    a = _image_args(T=4, C=2, k=0, patch_size=400, overlap=0.99, height=1000, width=1000,
                    ld_row=1000)                          # up to 100 x 100 tiles per pixel
    a.maps = ctypes.c_void_p(0x1000)
    assert hip_lib.mcgmil_attention_maps(ctypes.byref(a), None) == -2


def test_workspace_grows_with_passes(hip_lib):
    sizes = []
    for T in (0, 1, 100):
        a = _image_args(T=T, C=2)
        n = ctypes.c_size_t()
        assert hip_lib.mcgmil_image_workspace_size(ctypes.byref(a), ctypes.byref(n)) == 0
        sizes.append(n.value)
    assert sizes[0] < sizes[1] < sizes[2]
    assert sizes[2] - sizes[1] >= 99 * 2 * 4 * 100        # T * C fp32 values per cell (>=100 cells)
