"""MI355X parity of the image side (include/mcgmil_image.h through mcgmil.patcher.ImagePatcher):
tile percentages, selection, gather, attention maps and their statistics, image
reconstruction -- against the reference ImagePatcher's goldens (tests/golden/patcher_*.npz)
and the CPU restatement oracle/patcher_ref.py.

Bars: px, selection order (stable rule), instances, maps and reconstructed images are
bit-exact (integer counts, copies, and fp32 sums in the reference's order). Mean/std over
passes accumulate in fp64: abs <= 2.4e-7 (2 ulp of 1.0) on values in [0, 1]."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from golden.make_golden_patcher import synthetic_image
from oracle import patcher_ref as P

pytestmark = pytest.mark.gpu

# mean/std over passes: fp64 accumulation here, torch's float reductions in the reference --
# the results may differ in the last place; maps are <= 1, so 2 ulp of 1.0
STAT_ATOL = 2.4e-7

CASES = [11, 12, 13]


def _case(seed):
    z = np.load(os.path.join(GOLDEN, f"patcher_case{seed}.npz"))
    return {k: z[k] for k in z.files}


def _patcher(z, bag=None):
    from mcgmil.patcher import ImagePatcher
    p = ImagePatcher(patch_size=int(z["ps"]), overlap=float(z["overlap"]),
                     bag_size=int(z["bag_size"]) if bag is None else bag,
                     empty_thresh=float(z["thresh"]))
    p.get_tiles(int(z["h"]), int(z["w"]))
    return p


@pytest.mark.parametrize("seed", CASES)
def test_image_to_bag_matches_reference(cuda, seed):
    z = _case(seed)
    img = synthetic_image(int(z["seed"]), int(z["h"]), int(z["w"]), int(z["c"]))
    p = _patcher(z)
    inst, idx, cords = p.convert_img_to_bag(torch.from_numpy(img).to(cuda), shuffle=False)
    torch.cuda.synchronize()
    assert np.array_equal(p.last_px.cpu().numpy(), z["px"])                # bit-exact
    want = P.select(z["px"], float(z["thresh"]), int(z["bag_size"]))
    assert np.array_equal(idx, want)                                        # stable rule
    if int(z["bag_size"]) == -1:
        assert set(idx.tolist()) == set(z["ids"].tolist())                  # reference's set
    assert np.array_equal(np.sort(z["px"][idx]), np.sort(z["px"][z["ids"]]))
    assert torch.equal(inst.cpu(), P.crops(img, z["tiles"], idx))
    assert np.array_equal(cords, z["tiles"][idx, 4:6])


def test_shuffle_is_a_seeded_permutation(cuda):
    z = _case(12)
    img = torch.from_numpy(synthetic_image(12, int(z["h"]), int(z["w"]), int(z["c"]))).to(cuda)
    p = _patcher(z)
    base, ib, _ = p.convert_img_to_bag(img, shuffle=False)
    a, ia, _ = p.convert_img_to_bag(img, seed=5)
    b, ibb, _ = p.convert_img_to_bag(img, seed=5)
    c, ic, _ = p.convert_img_to_bag(img, seed=6)
    assert sorted(ia.tolist()) == sorted(ib.tolist()) and not np.array_equal(ia, ib)
    assert np.array_equal(ia, ibb) and torch.equal(a, b)
    assert not np.array_equal(ia, ic)
    pos = {t: n for n, t in enumerate(ib.tolist())}
    assert torch.equal(a, base[[pos[t] for t in ia.tolist()]])   # instance n is tile ia[n]
    np.random.seed(3)
    _, i1, _ = p.convert_img_to_bag(img)
    np.random.seed(3)
    _, i2, _ = p.convert_img_to_bag(img)
    assert np.array_equal(i1, i2)                                 # seed=None uses numpy's RNG


@pytest.mark.parametrize("dtype", [torch.uint8, torch.uint16, torch.bfloat16])
def test_image_dtypes(cuda, dtype):
    z = _case(11)
    img = synthetic_image(11, int(z["h"]), int(z["w"]), 2)
    if dtype == torch.bfloat16:
        src = torch.from_numpy(img).to(dtype)
    else:
        src = torch.from_numpy((img * 200).astype(np.int32)).to(dtype)
    ref = src.float()
    p = _patcher(z)
    inst, idx, _ = p.convert_img_to_bag(src.to(cuda), shuffle=False)
    px = P.nonzero_percent(ref, z["tiles"])
    assert torch.equal(p.last_px.cpu(), px)
    assert np.array_equal(idx, P.select(px, float(z["thresh"]), -1))
    assert torch.equal(inst.cpu(), P.crops(ref, z["tiles"], idx))


def test_bf16_instances_and_strided_image(cuda):
    z = _case(12)
    img = torch.from_numpy(synthetic_image(12, int(z["h"]), int(z["w"]), 3))
    big = torch.zeros(4, int(z["h"]), int(z["w"]) + 13)
    big[:3, :, 5:5 + int(z["w"])] = img
    view = big.to(cuda)[:3, :, 5:5 + int(z["w"])]                 # ld_row = W + 13
    p = _patcher(z)
    inst, idx, _ = p.convert_img_to_bag(view, shuffle=False, out_dtype=torch.bfloat16)
    assert inst.dtype == torch.bfloat16
    assert torch.equal(inst.cpu(), P.crops(img, z["tiles"], idx).to(torch.bfloat16))


@pytest.mark.parametrize("seed,out", [(11, torch.float32), (12, torch.bfloat16)])
def test_fused_normalize(cuda, seed, out):
    """dataset.py:70-71 applies T.Normalize(ImageNet mean/std) (utils.py:50-51) per instance;
    torchvision computes tensor.sub_(mean).div_(std) with fp32 mean/std."""
    z = _case(seed)
    img = torch.from_numpy(synthetic_image(seed, int(z["h"]), int(z["w"]), 1)).repeat(3, 1, 1)
    mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    p = _patcher(z)
    inst, idx, _ = p.convert_img_to_bag(img.to(cuda), shuffle=False, out_dtype=out,
                                        normalize=(mean, std))
    crops = P.crops(img, z["tiles"], idx)
    m = torch.tensor(mean, dtype=torch.float32)[:, None, None]
    s = torch.tensor(std, dtype=torch.float32)[:, None, None]
    want = torch.stack([x.sub(m).div(s) for x in crops]).to(out)
    assert torch.equal(inst.cpu(), want)


@pytest.mark.parametrize("src_dtype,out", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                           (torch.uint8, torch.bfloat16), (torch.bfloat16, torch.float32)])
def test_gather_wide_path(cuda, src_dtype, out):
    """8-aligned geometry (W - ps and the stride multiples of 8): the 8-wide gather path."""
    from mcgmil.patcher import ImagePatcher
    h, w = 600, 456
    img = synthetic_image(21, h, w, 3)
    src = torch.from_numpy(img) if src_dtype != torch.uint8 else torch.from_numpy((img * 200).astype(np.uint8))
    src = src.to(src_dtype)
    ref = src.float()
    p = ImagePatcher(patch_size=64, overlap=0.5, empty_thresh=0.3)
    tiles = p.get_tiles(h, w)
    mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    inst, idx, _ = p.convert_img_to_bag(src.to(cuda), shuffle=False, out_dtype=out, normalize=(mean, std))
    m = torch.tensor(mean)[:, None, None]
    sd = torch.tensor(std)[:, None, None]
    want = torch.stack([x.sub(m).div(sd) for x in P.crops(ref, tiles, idx)]).to(out)
    assert len(idx) > 10 and torch.equal(inst.cpu(), want)


def test_empty_and_capped_bags(cuda):
    from mcgmil.patcher import ImagePatcher
    p = ImagePatcher(patch_size=32, overlap=0.5, bag_size=-1, empty_thresh=0.5)
    p.get_tiles(100, 90)
    inst, idx, cords = p.convert_img_to_bag(torch.zeros(1, 100, 90, device=cuda))
    assert inst.shape == (0, 1, 32, 32) and idx.shape == (0,) and cords.shape == (0, 2)
    p = ImagePatcher(patch_size=32, overlap=0.5, bag_size=7, empty_thresh=0.5)
    p.get_tiles(100, 90)
    inst, idx, _ = p.convert_img_to_bag(torch.ones(1, 100, 90, device=cuda), shuffle=False)
    assert inst.shape[0] == 7 and idx.tolist() == list(range(7))   # all 100%: index order


@pytest.mark.parametrize("shuffle", [False, True])
def test_capped_bag_instances_in_bag_order(cuda, shuffle):
    """A capped bag (bag_size < the tiles above the threshold), shuffled or not, at the 8-wide and
    scalar gathers: instance n holds the crop of tile idx[n]. The gather walks the tiles in tile
    order and writes each selected tile to its bag position (gather_tiles_kernel)."""
    from mcgmil.patcher import ImagePatcher
    for h, w, ps, ov in ((300, 248, 32, 0.75), (150, 137, 20, 0.5)):
        img = synthetic_image(21, h, w, 3)
        p = ImagePatcher(patch_size=ps, overlap=ov, bag_size=9, empty_thresh=0.2)
        tiles = p.get_tiles(h, w)
        inst, idx, _ = p.convert_img_to_bag(torch.from_numpy(img).to(cuda), shuffle=shuffle, seed=3)
        px = P.nonzero_percent(img, tiles)
        assert len(idx) == 9 and sorted(idx.tolist()) == sorted(P.select(px, 0.2, 9).tolist())
        assert torch.equal(inst.cpu(), P.crops(img, tiles, idx))


def test_patch_size_equal_to_image(cuda):
    """ps == H == W gives the reference's duplicated tile (start points [0, 0])."""
    from mcgmil.patcher import ImagePatcher
    p = ImagePatcher(patch_size=64, overlap=0.5, empty_thresh=0.1)
    tiles = p.get_tiles(64, 64)
    assert len(tiles) == 4
    img = torch.rand(1, 64, 64)
    inst, idx, _ = p.convert_img_to_bag(img.to(cuda), shuffle=False)
    assert idx.tolist() == [0, 1, 2, 3] and torch.equal(inst.cpu(), img.expand(4, 1, 64, 64))
    A = torch.full((2, 1, 1, 4), 0.25, device=cuda)
    maps = p.reconstruct_attention_map(A, idx, (1, 64, 64))
    assert torch.equal(maps.cpu(), P.attention_maps(A.cpu(), tiles, idx, (1, 64, 64)))


@pytest.mark.parametrize("seed", CASES)
def test_attention_maps_match_reference(cuda, seed):
    z = _case(seed)
    p = _patcher(z)
    A = torch.from_numpy(z["A"]).to(cuda)
    shape = (int(z["c"]), int(z["h"]), int(z["w"]))
    maps = p.reconstruct_attention_map(A, z["ids"], shape)
    assert maps.shape == (int(z["T"]), int(z["C"])) + shape
    got = maps.cpu()
    assert torch.equal(got[0, :, 0], torch.from_numpy(z["map_t0"]))         # bit-exact
    assert torch.equal(got[-1, :, 0], torch.from_numpy(z["map_tl"]))
    assert torch.equal(got, P.attention_maps(z["A"], z["tiles"], z["ids"], shape))
    mean, std = p.attention_statistics(A, z["ids"], shape)
    np.testing.assert_allclose(mean.cpu().numpy(), z["map_mean"], rtol=0, atol=STAT_ATOL)
    np.testing.assert_allclose(std.cpu().numpy(), z["map_std"], rtol=0, atol=STAT_ATOL)


def test_attention_maps_edge_cases(cuda):
    z = _case(11)
    p = _patcher(z)
    shape = (1, int(z["h"]), int(z["w"]))
    A1 = torch.from_numpy(z["A"][:1]).to(cuda)                     # T == 1: std is NaN
    mean, std = p.attention_statistics(A1, z["ids"], shape)
    assert torch.isnan(std).all()
    assert torch.equal(mean.cpu(), P.attention_maps(z["A"][:1], z["tiles"], z["ids"], shape)[0, :, 0])
    A0 = torch.zeros(3, 1, 2, 0, device=cuda)                     # empty bag: 0 / 0
    assert torch.isnan(p.reconstruct_attention_map(A0, [], shape)).all()
    dup = np.concatenate([z["ids"][:5], z["ids"][:5]])             # repeated tiles count twice
    Ad = torch.rand(2, 1, 2, 10)
    got = p.reconstruct_attention_map(Ad.to(cuda), dup, shape).cpu()
    assert torch.equal(got, P.attention_maps(Ad, z["tiles"], dup, shape))


@pytest.mark.parametrize("seed", [11, 12])
def test_reconstruct_image(cuda, seed):
    z = _case(seed)
    c = int(z["c"])
    p = _patcher(z)
    patches = torch.rand(len(z["ids"]), c, int(z["ps"]), int(z["ps"]))
    shape = (c, int(z["h"]), int(z["w"]))
    got = p.reconstruct_image_from_patches(patches.to(cuda), z["ids"], shape).cpu()
    assert torch.equal(got, P.reconstruct_image(patches, z["tiles"], z["ids"], shape))
    img = torch.from_numpy(synthetic_image(seed, shape[1], shape[2], c))
    all_ids = np.arange(len(z["tiles"]))
    again = p.reconstruct_image_from_patches(P.crops(img, z["tiles"], all_ids).to(cuda), all_ids, shape)
    torch.testing.assert_close(again.cpu(), img, rtol=1e-6, atol=1e-6)   # round trip


def test_config5_scale(cuda):
    """7036 x 2800, ps 224, overlap 0.5 (1488 tiles), T=100, C=2.
    px against the oracle; maps for passes 0 and T-1 against the oracle (a map depends only on
    its own pass); fused mean/std against torch reductions of the GPU's own full maps."""
    from mcgmil.patcher import ImagePatcher
    h, w = 7036, 2800
    img = synthetic_image(5, h, w, 1)
    p = ImagePatcher(patch_size=224, overlap=0.5, empty_thresh=0.5)
    tiles = p.get_tiles(h, w)
    assert len(tiles) == 1488
    inst, idx, _ = p.convert_img_to_bag(torch.from_numpy(img).to(cuda), seed=1)
    px = P.nonzero_percent(img, tiles)
    assert torch.equal(p.last_px.cpu(), px)
    assert sorted(idx.tolist()) == sorted(P.select(px, 0.5, -1).tolist())
    assert torch.equal(inst[:24].cpu(), P.crops(img, tiles, idx[:24]))       # 8-wide gather
    k = len(idx)
    assert k > 100
    T, C = 100, 2
    g = torch.Generator().manual_seed(0)
    A = torch.softmax(torch.randn(T, 1, C, k, generator=g), dim=-1)
    Ad = A.to(cuda)
    maps = p.reconstruct_attention_map(Ad, idx, (1, h, w))[:, :, 0]          # [T, C, H, W]
    for t in (0, T - 1):
        ref = P.attention_maps(A[t:t + 1], tiles, idx, (1, h, w))[0, :, 0]
        assert torch.equal(maps[t].cpu(), ref)
    mean, std = p.attention_statistics(Ad, idx, (1, h, w))
    torch.testing.assert_close(mean, maps.double().mean(0).float(), rtol=0, atol=STAT_ATOL)
    torch.testing.assert_close(std, maps.double().std(0).float(), rtol=0, atol=STAT_ATOL)
