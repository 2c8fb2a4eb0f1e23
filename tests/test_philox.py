"""Oracle mask stream: Philox4x32-10 known answers and the keep rule (CPU only)."""
import numpy as np
import pytest
import torch

from oracle import philox

# Random123 kat_vectors, philox4x32 R=10 (ctr, key, expected)
KATS = [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]


@pytest.mark.parametrize("ctr,key,want", KATS)
def test_philox_kat_c(ctr, key, want):
    assert philox.philox4x32_10(ctr, key) == want


@pytest.mark.parametrize("ctr,key,want", KATS)
def test_philox_kat_python(ctr, key, want):
    assert philox.philox4x32_10_py(ctr, key) == want


def test_c_matches_python_random_counters():
    rng = np.random.default_rng(5)
    for _ in range(200):
        ctr = [int(x) for x in rng.integers(0, 2**32, 4)]
        key = [int(x) for x in rng.integers(0, 2**32, 2)]
        assert philox.philox4x32_10(ctr, key) == philox.philox4x32_10_py(ctr, key)


def test_threshold_and_scale_follow_torch():
    assert philox.drop_threshold(0.0) == 0
    assert philox.drop_threshold(1.0) == 65536
    assert philox.drop_threshold(0.1) == 6554
    for p in (0.05, 0.1, 0.15, 0.25, 0.3, 0.5, 0.7, 0.9):
        x = torch.ones(20000)
        y = torch.nn.functional.dropout(x, p, True)
        torch_scale = float(y[y != 0][0])
        assert philox.dropout_scale(p) == torch_scale, p
    assert philox.dropout_scale(1.0) == 0.0


def test_feature_mask_definition_by_hand():
    """keep(b,t,n,l) = u16 draw (l & 7) of Philox(ctr={l>>3, n, t, b}, key=seed) >= thr."""
    seed, bag, T, N, L, p = 0x1234_5678_9ABC_DEF0, 7, 3, 5, 64, 0.3
    keep = philox.feature_keep(seed, bag, T, N, L, p)
    thr = philox.drop_threshold(p)
    key = [seed & 0xFFFFFFFF, seed >> 32]
    for t in range(T):
        for n in range(N):
            for l in range(L):
                o = philox.philox4x32_10_py([l >> 3, n, t, bag], key)
                u = (o[(l & 7) >> 1] >> (16 * (l & 1))) & 0xFFFF
                assert keep[t, n, l] == (u >= thr)


def test_attention_mask_definition_by_hand():
    seed, bag, T, C, N, p = 99, 3, 2, 2, 21, 0.4
    keep = philox.attention_keep(seed, bag, T, C, N, p)
    thr = philox.drop_threshold(p)
    for t in range(T):
        for c in range(C):
            for n in range(N):
                o = philox.philox4x32_10_py([n >> 3, c, t | 0x80000000, bag], [seed, 0])
                u = (o[(n & 7) >> 1] >> (16 * (n & 1))) & 0xFFFF
                assert keep[t, c, n] == (u >= thr)


def test_t_offset_is_a_window_of_the_same_stream():
    full = philox.feature_keep(11, 2, 6, 9, 32, 0.1)
    part = philox.feature_keep(11, 2, 2, 9, 32, 0.1, t0=3)
    assert np.array_equal(full[3:5], part)
    fa = philox.attention_keep(11, 2, 6, 2, 9, 0.1)
    pa = philox.attention_keep(11, 2, 2, 2, 9, 0.1, t0=3)
    assert np.array_equal(fa[3:5], pa)


def test_pack_unpack_roundtrip():
    bits = philox.feature_keep_bits(5, 0, 2, 7, 128, 0.5)
    assert np.array_equal(philox.pack_feature_bits(philox.unpack_feature_bits(bits, 128)), bits)


@pytest.mark.parametrize("p", [0.0, 0.1, 0.5, 0.9, 1.0])
def test_drop_rate(p):
    keep = philox.feature_keep(2024, 0, 4, 256, 512, p)
    rate = 1.0 - keep.mean()
    target = philox.drop_threshold(p) / 65536.0
    sigma = np.sqrt(max(target * (1 - target), 1e-12) / keep.size)
    assert abs(rate - target) <= 6 * sigma + 1e-12


def test_streams_are_distinct():
    a = philox.feature_keep(1, 0, 2, 64, 512, 0.5)
    b = philox.feature_keep(1, 1, 2, 64, 512, 0.5)   # other bag
    c = philox.feature_keep(2, 0, 2, 64, 512, 0.5)   # other seed
    assert 0.4 < (a != b).mean() < 0.6 and 0.4 < (a != c).mean() < 0.6
    assert 0.4 < (a[0] != a[1]).mean() < 0.6          # other sample
