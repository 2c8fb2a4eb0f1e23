"""MI355X parity: the HIP kernels (through the C ABI) against the reference's golden outputs and
the CPU oracle. Tolerances from SURVEY.md §8(d), nrel = max|d| / max|ref|:
  fp32           : A nrel <= 1e-5, Y abs <= 1e-5, A_mean nrel <= 1e-5 (and abs <= 1e-4),
                   A_var nrel <= 1e-4, P_mean abs <= 1e-5
  bf16 kernel vs the bf16-rounded-input reference: the fp32 bounds x 10
  bf16 kernel vs the pure fp32 reference: A_mean nrel <= 5e-3, A_var nrel <= 2e-2,
                   Y abs <= 5e-3, P_mean abs <= 1e-3
Masks are bit-exact by construction (the kernel's Philox == oracle/philox_oracle.c), checked
directly in test_masks_bit_exact."""
import json
import os

import numpy as np
import pytest
import torch

from golden_util import GOLDEN, Case, names, nrel
from oracle import mcdo_ref, philox
from mcgmil import synthetic

pytestmark = pytest.mark.gpu

TOL32 = dict(A=1e-5, Y=1e-5, A_mean=1e-5, A_var=1e-4, P_mean=1e-5)
TOL_BF16_IN = {k: 10 * v for k, v in TOL32.items()}
TOL_BF16_VS_FP32 = dict(A=5e-3, Y=5e-3, A_mean=5e-3, A_var=2e-2, P_mean=1e-3)

MC_CASES = [n for n in names() if not n.startswith("forward") and not n.startswith("serial")]
FP32_CASES = [n for n in MC_CASES if "bf16in" not in n]
BF16_CASES = [n for n in MC_CASES if "bf16in" in n]


def head_on(arrays, dev):
    from mcgmil.ops import HeadTensors
    return HeadTensors(*[torch.from_numpy(np.ascontiguousarray(arrays[k])).to(dev)
                         for k in HeadTensors._fields])


def run(case, dev, dtype, replay=False, H=None, **launch):
    from mcgmil import ops
    Hn, _, arrays = case.inputs()
    Hn = Hn if H is None else H
    Ht = torch.from_numpy(Hn).to(dev).to(dtype).contiguous()
    offs = ops.bag_offsets_tensor([case.N], dev)
    kw = {}
    if replay:
        kF, kA = case.masks()
        kw["keep_feat"] = torch.from_numpy(philox.pack_feature_bits(kF).reshape(case.T * case.N, -1)).to(dev)
        kw["keep_att"] = torch.from_numpy(kA.astype(np.uint8).reshape(-1)).to(dev)
    out = ops.mcdo_forward(Ht, offs, head_on(arrays, dev), case.T, p_feat=case.p_f,
                           p_att=case.p_a, seed=case.mask_seed, bag_id_base=case.bag_ctr,
                           return_stats=True, **kw, **launch)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


def compare(case, out, tol):
    T, C, N = case.T, case.C, case.N
    Y = out["Y"][0]                                     # [T, C]
    A = out["A"].reshape(T, C, N)
    ref_Y = case.z["Y"][:, 0]
    np.testing.assert_allclose(Y, ref_Y, rtol=0, atol=tol["Y"])
    if "A" in case.z:
        assert nrel(A, case.z["A"][:, 0]) <= tol["A"]
    else:
        assert nrel(A[0], case.z["A_first"][0]) <= tol["A"]
        assert nrel(A[-1], case.z["A_last"][0]) <= tol["A"]
    Am = out["A_mean"].reshape(C, N)
    assert case.z["A_mean"].shape == (C, N)
    assert nrel(Am, case.z["A_mean"]) <= tol["A_mean"]
    assert np.max(np.abs(Am - case.z["A_mean"])) <= 1e-4            # the north-star bound
    Av = out["A_var"].reshape(C, N)
    if T > 1:
        # nrel, or an absolute floor far below any real variance (A ~ 1/N, var ~ 1e-8): the
        # reference's own fp32 var of T identical values is rounding noise (~1e-20), ours 0
        dv = np.max(np.abs(Av - case.z["A_var"]))
        assert nrel(Av, case.z["A_var"]) <= tol["A_var"] or dv <= 1e-15
        assert dv <= 1e-4
    else:
        assert np.isnan(Av).all()
    np.testing.assert_allclose(out["P_mean"][0], case.z["P_mean"], rtol=0, atol=tol["P_mean"])
    np.testing.assert_allclose(A.sum(-1), 1.0, atol=2e-5)


# ------------------------------------------------------------------ masks
def test_masks_bit_exact(cuda):
    from mcgmil import ops
    sizes = [5, 64, 0, 37, 130]
    T, L, C, seed, base = 6, 512, 2, 0xDEADBEEF12345, 40
    offs = ops.bag_offsets_tensor(sizes, cuda)
    R = sum(sizes)
    kf = ops.feature_keep(offs, R, T, L, 0.1, seed, bag_id_base=base, t_base=3).cpu().numpy()
    ka = ops.attention_keep(offs, R, T, C, 0.3, seed, bag_id_base=base, t_base=3).cpu().numpy()
    rf = ra = 0
    for b, n in enumerate(sizes):
        want_f = philox.feature_keep_bits(seed, base + b, T, n, L, 0.1, t0=3).reshape(T * n, L // 8)
        want_a = philox.attention_keep(seed, base + b, T, C, n, 0.3, t0=3).astype(np.uint8).reshape(-1)
        assert np.array_equal(kf[rf:rf + T * n], want_f), b
        assert np.array_equal(ka[ra:ra + T * C * n], want_a), b
        rf += T * n
        ra += T * C * n
    ids = torch.tensor([9, 1000, 3, 77, 5], dtype=torch.int32, device=cuda)
    kf2 = ops.feature_keep(offs, R, T, L, 0.1, seed, bag_ids=ids).cpu().numpy()
    want = philox.feature_keep_bits(seed, 77, T, 37, L, 0.1).reshape(T * 37, -1)
    o = T * (5 + 64)
    assert np.array_equal(kf2[o:o + T * 37], want)


# ------------------------------------------------------------------ golden parity
@pytest.mark.parametrize("name", FP32_CASES)
def test_fp32_replay_matches_reference(cuda, name):
    case = Case(name)
    compare(case, run(case, cuda, torch.float32, replay=True), TOL32)


@pytest.mark.parametrize("name", FP32_CASES)
def test_fp32_philox_matches_reference(cuda, name):
    case = Case(name)
    compare(case, run(case, cuda, torch.float32), TOL32)


@pytest.mark.parametrize("name", BF16_CASES)
def test_bf16_matches_bf16_input_reference(cuda, name):
    case = Case(name)
    compare(case, run(case, cuda, torch.bfloat16), TOL_BF16_IN)


def test_bf16_drift_vs_fp32_reference(cuda):
    case = Case("cfg3_N2048_T100_sep")
    compare(case, run(case, cuda, torch.bfloat16), TOL_BF16_VS_FP32)


@pytest.mark.parametrize("T", [17, 21])
def test_replay_equals_philox_with_short_tiles(cuda, T):
    """One bag of N = 2,048 at T = 17 / 21: 272 / 336 128-row tiles, so on 256 CUs the last round
    runs as 32- / 64-row short tiles (gate_pipe_kernel<..., RTV>). Replaying the kernel's own
    Philox masks (keep_feat / keep_att from feature_keep / attention_keep) gives bitwise the
    outputs of the in-kernel draws, through both the REPLAY and the Philox short-tile
    instantiations."""
    from mcgmil import ops
    N, L, C, seed, base = 2048, 512, 2, 0x5EED, 11
    sd = synthetic.head_state_dict(3, L=L, D=128, C=C, shared=False)
    head = head_on(synthetic.head_arrays(sd, C, False), cuda)
    H = torch.from_numpy(synthetic.bag_features(8, N, L)).to(cuda).bfloat16().contiguous()
    offs = ops.bag_offsets_tensor([N], cuda)
    kw = dict(p_feat=0.25, p_att=0.1, seed=seed, bag_id_base=base, return_stats=True)
    a = ops.mcdo_forward(H, offs, head, T, **kw)
    kf = ops.feature_keep(offs, N, T, L, 0.25, seed, bag_id_base=base)
    ka = ops.attention_keep(offs, N, T, C, 0.1, seed, bag_id_base=base)
    b = ops.mcdo_forward(H, offs, head, T, keep_feat=kf, keep_att=ka, **kw)
    torch.cuda.synchronize()
    for k in a:
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("name", ["small_N64_T4_sep", "edge_N37_T5_shared", "cfg2_N512_T30_sep"])
def test_bf16_replay_matches_oracle(cuda, name):
    case = Case(name)
    Hn, sd, _ = case.inputs()
    Hb = synthetic.bf16_round(Hn)
    arr = synthetic.head_arrays(synthetic.round_state_dict_bf16(sd), case.C, case.shared)
    kF, kA = case.masks()
    Y, A = mcdo_ref.mc_inference(Hb, mcdo_ref.HeadParams(arr), kF, kA, case.p_f, case.p_a)
    out = run(case, cuda, torch.bfloat16, replay=True, H=Hn)
    np.testing.assert_allclose(out["Y"][0], Y[:, 0].numpy(), atol=TOL_BF16_IN["Y"])
    assert nrel(out["A"].reshape(case.T, case.C, case.N), A[:, 0].numpy()) <= TOL_BF16_IN["A"]


# ------------------------------------------------------------------ batches
def test_varlen_batch_matches_per_bag_oracle(cuda):
    """Several bags (incl. N=1, an empty bag, odd sizes) in ONE launch == per-bag oracle."""
    from mcgmil import ops
    sizes = [64, 1, 0, 37, 300, 128]
    T, C, L, D, seed, base = 5, 2, 512, 128, 77, 11
    sd = synthetic.head_state_dict(3, L=L, D=D, C=C, shared=False)
    arrays = synthetic.head_arrays(sd, C, False)
    Hs = [synthetic.bag_features(100 + b, n, L) for b, n in enumerate(sizes)]
    H = torch.from_numpy(np.concatenate(Hs)).to(cuda)
    offs = ops.bag_offsets_tensor(sizes, cuda)
    out = ops.mcdo_forward(H, offs, head_on(arrays, cuda), T, p_feat=0.1, p_att=0.1, seed=seed,
                           bag_id_base=base, return_stats=True)
    Y = out["Y"].cpu().numpy()
    A = ops.split_bags(out["A"].cpu(), sizes, T * C)
    Am = ops.split_bags(out["A_mean"].cpu(), sizes, C)
    prm = mcdo_ref.HeadParams(arrays)
    for b, n in enumerate(sizes):
        if n == 0:
            assert np.all(Y[b] == 0)
            continue
        kF, kA = mcdo_ref.masks_for_bag(seed, base + b, T, n, L, C, 0.1, 0.1)
        Yr, Ar = mcdo_ref.mc_inference(Hs[b], prm, kF, kA, 0.1, 0.1)
        np.testing.assert_allclose(Y[b], Yr[:, 0].numpy(), atol=1e-5)
        assert nrel(A[b].numpy().reshape(T, C, n), Ar[:, 0].numpy()) <= 1e-5
        assert nrel(Am[b].numpy().reshape(C, n), Ar[:, 0].mean(0).numpy()) <= 1e-5


def test_torch_library_op_matches_ops(cuda):
    """torch.ops.mcgmil.mcdo_forward(_stats) (SURVEY §8(b) custom-op registration) runs the same
    kernels as ops.mcdo_forward: bitwise equal outputs, incl. a seed above 2^63."""
    from mcgmil import library, ops  # noqa: F401  (registers torch.ops.mcgmil.*)
    sizes = [64, 37, 300]
    T, C, L, D = 4, 2, 512, 128
    sd = synthetic.head_state_dict(5, L=L, D=D, C=C, shared=False)
    head = head_on(synthetic.head_arrays(sd, C, False), cuda)
    H = torch.from_numpy(np.concatenate([synthetic.bag_features(7 + b, n, L)
                                         for b, n in enumerate(sizes)])).to(cuda).bfloat16()
    offs = ops.bag_offsets_tensor(sizes, cuda)
    seed = (1 << 63) + 12345
    ref = ops.mcdo_forward(H, offs, head, T, p_feat=0.1, p_att=0.1, seed=seed, bag_id_base=3,
                           return_stats=True)
    signed = seed - (1 << 64)
    Y, A = torch.ops.mcgmil.mcdo_forward(H, offs, *head, T, 0.1, 0.1, signed, 3, 0)
    assert torch.equal(Y, ref["Y"]) and torch.equal(A, ref["A"])
    Y2, Am, Av, Pm = torch.ops.mcgmil.mcdo_forward_stats(H, offs, *head, T, 0.1, 0.1, signed, 3, 0)
    assert torch.equal(Y2, ref["Y"]) and torch.equal(Am, ref["A_mean"])
    assert torch.equal(Av.isnan(), ref["A_var"].isnan())
    assert torch.equal(Av.nan_to_num(), ref["A_var"].nan_to_num()) and torch.equal(Pm, ref["P_mean"])


def test_shard_with_bag_ids_is_bitwise_rank_independent(cuda):
    """A subset of the batch run with its global bag ids reproduces the full batch bit for bit
    (what makes 1/2/4/8-GPU sharding results identical)."""
    from mcgmil import ops
    sizes = [200, 50, 333, 17, 512]
    T, C, L = 8, 2, 512
    arrays = synthetic.head_arrays(synthetic.head_state_dict(4, C=C, shared=True), C, True)
    head = head_on(arrays, cuda)
    Hs = [torch.from_numpy(synthetic.bag_features(200 + b, n)).to(cuda).bfloat16() for b, n in enumerate(sizes)]
    full = ops.mcdo_forward(torch.cat(Hs), ops.bag_offsets_tensor(sizes, cuda), head, T,
                            p_feat=0.1, p_att=0.1, seed=5)
    sub = [4, 1, 3]
    ids = torch.tensor(sub, dtype=torch.int32, device=cuda)
    part = ops.mcdo_forward(torch.cat([Hs[i] for i in sub]),
                            ops.bag_offsets_tensor([sizes[i] for i in sub], cuda), head, T,
                            p_feat=0.1, p_att=0.1, seed=5, bag_ids=ids)
    assert torch.equal(part["Y"], full["Y"][sub])
    Af = ops.split_bags(full["A"], sizes, T * C)
    Ap = ops.split_bags(part["A"], [sizes[i] for i in sub], T * C)
    for j, i in enumerate(sub):
        assert torch.equal(Ap[j], Af[i])


@pytest.mark.parametrize("shared", [False, True])
def test_cfg3_full_size_properties(cuda, shared):
    """BASELINE config 3 at full size (N=2048, T=100, bf16, 4 bags): size-independent checks,
    including run-to-run bit equality (catches races and unprotected hazards in the kernels)."""
    from mcgmil import ops
    B, N, T, C = 4, 2048, 100, 2
    arrays = synthetic.head_arrays(synthetic.head_state_dict(0, C=C, shared=shared), C, shared)
    head = head_on(arrays, cuda)
    g = torch.Generator(device=cuda).manual_seed(0)
    H = torch.randn(B * N, 512, device=cuda, generator=g).abs().bfloat16()
    offs = ops.bag_offsets_tensor([N] * B, cuda)
    o1 = ops.mcdo_forward(H, offs, head, T, p_feat=0.1, p_att=0.1, seed=1, return_stats=True)
    for _ in range(3):
        o2 = ops.mcdo_forward(H, offs, head, T, p_feat=0.1, p_att=0.1, seed=1, return_stats=True)
        for k in o1:
            assert torch.equal(o1[k], o2[k]), k                  # deterministic
    A = o1["A"].view(B, T, C, N)
    assert torch.allclose(A.sum(-1), torch.ones(B, T, C, device=cuda), atol=1e-5)
    assert bool((A >= 0).all())
    assert torch.allclose(o1["A_mean"].view(B, C, N).sum(-1), torch.ones(B, C, device=cuda), atol=1e-5)
    assert torch.allclose(o1["A_mean"].view(B, C, N), A.mean(1), atol=1e-7)
    assert torch.allclose(o1["A_var"].view(B, C, N), A.var(1), rtol=1e-4, atol=1e-12)
    p = torch.softmax(o1["Y"], -1).mean(1)
    assert torch.allclose(o1["P_mean"], p, atol=1e-6)
    assert o1["Y"].std(1).min() > 0                               # samples differ
    o0 = ops.mcdo_forward(H, offs, head, T, p_feat=0.0, p_att=0.0, seed=1)
    assert torch.equal(o0["Y"], o0["Y"][:, :1].expand_as(o0["Y"]))  # p=0: all samples equal
    o3 = ops.mcdo_forward(H, offs, head, T, p_feat=0.1, p_att=0.1, seed=2)
    assert not torch.equal(o3["Y"], o1["Y"])                       # seed changes the draw


# ------------------------------------------------------------------ drop-in module
def _flatten_extractor():
    class Flat(torch.nn.Module):
        def forward(self, x):
            return torch.flatten(x, 1)
    return Flat()


def _module(case, cuda):
    from mcgmil import MultiHeadGatedAttentionMIL
    _, sd, _ = case.inputs()
    m = MultiHeadGatedAttentionMIL(num_classes=case.C, pretrained=False, L=case.L, D=case.D,
                                   feature_dropout=case.p_f, attention_dropout=case.p_a,
                                   shared_attention=case.shared)
    own = m.state_dict()
    missing, unexpected = m.load_state_dict(
        {k: torch.from_numpy(np.asarray(v)).reshape(own[k].shape) for k, v in sd.items()},
        strict=False)
    assert not unexpected and all(k.startswith("feature_extractor") for k in missing)
    m.feature_extractor = _flatten_extractor()   # feed extracted features as [1, N, L, 1, 1]
    return m.to(cuda)


def test_module_head_keys_match_reference():
    from mcgmil import MultiHeadGatedAttentionMIL
    ref = json.load(open(os.path.join(GOLDEN, "reference_head_keys.json")))
    for shared, tag in ((True, "shared"), (False, "separate")):
        m = MultiHeadGatedAttentionMIL(pretrained=False, shared_attention=shared)
        own = {k: list(v.shape) for k, v in m.state_dict().items()
               if not k.startswith("feature_extractor")}
        assert own == ref[tag]


@pytest.mark.parametrize("name", ["cfg2_N512_T30_sep", "cfg2_N512_T30_shared", "small_N64_T1_sep"])
def test_module_mc_inference_matches_reference(cuda, name):
    case = Case(name)
    assert case.bag_ctr == 0
    m = _module(case, cuda)
    H, _, _ = case.inputs()
    x = torch.from_numpy(H).view(1, case.N, case.L, 1, 1)
    Y, A = m.mc_inference(x, N=case.T, device=cuda, seed=case.mask_seed)
    assert Y.shape == (case.T, 1, case.C) and A.shape == (case.T, 1, case.C, case.N)
    np.testing.assert_allclose(Y.cpu().numpy(), case.z["Y"], atol=1e-5)
    assert nrel(A.cpu().numpy(), case.z["A"]) <= 1e-5
    Ys, As = m.mc_inference_serial(x, N=case.T, device=cuda, seed=case.mask_seed)
    assert torch.equal(Ys, Y) and torch.equal(As, A)
    Y3, A3, losses = m.mc_inference(x, N=case.T, device=cuda, seed=case.mask_seed,
                                    return_losses=True)
    assert torch.equal(Y3, Y) and losses is None


@pytest.mark.parametrize("name", names("forward"))
def test_module_forward_eval_matches_reference(cuda, name):
    case = Case(name)
    m = _module(case, cuda).eval()
    H, _, _ = case.inputs()
    x = torch.from_numpy(H).view(1, case.N, case.L, 1, 1).to(cuda)
    Y, A, aux = m(x)
    assert aux is None and Y.shape == (1, case.C) and A.shape == (1, case.C, case.N)
    np.testing.assert_allclose(Y.cpu().numpy(), case.z["Y"], atol=1e-5)
    assert nrel(A.cpu().numpy(), case.z["A"]) <= 1e-5


def test_module_p0_mc_inference_equals_forward(cuda):
    case = Case("forward_N64_sep")
    m = _module(case, cuda)
    m.feature_dropout.p = 0.0
    for d in m.attention_dropouts:
        d.p = 0.0
    H, _, _ = case.inputs()
    x = torch.from_numpy(H).view(1, case.N, case.L, 1, 1).to(cuda)
    Y, A = m.mc_inference(x, N=3, device=cuda, seed=1)
    Yf, Af, _ = m.eval()(x)
    for t in range(3):
        assert torch.equal(Y[t], Yf) and torch.equal(A[t], Af)


def test_module_rejects_cpu_and_training(cuda):
    from mcgmil import MultiHeadGatedAttentionMIL
    m = MultiHeadGatedAttentionMIL(pretrained=False)
    with pytest.raises(RuntimeError):
        m.mc_inference(torch.zeros(1, 2, 3, 32, 32), N=2, device="cpu")
    m.train()
    with pytest.raises(NotImplementedError):
        m(torch.zeros(1, 2, 3, 32, 32))


def test_unsupported_config_raises(cuda):
    from mcgmil import ops, _lib
    C = 5
    arrays = synthetic.head_arrays(synthetic.head_state_dict(0, C=C, shared=True), C, True)
    H = torch.zeros(8, 512, device=cuda)
    with pytest.raises(_lib.MCGMILError):
        ops.mcdo_forward(H, ops.bag_offsets_tensor([8], cuda), head_on(arrays, cuda), 2,
                         p_feat=0.1, p_att=0.1, seed=0)


# ------------------------------------------------------------------ other head shapes
# (L, D, C, shared): which kernel instantiation each exercises
SHAPES = [
    (512, 128, 4, False),   # P = 32 gate tile pairs -> generic whole-tile kernel, 4 classes
    (96, 32, 2, True),      # L % 64 != 0 -> generic kernel
    (256, 48, 3, False),    # P = 9 -> pipelined, 2 pairs/wave spanning gates (per-class partials)
    (1024, 64, 1, True),    # P = 4 -> pipelined, 1 pair/wave, idle waves
    (512, 64, 3, False),    # P = 12 -> pipelined, one class per wave
    (512, 64, 4, False),    # G*D = 256 -> 32x32x16 kernel (bf16), 4 classes, one per 2 waves
    (256, 256, 2, True),    # G*D = 256 -> 32x32x16 kernel (bf16), shared gate, both classes
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("L,D,C,shared", SHAPES)
def test_head_shapes_match_oracle(cuda, L, D, C, shared, dtype):
    from mcgmil import ops
    sizes = [77, 130, 3]
    T, seed, base = 4, 9, 5
    sd = synthetic.head_state_dict(L + D + C, L=L, D=D, C=C, shared=shared)
    Hs = [synthetic.bag_features(300 + b, n, L) for b, n in enumerate(sizes)]
    if dtype == torch.bfloat16:
        sd_ref = synthetic.round_state_dict_bf16(sd)
        Hs_ref = [synthetic.bf16_round(h) for h in Hs]
        tol = TOL_BF16_IN
    else:
        sd_ref, Hs_ref, tol = sd, Hs, TOL32
    arrays = synthetic.head_arrays(sd, C, shared)
    prm = mcdo_ref.HeadParams(synthetic.head_arrays(sd_ref, C, shared))
    H = torch.from_numpy(np.concatenate(Hs)).to(cuda).to(dtype).contiguous()
    out = ops.mcdo_forward(H, ops.bag_offsets_tensor(sizes, cuda), head_on(arrays, cuda), T,
                           p_feat=0.2, p_att=0.1, seed=seed, bag_id_base=base, return_stats=True)
    Y = out["Y"].cpu().numpy()
    A = ops.split_bags(out["A"].cpu(), sizes, T * C)
    for b, n in enumerate(sizes):
        kF, kA = mcdo_ref.masks_for_bag(seed, base + b, T, n, L, C, 0.2, 0.1)
        Yr, Ar = mcdo_ref.mc_inference(Hs_ref[b], prm, kF, kA, 0.2, 0.1)
        np.testing.assert_allclose(Y[b], Yr[:, 0].numpy(), atol=tol["Y"])
        assert nrel(A[b].numpy().reshape(T, C, n), Ar[:, 0].numpy()) <= tol["A"]


# ------------------------------------------------------------------ caller statistics (a11)
@pytest.mark.parametrize("name", ["cfg2_N512_T30_sep", "cfg2_N512_T30_shared"])
def test_mc_predict_bags_caller_stats(cuda, name):
    """mcgmil.infer.mc_predict_bags (the infer.py / net_utils.mc_test counterpart) against the
    numpy restatement of infer.py:47-57 / net_utils.py:205-210 on the reference's own outputs."""
    from mcgmil import infer
    from oracle import caller_stats
    case = Case(name)
    m = _module(case, cuda)
    H, _, _ = case.inputs()
    res = infer.mc_predict_bags(m, [torch.from_numpy(H).to(cuda)], T=case.T, seed=case.mask_seed,
                                bag_ids=[case.bag_ctr])[0]
    want = caller_stats.caller_stats(case.z["Y"][:, 0], case.z["A"][:, 0])
    np.testing.assert_allclose(res["Y"].cpu().numpy(), case.z["Y"][:, 0], atol=TOL32["Y"])
    np.testing.assert_allclose(res["probs"].cpu().numpy(), want["probs"], atol=1e-5)
    np.testing.assert_allclose(res["prob_mean"].cpu().numpy(), want["prob_mean"], atol=TOL32["P_mean"])
    assert res["prediction"] == want["prediction"]
    for k in ("pos_mean", "pos_median", "pos_std", "pos_iqr", "pos_min", "pos_max", "mean_entropy"):
        assert abs(res[k] - want[k]) <= 1e-5, (k, res[k], want[k])
    assert nrel(res["A_mean"].cpu().numpy(), want["A_mean"]) <= TOL32["A_mean"]
    assert nrel(res["A_var"].cpu().numpy(), want["A_var"]) <= TOL32["A_var"]


# ------------------------------------------------------------------ BASELINE config 4 workload
def test_cfg4_ragged_batch(cuda):
    """Config 4's workload on one GPU: 64 bags with N_b drawn as BASELINE config 4 draws them
    (rng(0).integers(256, 2049)), T=100, bf16, ONE varlen launch with global bag ids (the ids a
    rank of the 8-GPU run would pass). The smallest, the largest and two other bags are checked
    against the oracle (bf16-rounded inputs, masks from the C Philox), every bag through the
    size-independent properties, and the launch is bitwise repeatable."""
    from mcgmil import ops
    sizes = np.random.default_rng(0).integers(256, 2049, 4096)[:64].tolist()
    ids = list(range(1000, 1064))
    T, C, L, D, seed = 100, 2, 512, 128, 42
    sd = synthetic.head_state_dict(0, L=L, D=D, C=C, shared=False)
    arrays = synthetic.head_arrays(sd, C, False)
    prm = mcdo_ref.HeadParams(synthetic.head_arrays(synthetic.round_state_dict_bf16(sd), C, False))
    Hs = [synthetic.bf16_round(synthetic.bag_features(2000 + b, n, L)) for b, n in enumerate(sizes)]
    H = torch.from_numpy(np.concatenate(Hs)).to(cuda).bfloat16()
    offs = ops.bag_offsets_tensor(sizes, cuda)
    bid = torch.tensor(ids, dtype=torch.int32, device=cuda)
    out = ops.mcdo_forward(H, offs, head_on(arrays, cuda), T, p_feat=0.1, p_att=0.1, seed=seed,
                           bag_ids=bid, return_stats=True)
    again = ops.mcdo_forward(H, offs, head_on(arrays, cuda), T, p_feat=0.1, p_att=0.1, seed=seed,
                             bag_ids=bid, return_stats=True)
    for k in out:
        assert torch.equal(out[k], again[k]), k
    Y = out["Y"].cpu().numpy()
    A = ops.split_bags(out["A"].cpu(), sizes, T * C)
    Am = ops.split_bags(out["A_mean"].cpu(), sizes, C)
    Av = ops.split_bags(out["A_var"].cpu(), sizes, C)
    for b, n in enumerate(sizes):                         # properties, every bag
        Ab = A[b].view(T, C, n)
        assert torch.allclose(Ab.sum(-1), torch.ones(T, C), atol=1e-5)
        assert torch.allclose(Am[b].view(C, n), Ab.mean(0), atol=1e-7)
        assert torch.allclose(Av[b].view(C, n), Ab.var(0), rtol=1e-4, atol=1e-12)
    P = torch.softmax(out["Y"], -1).mean(1)
    assert torch.allclose(out["P_mean"], P, atol=1e-6)
    check = sorted({int(np.argmin(sizes)), int(np.argmax(sizes)), 7, 40})
    for b in check:                                        # against the oracle
        n = sizes[b]
        kF, kA = mcdo_ref.masks_for_bag(seed, ids[b], T, n, L, C, 0.1, 0.1)
        Yr, Ar = mcdo_ref.mc_inference(Hs[b], prm, kF, kA, 0.1, 0.1)
        np.testing.assert_allclose(Y[b], Yr[:, 0].numpy(), atol=TOL_BF16_IN["Y"])
        assert nrel(A[b].numpy().reshape(T, C, n), Ar[:, 0].numpy()) <= TOL_BF16_IN["A"]
        assert nrel(Am[b].numpy().reshape(C, n), Ar[:, 0].mean(0).numpy()) <= TOL_BF16_IN["A_mean"]


def test_cfg4_full_size_one_launch(cuda):
    """BASELINE config 4 at its stated size on one GPU: all 4,096 bags, N_b = rng(0).integers(256,
    2049, 4096) (sum ~4.72 M instances), T = 100, bf16 separate heads, ONE varlen launch with the
    global bag ids. Every bag: A sums to 1 over its instances for every (t, c), A_mean / A_var
    equal the mean / unbiased variance of its A over T, P_mean the mean softmax of its Y; the whole
    launch is bitwise repeatable; the smallest, the largest and two other bags against the
    reference restatement on the same bf16 operands (fp32 bounds x 10)."""
    from mcgmil import ops
    sizes = np.random.default_rng(0).integers(256, 2049, 4096).tolist()
    B, T, C, L, seed = len(sizes), 100, 2, 512, 42
    R = int(sum(sizes))
    sd = synthetic.head_state_dict(0, C=C, shared=False)
    head = head_on(synthetic.head_arrays(sd, C, False), cuda)
    g = torch.Generator(device=cuda).manual_seed(4)
    H = torch.randn(R, L, device=cuda, generator=g).abs_().bfloat16()
    offs = ops.bag_offsets_tensor(sizes, cuda)
    ids = torch.arange(B, dtype=torch.int32, device=cuda)
    kw = dict(p_feat=0.1, p_att=0.1, seed=seed, bag_ids=ids, return_stats=True)
    out = ops.mcdo_forward(H, offs, head, T, **kw)
    again = ops.mcdo_forward(H, offs, head, T, **kw)
    for k in out:
        assert torch.equal(out[k], again[k]), k
    del again
    n_t = torch.tensor(sizes, device=cuda, dtype=torch.int64)
    # A: per bag [T, C, N_b] -> sums over instances, one per (bag, t, c)
    sums = torch.segment_reduce(out["A"], "sum", lengths=n_t.repeat_interleave(T * C))
    assert float((sums - 1).abs().max()) <= 1e-5
    assert bool((out["A"] >= 0).all())
    # A_mean / A_var against torch's mean / var over T, bag by bag on the device
    err_m = torch.zeros((), device=cuda)
    err_v = torch.zeros((), device=cuda)
    Ab = torch.split(out["A"], (n_t * T * C).tolist())
    Am = torch.split(out["A_mean"], (n_t * C).tolist())
    Av = torch.split(out["A_var"], (n_t * C).tolist())
    for b, n in enumerate(sizes):
        a = Ab[b].view(T, C, n)
        err_m = torch.maximum(err_m, (Am[b].view(C, n) - a.mean(0)).abs().max())
        v = a.var(0)
        err_v = torch.maximum(err_v, ((Av[b].view(C, n) - v).abs() - 1e-4 * v.abs()).max())
    assert float(err_m) <= 1e-7 and float(err_v) <= 1e-12
    P = torch.softmax(out["Y"], -1).mean(1)
    assert torch.allclose(out["P_mean"], P, atol=1e-6)
    prm = mcdo_ref.HeadParams(synthetic.head_arrays(synthetic.round_state_dict_bf16(sd), C, False))
    starts = np.concatenate([[0], np.cumsum(sizes)])
    for b in sorted({int(np.argmin(sizes)), int(np.argmax(sizes)), 1000, 4095}):
        n = sizes[b]
        Hb = H[starts[b]:starts[b + 1]].float().cpu().numpy()
        kF, kA = mcdo_ref.masks_for_bag(seed, b, T, n, L, C, 0.1, 0.1)
        Yr, Ar = mcdo_ref.mc_inference(Hb, prm, kF, kA, 0.1, 0.1)
        np.testing.assert_allclose(out["Y"][b].cpu().numpy(), Yr[:, 0].numpy(), atol=TOL_BF16_IN["Y"])
        assert nrel(Ab[b].cpu().numpy().reshape(T, C, n), Ar[:, 0].numpy()) <= TOL_BF16_IN["A"]
        assert nrel(Am[b].cpu().numpy().reshape(C, n), Ar[:, 0].mean(0).numpy()) <= TOL_BF16_IN["A_mean"]
