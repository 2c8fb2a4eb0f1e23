"""The single-launch hot path (gate_fused_kernel via mcgmil_gate_softmax_pool, reference
model.py:280-316) against the two-kernel
path (gate_pipe_kernel / gate_pp_kernel -> workspace -> softmax_pool_kernel) and against the
reference's golden outputs.

Both paths run the same tile code and the same softmax_group, so every output must be BITWISE
equal. The cases cover the fused kernel's region shapes: several t-groups per region (small N),
one t-group per region (N = 2048 at cap 4096), bags larger than the LDS cap (logits through the
global workspace, incl. > 4,096 instances: the streaming softmax), empty bags (Y = 0), ragged
batches (the device region plan) and uniform ones (arithmetic region map), C = 1, 2, 4.
The launch is chosen through mcgmil_args.flags (path=, gate=): the MCGMIL_FUSED / MCGMIL_GATE
overrides are read once per process (tests/test_capi.py runs them in a subprocess)."""
import numpy as np
import pytest
import torch

from golden_util import Case
from oracle import mcdo_ref
from mcgmil import synthetic

pytestmark = pytest.mark.gpu


def head_on(arrays, dev):
    from mcgmil.ops import HeadTensors
    return HeadTensors(*[torch.from_numpy(np.ascontiguousarray(arrays[k])).to(dev)
                         for k in HeadTensors._fields])


def regions(H, offs, head, T, path="auto", gate="auto"):
    import ctypes
    from mcgmil import _lib, ops
    a = ops.make_args(H, offs, head, T, head.C, head.G, head.D, 0.1, 0.1, seed=1, path=path, gate=gate)
    n = ctypes.c_size_t()
    _lib.check(_lib.load().mcgmil_workspace_size(ctypes.byref(a), ctypes.byref(n)), "ws")
    ws = torch.empty(max(n.value, 1), dtype=torch.uint8, device=H.device)
    a.workspace, a.workspace_bytes = ctypes.c_void_p(ws.data_ptr()), n.value
    Y = torch.empty(offs.numel() - 1, T, head.C, device=H.device)
    a.Y = ctypes.c_void_p(Y.data_ptr())
    r = ctypes.c_int64()
    _lib.check(_lib.load().mcgmil_fused_regions(ctypes.byref(a), ctypes.byref(r)), "fused_regions")
    return r.value


CASES = [
    # name, dtype, sizes, T, C, shared, D
    ("bf16_sep_uniform_N2048", torch.bfloat16, [2048] * 3, 7, 2, False, 128),
    ("bf16_sep_uniform_N300", torch.bfloat16, [300] * 4, 30, 2, False, 128),
    ("bf16_sep_ragged", torch.bfloat16, [300, 0, 5000, 1, 129, 4096, 4097, 777], 5, 2, False, 128),
    ("f32_sep_ragged", torch.float32, [17, 2048, 0, 640, 4100], 6, 2, False, 128),
    ("f32_shared_uniform_N96", torch.float32, [96] * 5, 40, 2, True, 128),
    ("f32_c4_sep_ragged", torch.float32, [50, 1500, 1024, 1025, 3], 4, 4, False, 64),
    ("bf16_c1_ragged", torch.bfloat16, [33, 4000, 5], 9, 1, False, 128),
    # bf16 heads of <= 8 gate tile pairs (auto: gate_pp_kernel, no fused form): both paths with the
    # gate forced to gate_pipe_kernel, whose tile the fused launch runs; incl. bags over the cap and
    # D = 64 separate heads
    ("bf16_shared_uniform_N2048", torch.bfloat16, [2048] * 3, 7, 2, True, 128),
    ("bf16_shared_uniform_N300", torch.bfloat16, [300] * 4, 30, 2, True, 128),
    ("bf16_shared_ragged", torch.bfloat16, [300, 0, 5000, 1, 129, 2048, 2049, 777], 5, 2, True, 128),
    ("bf16_c4_shared_ragged", torch.bfloat16, [50, 1500, 512, 513, 3], 4, 4, True, 128),
    ("bf16_sep_d64_ragged", torch.bfloat16, [700, 96, 2049, 0], 6, 2, False, 64),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_fused_equals_two_kernel_path(cuda, case):
    from mcgmil import ops
    name, dtype, sizes, T, C, shared, D = case
    L = 512
    sd = synthetic.head_state_dict(5, L=L, D=D, C=C, shared=shared)
    head = head_on(synthetic.head_arrays(sd, C, shared), cuda)
    H = torch.cat([torch.from_numpy(synthetic.bag_features(60 + b, n, L)) for b, n in enumerate(sizes)]) \
        .to(cuda).to(dtype).contiguous()
    offs = ops.bag_offsets_tensor(sizes, cuda)
    ids = torch.tensor([7 * b + 3 for b in range(len(sizes))], dtype=torch.int32, device=cuda)
    kw = dict(p_feat=0.1, p_att=0.1, seed=1234, bag_ids=ids, return_stats=True)
    gate = "pipe" if dtype == torch.bfloat16 and head.G * D // 16 <= 8 else "auto"
    if gate == "pipe":          # gate_pp_kernel heads have no fused form under auto
        assert regions(H, offs, head, T, path="fused") == 0
    assert regions(H, offs, head, T, path="two_kernel", gate=gate) == 0
    ref = ops.mcdo_forward(H, offs, head, T, path="two_kernel", gate=gate, **kw)
    nreg = regions(H, offs, head, T, path="fused", gate=gate)
    out = ops.mcdo_forward(H, offs, head, T, path="fused", gate=gate, **kw)
    torch.cuda.synchronize()
    assert nreg > 0
    for k in ref:
        assert torch.equal(out[k], ref[k]) or (k == "A_var" and T == 1), k
    # empty bags: Y = 0 (the reference would not produce a bag of 0 instances; the kernel's rule)
    for b, n in enumerate(sizes):
        if n == 0:
            assert torch.count_nonzero(out["Y"][b]) == 0


def test_fused_auto_policy(cuda):
    """path="auto" (the default) takes the fused launch only for bf16 batches of equal-size bags
    with >= 16,384 regions: 16 bags of N=2048, T=100 (800 regions of two t-groups) do not, 512 bags
    (25,600, the bench's step) do, ragged, fp32 or bf16 shared-head batches do not.
    path="two_kernel": never."""
    from mcgmil import ops
    sd = synthetic.head_state_dict(0, C=2, shared=False)
    head = head_on(synthetic.head_arrays(sd, 2, False), cuda)
    small = torch.zeros(16 * 2048, 512, device=cuda, dtype=torch.bfloat16)
    small_offs = ops.bag_offsets_tensor([2048] * 16, cuda)
    big = torch.zeros(512 * 2048, 512, device=cuda, dtype=torch.bfloat16)
    big_offs = ops.bag_offsets_tensor([2048] * 512, cuda)
    assert regions(small, small_offs, head, 100) == 0
    assert regions(big, big_offs, head, 100) == 512 * 50
    assert regions(big, big_offs, head, 100, path="two_kernel") == 0
    # ragged batches (config 4) stay on the two-kernel path under auto, however many regions
    ragged_offs = ops.bag_offsets_tensor([2047, 2049] * 256, cuda)
    assert regions(big, ragged_offs, head, 100) == 0
    assert regions(big, ragged_offs, head, 100, path="fused") > 16384
    # fp32 stays on the two-kernel path under auto (the fused fp32 tile loop spills: 13-18% slower)
    big32 = torch.zeros(1280 * 512, 512, device=cuda, dtype=torch.float32)   # 1280 bags x 13 regions
    offs32 = ops.bag_offsets_tensor([512] * 1280, cuda)
    assert regions(big32, offs32, head, 100) == 0
    assert regions(big32, offs32, head, 100, path="fused") == 1280 * 13
    # bf16 shared heads stay on gate_pp_kernel + softmax_pool_kernel (the fused 8-wave tile measured
    # 5.53 vs 4.04-4.10 ms per 64 bags); fused only with the gate forced to the 8-wave tile
    sd = synthetic.head_state_dict(0, C=2, shared=True)
    shead = head_on(synthetic.head_arrays(sd, 2, True), cuda)
    assert regions(big, big_offs, shead, 100) == 0
    assert regions(big, big_offs, shead, 100, path="fused") == 0
    assert regions(big, big_offs, shead, 100, path="fused", gate="pp") == 0
    assert regions(big, big_offs, shead, 100, path="fused", gate="pipe") == 512 * 50


from test_gpu_parity import BF16_CASES, FP32_CASES, TOL32, TOL_BF16_IN, compare, run  # noqa: E402


@pytest.mark.parametrize("name", FP32_CASES + BF16_CASES)
def test_fused_matches_reference_goldens(cuda, name):
    """The fused launch (forced) on every reference-made golden MC case, with the kernel's own
    Philox masks, at the bounds of tests/test_gpu_parity.py."""
    case = Case(name)
    bf16 = name in BF16_CASES
    out = run(case, cuda, torch.bfloat16 if bf16 else torch.float32, path="fused")
    compare(case, out, TOL_BF16_IN if bf16 else TOL32)


def test_fused_config3_bag_vs_oracle(cuda):
    """One config-3 bag (N=2048, T=100, bf16 operands) through the fused launch against the CPU
    oracle on the bf16-rounded inputs (the fp32 bounds x 10)."""
    from mcgmil import ops
    N, T, seed = 2048, 100, 77
    sd = synthetic.head_state_dict(seed, C=2, shared=False)
    Hn = synthetic.bf16_round(synthetic.bag_features(seed + 1, N))
    head = head_on(synthetic.head_arrays(sd, 2, False), cuda)
    out = ops.mcdo_forward(torch.from_numpy(Hn).to(cuda).bfloat16(), ops.bag_offsets_tensor([N], cuda),
                           head, T, p_feat=0.1, p_att=0.1, seed=seed, bag_id_base=9, return_stats=True,
                           path="fused")
    torch.cuda.synchronize()
    kF, kA = mcdo_ref.masks_for_bag(seed, 9, T, N, 512, 2, 0.1, 0.1)
    Yr, Ar = mcdo_ref.mc_inference(Hn, mcdo_ref.HeadParams(synthetic.head_arrays(
        synthetic.round_state_dict_bf16(sd), 2, False)), kF, kA, 0.1, 0.1)
    Yr, Ar = Yr.numpy()[:, 0], Ar.numpy()[:, 0]
    np.testing.assert_allclose(out["Y"][0].cpu().numpy(), Yr, rtol=0, atol=1e-4)
    A = out["A"].cpu().numpy().reshape(T, 2, N)
    assert np.abs(A - Ar).max() / np.abs(Ar).max() <= 1e-4


# ------------------------------------------------------------------ the launch bench.py times
def _oracle_bag(H_rows, sd, T, seed, bag_ctr, N):
    """Reference outputs (mcdo_ref, model.py:280-316) of one bag on its bf16 operands exactly:
    H rows already bf16-representable, weights bf16-rounded; masks from the C Philox."""
    kF, kA = mcdo_ref.masks_for_bag(seed, bag_ctr, T, N, 512, 2, 0.1, 0.1)
    prm = mcdo_ref.HeadParams(synthetic.head_arrays(synthetic.round_state_dict_bf16(sd), 2, False))
    Yr, Ar = mcdo_ref.mc_inference(H_rows, prm, kF, kA, 0.1, 0.1)
    return Yr.numpy()[:, 0], Ar.numpy()[:, 0]                  # [T, C], [T, C, N]


def _check_vs_oracle(out, b, sizes_before, N, T, Yr, Ar):
    from test_gpu_parity import TOL_BF16_IN
    Y = out["Y"][b].cpu().numpy()
    o = T * 2 * sizes_before
    A = out["A"][o:o + T * 2 * N].cpu().numpy().reshape(T, 2, N)
    Am = out["A_mean"][2 * sizes_before:2 * sizes_before + 2 * N].cpu().numpy().reshape(2, N)
    np.testing.assert_allclose(Y, Yr, rtol=0, atol=TOL_BF16_IN["Y"])
    assert np.abs(A - Ar).max() / np.abs(Ar).max() <= TOL_BF16_IN["A"]
    assert np.abs(Am - Ar.mean(0)).max() / np.abs(Ar.mean(0)).max() <= TOL_BF16_IN["A_mean"]


@pytest.mark.parametrize("B", [8, 16])
def test_fused_xcd_region_map_uniform_bags(cuda, B):
    """The fused kernel's XCD region map (decode_region, mcgmil_kernels.h: uniform bags with
    B % 8 == 0 -- the branch bench.py's 512-bag step runs): B bags of N = 256, T = 100, bf16
    separate heads, per-bag global ids, forced fused through mcgmil_args.flags. Every output
    bitwise equal to the two-kernel path; the first bag, the last and one on another XCD
    (b % 8 == 5) against the reference restatement on the same bf16 operands."""
    from mcgmil import ops
    N, T, seed = 256, 100, 4242
    sd = synthetic.head_state_dict(11, C=2, shared=False)
    head = head_on(synthetic.head_arrays(sd, 2, False), cuda)
    Hs = [synthetic.bf16_round(synthetic.bag_features(900 + b, N)) for b in range(B)]
    H = torch.from_numpy(np.concatenate(Hs)).to(cuda).bfloat16()
    offs = ops.bag_offsets_tensor([N] * B, cuda)
    ids = [31 * b + 5 for b in range(B)]
    kw = dict(p_feat=0.1, p_att=0.1, seed=seed, return_stats=True,
              bag_ids=torch.tensor(ids, dtype=torch.int32, device=cuda))
    assert offs.uniform_rows == N
    assert regions(H, offs, head, T) == 0                       # auto: too few regions
    a = ops.make_args(H, offs, head, T, 2, 2, 128, 0.1, 0.1, seed=1, path="fused")
    import ctypes
    from mcgmil import _lib
    n = ctypes.c_size_t()
    _lib.check(_lib.load().mcgmil_workspace_size(ctypes.byref(a), ctypes.byref(n)), "ws")
    ws = torch.empty(n.value, dtype=torch.uint8, device=cuda)
    a.workspace, a.workspace_bytes = ctypes.c_void_p(ws.data_ptr()), n.value
    r = ctypes.c_int64()
    _lib.check(_lib.load().mcgmil_fused_regions(ctypes.byref(a), ctypes.byref(r)), "fused_regions")
    assert r.value == B * 7                                     # 16 t-groups per region: 7 per bag
    out = ops.mcdo_forward(H, offs, head, T, path="fused", **kw)
    ref = ops.mcdo_forward(H, offs, head, T, path="two_kernel", **kw)
    again = ops.mcdo_forward(H, offs, head, T, path="fused", **kw)
    torch.cuda.synchronize()
    for k in ref:
        assert torch.equal(out[k], ref[k]), k
        assert torch.equal(out[k], again[k]), k
    for b in sorted({0, 5, B - 1}):
        Yr, Ar = _oracle_bag(Hs[b], sd, T, seed, ids[b], N)
        _check_vs_oracle(out, b, b * N, N, T, Yr, Ar)


def test_fused_bench_step_shape(cuda):
    """bench.py's own step: 512 bags of N = 2048, T = 100, bf16 separate heads, default (auto)
    policy = ONE gate_fused_kernel launch of 25,600 regions over the XCD region map. All outputs
    bitwise equal to the two-kernel path and repeatable; bags 0, 13 (XCD 5) and 511 against the
    reference restatement on the same bf16 operands (fp32 bounds x 10)."""
    from mcgmil import ops
    B, N, T, seed = 512, 2048, 100, 42
    sd = synthetic.head_state_dict(0, C=2, shared=False)
    head = head_on(synthetic.head_arrays(sd, 2, False), cuda)
    g = torch.Generator(device=cuda).manual_seed(1000)
    H = torch.randn(B * N, 512, device=cuda, generator=g).abs_().bfloat16()
    offs = ops.bag_offsets_tensor([N] * B, cuda)
    ids = torch.arange(B, dtype=torch.int32, device=cuda)
    kw = dict(p_feat=0.1, p_att=0.1, seed=seed, bag_ids=ids, return_stats=True)
    assert regions(H, offs, head, T) == B * 50
    out = ops.mcdo_forward(H, offs, head, T, **kw)               # auto -> fused
    ref = ops.mcdo_forward(H, offs, head, T, path="two_kernel", **kw)
    torch.cuda.synchronize()
    for k in ref:
        assert torch.equal(out[k], ref[k]), k
    del ref
    again = ops.mcdo_forward(H, offs, head, T, **kw)
    for k in out:
        assert torch.equal(out[k], again[k]), k
    del again
    A = out["A"].view(B, T, 2, N)
    assert torch.allclose(A.sum(-1), torch.ones(B, T, 2, device=cuda), atol=1e-5)
    for b in (0, 13, 511):
        Hb = H[b * N:(b + 1) * N].float().cpu().numpy()
        Yr, Ar = _oracle_bag(Hb, sd, T, seed, b, N)
        _check_vs_oracle(out, b, b * N, N, T, Yr, Ar)


def test_path_and_gate_flags_agree(cuda):
    """mcgmil_args.flags: the fused launch, the two-kernel launch and the two-kernel launch with
    the gate kernel forced (gate="pipe") give bitwise the same outputs; an unknown path raises."""
    from mcgmil import ops
    sizes = [300] * 8
    sd = synthetic.head_state_dict(3, C=2, shared=False)
    head = head_on(synthetic.head_arrays(sd, 2, False), cuda)
    H = torch.from_numpy(np.concatenate([synthetic.bag_features(70 + b, n) for b, n in enumerate(sizes)])) \
        .to(cuda).bfloat16()
    offs = ops.bag_offsets_tensor(sizes, cuda)
    kw = dict(p_feat=0.1, p_att=0.1, seed=9, return_stats=True)
    a = ops.mcdo_forward(H, offs, head, 30, path="fused", **kw)
    b = ops.mcdo_forward(H, offs, head, 30, path="two_kernel", **kw)
    c = ops.mcdo_forward(H, offs, head, 30, path="two_kernel", gate="pipe", **kw)
    for k in a:
        assert torch.equal(a[k], b[k]) and torch.equal(a[k], c[k]), k
    with pytest.raises(ValueError):
        ops.mcdo_forward(H, offs, head, 30, path="bogus", **kw)


def _random_cases(n=12, seed=2024):
    rng = np.random.default_rng(seed)
    cases = []
    for i in range(n):
        C = int(rng.choice([1, 2, 3, 4]))
        shared = bool(rng.integers(0, 2)) if C > 1 else False
        D = int(rng.choice([64, 128]))
        B = int(rng.integers(1, 7))
        sizes = [int(x) for x in rng.integers(0, 700, B)]
        if rng.random() < 0.3:
            sizes = [sizes[0]] * B                           # uniform: arithmetic region map
        T = int(rng.integers(1, 41))
        p_f = float(rng.choice([0.0, 0.1, 0.37, 1.0]))
        p_a = float(rng.choice([0.0, 0.1, 0.5, 1.0]))
        dtype = torch.bfloat16 if rng.random() < 0.5 else torch.float32
        cases.append((f"r{i}", dtype, sizes, T, C, shared, D, p_f, p_a))
    return cases


@pytest.mark.parametrize("case", _random_cases(), ids=lambda c: c[0])
def test_random_shapes_fused_two_kernel_oracle(cuda, case):
    """Seeded random sweep over the fused launch's parameter space (bag sizes incl. 0, T, C, head
    layout, D, dropout p incl. 0 and 1, dtype): the fused and two-kernel paths bitwise equal, and
    every non-empty bag against the reference restatement (mcdo_ref, model.py:280-316) with the
    kernel's own masks, on the same operands (bf16-rounded for bf16) at the fp32 bounds (x 10)."""
    from mcgmil import ops
    from test_gpu_parity import TOL32, TOL_BF16_IN
    name, dtype, sizes, T, C, shared, D, p_f, p_a = case
    L, seed = 512, 4000 + int(name[1:])
    sd = synthetic.head_state_dict(seed, L=L, D=D, C=C, shared=shared)
    bf16 = dtype == torch.bfloat16
    Hs = [synthetic.bag_features(seed + 10 + b, n, L) for b, n in enumerate(sizes)]
    if bf16:
        Hs = [synthetic.bf16_round(h) for h in Hs]
    head = head_on(synthetic.head_arrays(sd, C, shared), cuda)
    H = torch.from_numpy(np.concatenate(Hs)).to(cuda).to(dtype).contiguous()
    offs = ops.bag_offsets_tensor(sizes, cuda)
    kw = dict(p_feat=p_f, p_att=p_a, seed=seed, bag_id_base=17, return_stats=True)
    two = ops.mcdo_forward(H, offs, head, T, path="two_kernel", **kw)
    # bf16 heads on gate_pp_kernel (<= 8 gate tile pairs) fuse on the 8-wave tile only: compare the
    # fused launch with the two-kernel path on that same tile (gate="pipe")
    gate = "pipe" if bf16 and head.G * D // 16 <= 8 else "auto"
    fz = ops.mcdo_forward(H, offs, head, T, path="fused", gate=gate, **kw)
    same = two if gate == "auto" else ops.mcdo_forward(H, offs, head, T, path="two_kernel", gate=gate, **kw)
    for k in two:
        assert torch.equal(torch.nan_to_num(fz[k], nan=7.0), torch.nan_to_num(same[k], nan=7.0)), k
    tol = TOL_BF16_IN if bf16 else TOL32
    sd_ref = synthetic.round_state_dict_bf16(sd) if bf16 else sd
    prm = mcdo_ref.HeadParams(synthetic.head_arrays(sd_ref, C, shared))
    Y = two["Y"].cpu().numpy()
    A = ops.split_bags(two["A"].cpu(), sizes, T * C)
    for b, n in enumerate(sizes):
        if n == 0:
            assert np.all(Y[b] == 0)
            continue
        kF, kA = mcdo_ref.masks_for_bag(seed, 17 + b, T, n, L, C, p_f, p_a)
        Yr, Ar = mcdo_ref.mc_inference(Hs[b], prm, kF, kA, p_f, p_a)
        np.testing.assert_allclose(Y[b], Yr[:, 0].numpy(), rtol=0, atol=tol["Y"])
        Ar = Ar[:, 0].numpy()
        assert np.abs(A[b].numpy().reshape(T, C, n) - Ar).max() <= tol["A"] * max(np.abs(Ar).max(), 1e-30)


@pytest.mark.parametrize("path,shared", [("fused", False), ("fused", True), ("two_kernel", False), ("two_kernel", True)])
def test_clock_probe(cuda, path, shared):
    """MCGMIL_CLOCK_PROBE (the clock bench.py states in every roofline): the probed launch runs the
    PROBE instantiation of the same tile kernel -- outputs bitwise equal to the unprobed launch --
    and every workgroup that owns a record slot writes start/end (s_memtime, s_memrealtime) stamps
    from which a plausible shader clock follows."""
    import ctypes
    from mcgmil import _lib, ops
    B, N, T = (128, 256, 100) if path == "fused" else (4, 700, 20)
    sd = synthetic.head_state_dict(8, C=2, shared=shared)
    head = head_on(synthetic.head_arrays(sd, 2, shared), cuda)
    H = torch.rand(B * N, 512, device=cuda).bfloat16()
    offs = ops.bag_offsets_tensor([N] * B, cuda)
    packed = ops.packed_weights(head, torch.bfloat16)      # the stages need packed weights
    outs = []
    for probe in (False, True):
        # shared heads fuse only on the 8-wave tile (gate="pipe"); the two-kernel path probes gate_pp_kernel
        a = ops.make_args(H, offs, head, T, 2, head.G, 128, 0.1, 0.1, seed=3, path=path,
                          gate="pipe" if shared and path == "fused" else "auto")
        a.packed_w = ctypes.c_void_p(packed.data_ptr())
        n = ctypes.c_size_t()
        lib = _lib.load()
        _lib.check(lib.mcgmil_workspace_size(ctypes.byref(a), ctypes.byref(n)), "ws")
        ws = torch.empty(n.value, dtype=torch.uint8, device=cuda)
        a.workspace, a.workspace_bytes = ctypes.c_void_p(ws.data_ptr()), n.value
        Y = torch.empty(B, T, 2, device=cuda)
        A = torch.empty(T * 2 * B * N, device=cuda)
        a.Y, a.A = ctypes.c_void_p(Y.data_ptr()), ctypes.c_void_p(A.data_ptr())
        rec = ops.clock_record(cuda)
        if probe:
            a.debug, a.flags = ctypes.c_void_p(rec.data_ptr()), a.flags | _lib.CLOCK_PROBE
        regions = ctypes.c_int64()
        _lib.check(lib.mcgmil_fused_regions(ctypes.byref(a), ctypes.byref(regions)), "regions")
        assert (regions.value > 0) == (path == "fused")
        sh = ctypes.c_void_p(torch.cuda.current_stream(cuda).cuda_stream)
        _lib.check(lib.mcgmil_gate_softmax_pool(ctypes.byref(a), sh), "gate_softmax_pool")
        torch.cuda.synchronize()
        outs.append((Y.clone(), A.clone(), rec.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert int(torch.count_nonzero(outs[0][2])) == 0          # no probe: nothing written
    r = outs[1][2]
    wrote = int(((r[:, 2] > r[:, 0]) & (r[:, 3] > r[:, 1])).sum())
    grid = regions.value if path == "fused" else (T * B * N + 127) // 128
    assert wrote == min(grid, _lib.CLOCK_SLOTS)
    c = ops.clock_mhz(outs[1][2])
    assert c is not None and 500.0 < c["median"] < 3000.0, c
