"""The C ABI library (CPU-side checks only: no kernel launches without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import REPO

HEADERS = [os.path.join(REPO, "include", h) for h in ("mcgmil.h", "mcgmil_image.h", "mcgmil_features.h",
                                                            "mcgmil_calib.h")]


def declared_functions():
    src = "".join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|size_t|const char\*)\s+(mcgmil_\w+)\s*\(", src, re.M)))


def test_header_declares_entry_points():
    fns = declared_functions()
    for f in ("mcgmil_mcdo_forward", "mcgmil_workspace_size", "mcgmil_pack_weights",
              "mcgmil_last_error", "mcgmil_feature_keep", "mcgmil_attention_keep"):
        assert f in fns


def test_library_exports_every_declared_symbol(hip_lib):
    from mcgmil import _lib
    for f in declared_functions():
        assert hasattr(hip_lib, f), f
    assert set(declared_functions()) == set(_lib.EXPORTED)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.lib_path()], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (mcgmil_\w+)", out))
    assert set(declared_functions()) <= exported


def test_library_targets_gfx950(hip_lib):
    from mcgmil import _lib
    data = open(_lib.lib_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data   # the embedded offload bundle's target


def test_args_struct_matches_binding(hip_lib):
    from mcgmil import _lib
    assert hip_lib.mcgmil_abi_version() == 6 == _lib.ABI_VERSION
    assert hip_lib.mcgmil_conv_args_size() == ctypes.sizeof(_lib.ConvArgs)
    assert hip_lib.mcgmil_stem_args_size() == ctypes.sizeof(_lib.StemArgs)
    assert hip_lib.mcgmil_args_size() == ctypes.sizeof(_lib.Args)
    assert hip_lib.mcgmil_image_args_size() == ctypes.sizeof(_lib.ImageArgs)
    assert hip_lib.mcgmil_bn_args_size() == ctypes.sizeof(_lib.BnArgs)


def _args(**kw):
    from mcgmil import _lib
    a = _lib.Args()
    a.L, a.D, a.C, a.G, a.T, a.num_bags, a.total_rows = 512, 128, 2, 2, 100, 1, 2048
    a.h_dtype = _lib.MCGMIL_BF16
    a.bag_offsets = ctypes.c_void_p(0x1000)
    a.p_feat = a.p_att = 0.1
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def _ws(hip_lib, a):
    n = ctypes.c_size_t()
    rc = hip_lib.mcgmil_workspace_size(ctypes.byref(a), ctypes.byref(n))
    return rc, n.value


def test_workspace_size_formula(hip_lib):
    rc, n = _ws(hip_lib, _args())
    assert rc == 0
    packed = (2 * 16 + 1) * 16 * 512 * 2                     # (2P+1) tiles x KS x 512 x bf16
    scores = 100 * 2048 * 2 * 4
    plan = ((100 * 2048 // 16 * 4 + 255) // 256) * 256      # tile plan (int32 per 16-row tile)
    regions = 256                                            # fused region plan: int32 [B+1]
    assert n == ((packed + 255) // 256) * 256 + 2 * scores + plan + regions
    rc, n2 = _ws(hip_lib, _args(packed_w=ctypes.c_void_p(0x2000)))
    assert rc == 0 and n2 == 2 * scores + plan + regions


@pytest.mark.parametrize("field,value,code", [
    ("L", 500, -2), ("L", 4096, -2), ("D", 100, -2), ("C", 5, -2), ("C", 0, -2), ("G", 3, -1),
    ("T", 0, -1), ("num_bags", 0, -1), ("p_feat", 1.5, -1), ("p_att", -0.1, -1),
    ("h_dtype", 7, -1), ("bag_offsets", None, -1), ("total_rows", -1, -1),
    ("flags", 3, -1), ("flags", 12, -1), ("flags", 16, -1), ("flags", 32, -1), ("reserved", 1, -1),
])
def test_validation_errors(hip_lib, field, value, code):
    rc, _ = _ws(hip_lib, _args(**{field: value}))
    assert rc == code
    assert len(hip_lib.mcgmil_last_error()) > 0


def _regions(hip_lib, a):
    rc, n = _ws(hip_lib, a)
    assert rc == 0
    a.workspace, a.workspace_bytes = ctypes.c_void_p(0x100000), n
    a.H, a.ldh = ctypes.c_void_p(0x3000), 512
    a.bv = a.bu = a.wa = a.ba = ctypes.c_void_p(0x4000)
    r = ctypes.c_int64(-1)
    assert hip_lib.mcgmil_fused_regions(ctypes.byref(a), ctypes.byref(r)) == 0
    return r.value


def test_path_flags_select_the_launch(hip_lib, monkeypatch):
    """mcgmil_args.flags picks the launch mcgmil_gate_softmax_pool makes (host logic, no launch):
    auto = fused only for bf16 batches of equal-size bags with >= 16,384 regions; FUSED whenever
    it applies; TWO_KERNEL never; MCGMIL_GATE_PP keeps bf16 heads off the fused (pipe) tile code;
    bf16 heads on gate_pp_kernel (shared) fuse only with the gate forced to gate_pipe_kernel."""
    from mcgmil import _lib
    F, G = _lib.PATH_FLAGS, _lib.GATE_FLAGS
    small = dict(num_bags=16, total_rows=16 * 2048, uniform_bag_rows=2048)
    big = dict(num_bags=512, total_rows=512 * 2048, uniform_bag_rows=2048)
    assert _regions(hip_lib, _args(**small)) == 0
    assert _regions(hip_lib, _args(**big)) == 512 * 50
    assert _regions(hip_lib, _args(flags=F["fused"], **small)) == 16 * 50
    assert _regions(hip_lib, _args(flags=F["two_kernel"], **big)) == 0
    assert _regions(hip_lib, _args(flags=F["fused"] | G["pp"], **small)) == 0
    assert _regions(hip_lib, _args(flags=F["fused"] | G["pipe"], **small)) == 16 * 50
    assert _regions(hip_lib, _args(G=1, **big)) == 0                          # shared: gate_pp_kernel
    assert _regions(hip_lib, _args(G=1, flags=F["fused"], **small)) == 0
    assert _regions(hip_lib, _args(G=1, flags=F["fused"] | G["pipe"], **small)) == 16 * 50
    assert _regions(hip_lib, _args(G=1, flags=G["pipe"], **big)) == 512 * 50
    assert _regions(hip_lib, _args(flags=F["fused"], h_dtype=_lib.MCGMIL_F32, **small)) == 16 * 50
    assert _regions(hip_lib, _args(h_dtype=_lib.MCGMIL_F32, **big)) == 0      # fp32: auto stays off


_ENV_PROBE = r"""
import ctypes, sys
sys.path[:0] = [{repo!r}, {pkg!r}]
import test_capi as t
from mcgmil import _lib
lib = _lib.load()
F = _lib.PATH_FLAGS
small = dict(num_bags=16, total_rows=16 * 2048, uniform_bag_rows=2048)
big = dict(num_bags=512, total_rows=512 * 2048, uniform_bag_rows=2048)
print(t._regions(lib, t._args(flags=F["two_kernel"], **small)), t._regions(lib, t._args(flags=F["fused"], **big)),
      t._regions(lib, t._args(flags=F["fused"], **small)))
"""


@pytest.mark.parametrize("env,want", [("1", [16 * 50, 512 * 50, 16 * 50]), ("0", [0, 0, 0]),
                                      ("auto", [0, 512 * 50, 0])])
def test_fused_environment_override(hip_lib, env, want):
    """MCGMIL_FUSED in the environment overrides the flags; it is read once per process, so each
    setting runs in a fresh interpreter (host logic, no launch)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    code = _ENV_PROBE.format(repo=here, pkg=os.path.join(repo, "montecarlo-gated-mil_amd"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, MCGMIL_FUSED=env))
    assert r.returncode == 0, r.stderr[-2000:]
    assert [int(v) for v in r.stdout.split()[-3:]] == want


def test_forward_rejects_missing_workspace(hip_lib):
    a = _args()
    rc = hip_lib.mcgmil_mcdo_forward(ctypes.byref(a), None)
    assert rc == -4
    assert b"workspace" in hip_lib.mcgmil_last_error()


def test_gate_rejects_misaligned_H(hip_lib):
    a = _args(packed_w=ctypes.c_void_p(0x2000))
    rc, n = _ws(hip_lib, a)
    a.workspace, a.workspace_bytes = ctypes.c_void_p(0x10000), n
    a.H, a.ldh = ctypes.c_void_p(0x3002), 512
    a.bv = a.bu = a.wa = a.ba = ctypes.c_void_p(0x4000)
    assert hip_lib.mcgmil_gate_scores(ctypes.byref(a), None) == -3
    a.H, a.ldh = ctypes.c_void_p(0x3000), 509
    assert hip_lib.mcgmil_gate_scores(ctypes.byref(a), None) == -1  # ldh < L


def test_mfma_calib_sizes_and_validation(hip_lib):
    """mcgmil_calib.h: FLOPs per workgroup-step (8 waves x 32 bf16 16x16x32 / 128 fp32 16x16x4
    MFMAs) and the argument checks (no launches)."""
    from mcgmil import _lib
    assert hip_lib.mcgmil_mfma_calib_flops_per_step(_lib.MCGMIL_BF16) == 8 * 32 * 16 * 16 * 32 * 2
    assert hip_lib.mcgmil_mfma_calib_flops_per_step(_lib.MCGMIL_F32) == 8 * 128 * 16 * 16 * 4 * 2
    assert hip_lib.mcgmil_mfma_calib_flops_per_step(7) == 0
    sink = ctypes.c_void_p(0x1000)
    assert hip_lib.mcgmil_mfma_calib(7, 256, 10, 1, sink, None, None) == -1
    assert hip_lib.mcgmil_mfma_calib(_lib.MCGMIL_BF16, 0, 10, 1, sink, None, None) == -1
    assert hip_lib.mcgmil_mfma_calib(_lib.MCGMIL_BF16, 256, 0, 1, sink, None, None) == -1
    assert hip_lib.mcgmil_mfma_calib(_lib.MCGMIL_BF16, 256, 10, 1, None, None, None) == -1


def _bn(**kw):
    from mcgmil import _lib
    a = _lib.BnArgs()
    a.rows, a.channels, a.dtype, a.eps = 4096, 64, _lib.MCGMIL_BF16, 1e-5
    a.x = a.y = ctypes.c_void_p(0x10000)
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_bn_workspace_size_and_validation(hip_lib):
    """mcgmil_features.h: the workspace query and the argument checks (no launches)."""
    from mcgmil import _lib
    n = ctypes.c_size_t()
    assert hip_lib.mcgmil_bn_workspace_size(ctypes.byref(_bn()), ctypes.byref(n)) == 0
    assert n.value >= 2 * 64 * 4 * 5 and n.value % 256 == 0       # ab + 4 partial workgroups
    bad = {"channels": 12, "rows": 0, "dtype": 7, "relu": 2, "eps": -1.0}
    for k, v in bad.items():
        rc = hip_lib.mcgmil_bn_workspace_size(ctypes.byref(_bn(**{k: v})), ctypes.byref(n))
        assert rc in (-1, -2), (k, rc)
    assert hip_lib.mcgmil_bn_workspace_size(ctypes.byref(_bn(channels=4096)), ctypes.byref(n)) == -2
    assert hip_lib.mcgmil_bn_workspace_size(ctypes.byref(_bn(x=ctypes.c_void_p(0x10008))),
                                            ctypes.byref(n)) == -3
    rc = hip_lib.mcgmil_bn_workspace_size(ctypes.byref(_bn(running_mean=ctypes.c_void_p(0x2000))),
                                          ctypes.byref(n))
    assert rc == -1 and b"running_var" in hip_lib.mcgmil_last_error()
    # a missing workspace is refused before anything is launched
    assert hip_lib.mcgmil_batchnorm_act(ctypes.byref(_bn()), None) == -4


def _stem(**kw):
    from mcgmil import _lib
    a = _lib.StemArgs()
    a.batch, a.in_channels, a.height, a.width = 4, 3, 224, 224
    a.out_channels, a.kernel, a.stride, a.pad = 64, 7, 2, 3
    a.pool_kernel, a.pool_stride, a.pool_pad, a.relu, a.eps = 3, 2, 1, 1, 1e-5
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_stem_sizes_and_validation(hip_lib):
    """mcgmil_stem_*: packed-weight and workspace queries (the workspace holds the 112 x 112 x 64
    activation when pooling) and the shapes the kernel refuses (no launches)."""
    n = ctypes.c_size_t()
    assert hip_lib.mcgmil_stem_packed_size(ctypes.byref(_stem()), ctypes.byref(n)) == 0
    assert n.value == 6 * 4 * 64 * 16                                  # 21 (ci, kh) rows -> 6 K steps
    assert hip_lib.mcgmil_stem_workspace_size(ctypes.byref(_stem()), ctypes.byref(n)) == 0
    assert n.value >= 4 * 112 * 112 * 64 * 2 and n.value % 256 == 0
    n2 = ctypes.c_size_t()
    assert hip_lib.mcgmil_stem_workspace_size(ctypes.byref(_stem(pool_kernel=0)), ctypes.byref(n2)) == 0
    assert n2.value < 4 * 112 * 112 * 64 * 2                           # conv written into y directly
    for k, v in {"in_channels": 5, "out_channels": 128, "stride": 1, "width": 223, "kernel": 9,
                 "width_wide": 1000}.items():
        a = _stem(width=1000) if k == "width_wide" else _stem(**{k: v})
        assert hip_lib.mcgmil_stem_workspace_size(ctypes.byref(a), ctypes.byref(n)) == -2, k
    assert hip_lib.mcgmil_stem_workspace_size(ctypes.byref(_stem(relu=3)), ctypes.byref(n)) == -1
    assert hip_lib.mcgmil_stem_workspace_size(ctypes.byref(_stem(flags=1)), ctypes.byref(n)) == 0
    assert hip_lib.mcgmil_stem_workspace_size(ctypes.byref(_stem(flags=2)), ctypes.byref(n)) == -1
    assert hip_lib.mcgmil_stem_workspace_size(ctypes.byref(_stem(reserved=1)), ctypes.byref(n)) == -1
    assert hip_lib.mcgmil_stem_forward(ctypes.byref(_stem()), None) == -1   # NULL x / w / y


def test_conv_stats_parts_and_validation(hip_lib):
    """mcgmil_conv_stats_parts: one statistics row per workgroup row of the kernel the layer uses
    (0 for the 256 x 256 shape), and the argument checks (no launches)."""
    from mcgmil import _lib
    p = ctypes.c_int32()

    def conv(cin, cout, k, s, pad, hw=28, **kw):
        a = _lib.ConvArgs()
        a.batch, a.height, a.width, a.in_channels = 8, hw, hw, cin
        a.out_channels, a.kernel_h, a.kernel_w, a.stride, a.pad = cout, k, k, s, pad
        for key, v in kw.items():
            setattr(a, key, v)
        return a
    assert hip_lib.mcgmil_conv_stats_parts(ctypes.byref(conv(64, 64, 3, 1, 1, 56)), ctypes.byref(p)) == 0
    assert p.value >= 1                                                  # layer-1 halo kernel
    assert hip_lib.mcgmil_conv_stats_parts(ctypes.byref(conv(64, 128, 3, 2, 1, 56)), ctypes.byref(p)) == 0
    assert p.value >= 1
    assert hip_lib.mcgmil_conv_stats_parts(ctypes.byref(conv(256, 256, 3, 1, 1, 14)), ctypes.byref(p)) == 0
    assert p.value == 0                                                  # 256 x 256 tiles
    assert hip_lib.mcgmil_conv_stats_parts(ctypes.byref(conv(48, 64, 3, 1, 1)), ctypes.byref(p)) == -2
    assert hip_lib.mcgmil_conv_stats_parts(ctypes.byref(conv(64, 64, 3, 0, 1)), ctypes.byref(p)) == -1
    assert hip_lib.mcgmil_conv_stats_parts(ctypes.byref(conv(64, 64, 3, 1, 1, 20000)), ctypes.byref(p)) == -2
    assert hip_lib.mcgmil_conv2d(ctypes.byref(conv(64, 64, 3, 1, 1)), None) == -1   # NULL x / w / y
    # input BatchNorm: the 3x3 / stride 1 halo kernels only
    for args, want in ((conv(64, 64, 3, 1, 1, 56), 1), (conv(128, 128, 3, 1, 1, 28), 1),
                       (conv(64, 128, 3, 2, 1, 56), 0), (conv(64, 128, 1, 1, 0), 0),
                       (conv(256, 256, 3, 1, 1, 14), 0), (conv(128, 128, 3, 1, 1, 100), 0)):
        assert hip_lib.mcgmil_conv_input_bn(ctypes.byref(args), ctypes.byref(p)) == 0
        assert p.value == want, (args.in_channels, args.width, p.value)
    assert hip_lib.mcgmil_conv_input_bn(ctypes.byref(conv(64, 64, 3, 1, 1, in_relu=2)), ctypes.byref(p)) == -1
    # flags (mcgmil_conv_flags): NOHALO keeps layer 1 off the halo kernel (no input BN there),
    # SMALL gives the 256-channel layer statistics rows again (256 x 128 tiles); bad values refused
    assert hip_lib.mcgmil_conv_input_bn(ctypes.byref(conv(64, 64, 3, 1, 1, 56, flags=1)), ctypes.byref(p)) == 0
    assert p.value == 0
    assert hip_lib.mcgmil_conv_stats_parts(ctypes.byref(conv(256, 256, 3, 1, 1, 14, flags=2)), ctypes.byref(p)) == 0
    assert p.value >= 1
    # 1x1 / stride 2 from 64 channels (layer 2's downsample): the streaming kernel's pixel streams,
    # one row each, at most one per 16-pixel fragment; 256 -> 512 stays on the 256 x 256 dma tiles
    assert hip_lib.mcgmil_conv_stats_parts(ctypes.byref(conv(64, 128, 1, 2, 0, 56)), ctypes.byref(p)) == 0
    assert 1 <= p.value <= (8 * 28 * 28 + 15) // 16
    assert hip_lib.mcgmil_conv_stats_parts(ctypes.byref(conv(64, 128, 1, 2, 0, 4)), ctypes.byref(p)) == 0
    assert p.value == 2                                                  # 32 pixels: 2 fragments
    assert hip_lib.mcgmil_conv_stats_parts(ctypes.byref(conv(256, 512, 1, 2, 0, 14)), ctypes.byref(p)) == 0
    assert p.value == 0
    assert hip_lib.mcgmil_conv_stats_parts(ctypes.byref(conv(64, 64, 3, 1, 1, flags=4)), ctypes.byref(p)) == -1
    assert hip_lib.mcgmil_conv_stats_parts(ctypes.byref(conv(64, 64, 3, 1, 1, reserved=1)), ctypes.byref(p)) == -1


def test_conv_workspace_size(hip_lib):
    """mcgmil_conv_workspace_size: the K split of the last 256 x 256 tiles (without a GPU the plan
    assumes 256 CUs). Config 5's layer 4 (k = 1,507, 7 x 7 x 512: 289 pixel tiles per channel tile
    over 128 workgroup rows) cuts its 33 left tiles into 3 K ranges: 33 x 2 channel tiles x 3
    ranges of 256 x 256 fp32 sums; layer 3 (1,154 tiles over 256 rows: 130 left, 1 range per row)
    and the 1x1 (4 K steps) take none, nor do kernels other than the 256 x 256 one."""
    from mcgmil import _lib
    n = ctypes.c_size_t()

    def conv(cin, cout, k, s, pad, hw, batch=1507, **kw):
        a = _lib.ConvArgs()
        a.batch, a.height, a.width, a.in_channels = batch, hw, hw, cin
        a.out_channels, a.kernel_h, a.kernel_w, a.stride, a.pad = cout, k, k, s, pad
        for key, v in kw.items():
            setattr(a, key, v)
        return a
    for args, want in ((conv(512, 512, 3, 1, 1, 7), 33 * 2 * 3 * 256 * 256 * 4),
                       (conv(256, 512, 3, 2, 1, 14), 33 * 2 * 3 * 256 * 256 * 4),
                       (conv(256, 512, 1, 2, 0, 14), 0), (conv(256, 256, 3, 1, 1, 14), 0),
                       (conv(128, 128, 3, 1, 1, 28), 0), (conv(512, 512, 3, 1, 1, 7, flags=2), 0),
                       (conv(512, 512, 3, 1, 1, 7, batch=2), 0)):
        assert hip_lib.mcgmil_conv_workspace_size(ctypes.byref(args), ctypes.byref(n)) == 0
        assert n.value == want, (args.in_channels, args.width, args.batch, n.value)
    assert hip_lib.mcgmil_conv_workspace_size(ctypes.byref(conv(512, 512, 3, 1, 1, 7)), None) == -1
    assert hip_lib.mcgmil_conv_workspace_size(ctypes.byref(conv(48, 512, 3, 1, 1, 7)), ctypes.byref(n)) == -2
    # a misaligned workspace is refused before anything launches
    bad = conv(512, 512, 3, 1, 1, 7, x=4096, w=4096, y=4096, workspace=4096 + 16, workspace_bytes=1 << 30)
    assert hip_lib.mcgmil_conv2d(ctypes.byref(bad), None) == -3


def test_batchnorm_coefficients_validation(hip_lib):
    """mcgmil_batchnorm_coefficients argument checks (no launches)."""
    from mcgmil import _lib
    ab = ctypes.cast((ctypes.c_float * 128)(), ctypes.c_void_p)
    a = _lib.BnArgs()
    a.rows, a.channels, a.dtype = 100, 64, _lib.MCGMIL_BF16
    assert hip_lib.mcgmil_batchnorm_coefficients(None, ab, None) == -1
    assert hip_lib.mcgmil_batchnorm_coefficients(ctypes.byref(a), None, None) == -1
    # batch statistics from a pass over x: x and a workspace are required
    assert hip_lib.mcgmil_batchnorm_coefficients(ctypes.byref(a), ab, None) == -1
    a.x = ctypes.c_void_p(4096)
    assert hip_lib.mcgmil_batchnorm_coefficients(ctypes.byref(a), ab, None) == -4
    a.channels = 12
    assert hip_lib.mcgmil_batchnorm_coefficients(ctypes.byref(a), ab, None) == -2
