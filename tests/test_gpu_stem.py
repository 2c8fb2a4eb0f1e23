"""GPU parity of the fused ResNet stem (include/mcgmil_features.h, mcgmil_stem_forward): the
torchvision stem maxpool(relu(bn1(conv1(x)))) of the reference's backbone (model.py:166-177) as
torch.autocast runs it in bf16 on every instance of a bag (infer.py:191), with BatchNorm on the
bag's own statistics (infer.py:105-109) or on running statistics.

Reference: fp64 throughout, on the same bf16 input and bf16-rounded weight. The kernel's
convolution accumulates in fp32 and rounds once to bf16 (|dconv| <= 2^-8 |conv| + 1e-5 conv(|x|,
|w|), as tests/test_gpu_conv.py), its statistics are fp32 sums of those rounded values combined in
fp64, and y = conv * a_c + b_c is evaluated in fp32 and rounded once. So, elementwise before the
pooling, |dy| <= |a_c| * |dconv| + 2^-8 |y| + 2e-3 * |a_c| * std_c (the statistics of rounded
values, a bound far above its typical size); max-pooling keeps the window's largest bound.
"""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _stem_layers(cin, k, pad, dev, seed, running=False):
    g = torch.Generator().manual_seed(seed)
    conv = nn.Conv2d(cin, 64, k, 2, pad, bias=False)
    bn = nn.BatchNorm2d(64)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * (2.0 / (cin * k * k)) ** 0.5)
        bn.weight.copy_(torch.randn(64, generator=g) * 0.5 + 1.0)
        bn.weight[::7] *= -1.0
        bn.bias.copy_(torch.randn(64, generator=g) * 0.3)
        bn.running_mean.copy_(torch.randn(64, generator=g) * 0.2)
        bn.running_var.copy_(torch.rand(64, generator=g) + 0.5)
    if not running:
        from mcgmil.resnet import deactivate_batchnorm
        deactivate_batchnorm(bn)
    return conv.to(dev).eval(), bn.to(dev).eval()


def _reference(x, conv, bn, pool, running):
    """fp64 stem on the bf16 input / weight, plus the elementwise error bound (see module doc)."""
    wb = conv.weight.detach().bfloat16().double()
    xd = x.double()
    s, p = conv.stride, conv.padding
    c = F.conv2d(xd, wb, None, s, p)
    mag = F.conv2d(xd.abs(), wb.abs(), None, s, p)
    if running:
        mean, var = bn.running_mean.double(), bn.running_var.double()
    else:
        mean, var = c.mean(dim=(0, 2, 3)), c.var(dim=(0, 2, 3), unbiased=False)
    a = bn.weight.double() / torch.sqrt(var + bn.eps)
    b = bn.bias.double() - mean * a
    y = c * a[None, :, None, None] + b[None, :, None, None]
    dconv = 2.0 ** -8 * c.abs() + 1e-5 * mag
    stat = 0.0 if running else 2e-3 * (a.abs() * torch.sqrt(var))[None, :, None, None]
    bound = a.abs()[None, :, None, None] * dconv + 2.0 ** -8 * y.abs() + stat + 1e-6
    y = torch.relu(y)
    if pool is not None:
        y = F.max_pool2d(y, pool.kernel_size, pool.stride, pool.padding)
        bound = F.max_pool2d(bound, pool.kernel_size, pool.stride, pool.padding)
    return y, bound, mean, var


# (N, Cin, H, W, k, pad, pooled): the torchvision stem at the patcher's 224 px, then ragged
# sizes (OH not a multiple of the 4-row tile, OW not a multiple of 16), other channel counts,
# even / odd padding (tap offset 0 / 1), no pooling
CASES = [
    (6, 3, 224, 224, 7, 3, True),
    (3, 3, 30, 50, 7, 3, True),
    (2, 1, 17, 34, 5, 2, True),
    (2, 4, 40, 24, 3, 1, False),
    (1, 3, 12, 8, 7, 3, True),
    (5, 2, 64, 96, 6, 2, False),
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("running", [False, True])
def test_stem_matches_fp64(cuda, case, running):
    from mcgmil.features import stem, stem_fusable
    N, cin, H, W, k, pad, pooled = case
    conv, bn = _stem_layers(cin, k, pad, cuda, N + H + W + k, running)
    pool = nn.MaxPool2d(3, 2, 1) if pooled else None
    g = torch.Generator(device=cuda).manual_seed(H * W + cin)
    x = (torch.randn(N, cin, H, W, device=cuda, generator=g) * 1.3 + 0.2).bfloat16()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        assert stem_fusable(conv, bn, pool, x)
        y = stem(conv, bn, True, pool, x)
    ref, bound, _, _ = _reference(x, conv, bn, pool, running)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    assert y.shape == ref.shape, (y.shape, ref.shape)
    err = (y.double() - ref).abs()
    assert torch.all(err <= bound), float((err - bound).max())


def test_stem_batch_statistics_and_determinism(cuda):
    """The statistics the BN used (batch_mean / batch_invstd through the C ABI) match fp64 over
    the fp32-accumulated rounded activation, and two runs are bitwise equal."""
    import ctypes
    from mcgmil import _lib
    from mcgmil.features import packed_stem_weight, _stem_args
    conv, bn = _stem_layers(3, 7, 3, cuda, 1)
    g = torch.Generator(device=cuda).manual_seed(9)
    x = (torch.randn(8, 3, 224, 224, device=cuda, generator=g) + 3.0).bfloat16()   # mean >> std
    L = _lib.load()
    outs = []
    for _ in range(2):
        a = _stem_args(conv, x)
        a.pool_kernel, a.pool_stride, a.pool_pad, a.relu, a.eps = 3, 2, 1, 1, bn.eps
        w = packed_stem_weight(conv, x)
        y = torch.empty((8, 64, 56, 56), dtype=torch.bfloat16, device=cuda, memory_format=torch.channels_last)
        mean = torch.empty(64, device=cuda)
        inv = torch.empty(64, device=cuda)
        gamma, beta = bn.weight.detach().float().contiguous(), bn.bias.detach().float().contiguous()
        a.x, a.w, a.y = x.data_ptr(), w.data_ptr(), y.data_ptr()
        a.gamma, a.beta = gamma.data_ptr(), beta.data_ptr()
        a.batch_mean, a.batch_invstd = mean.data_ptr(), inv.data_ptr()
        n = ctypes.c_size_t()
        _lib.check(L.mcgmil_stem_workspace_size(ctypes.byref(a), ctypes.byref(n)), "ws")
        ws = torch.empty(n.value, dtype=torch.uint8, device=cuda)
        a.workspace, a.workspace_bytes = ws.data_ptr(), n.value
        _lib.check(L.mcgmil_stem_forward(ctypes.byref(a), torch.cuda.current_stream().cuda_stream), "stem")
        torch.cuda.synchronize()
        outs.append((y.clone(), mean.clone(), inv.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    _, _, rmean, rvar = _reference(x, conv, bn, None, False)
    m, iv = outs[0][1].double(), outs[0][2].double()
    std = torch.sqrt(rvar)
    assert torch.all((m - rmean).abs() <= 2e-3 * std + 2.0 ** -8 * rmean.abs() * 1e-2), float((m - rmean).abs().max())
    assert torch.all((iv * torch.sqrt(rvar + bn.eps) - 1.0).abs() <= 5e-3)


def test_stem_fusable_gates(cuda):
    """Where the torch layers stay: CPU, fp32 without autocast, 5+ channels, stride 1, odd width,
    autograd, BN that would update running statistics, a non-max pool."""
    from mcgmil.features import stem_fusable
    conv, bn = _stem_layers(3, 7, 3, cuda, 2)
    pool = nn.MaxPool2d(3, 2, 1)
    x = torch.randn(2, 3, 32, 32, device=cuda).bfloat16()
    with torch.no_grad():
        assert stem_fusable(conv, bn, pool, x)
        assert stem_fusable(conv, bn, None, x)
        assert not stem_fusable(conv, bn, nn.AvgPool2d(2), x)
        assert not stem_fusable(conv, bn, pool, x[..., :31])                       # odd width
        assert not stem_fusable(conv, bn, pool, x.float())                         # fp32, no autocast
        with torch.autocast("cuda", dtype=torch.bfloat16):
            assert stem_fusable(conv, bn, pool, x.float())
        c5, b5 = _stem_layers(5, 7, 3, cuda, 3)
        assert not stem_fusable(c5, b5, pool, torch.randn(1, 5, 32, 32, device=cuda).bfloat16())
        c1 = nn.Conv2d(3, 64, 7, 1, 3, bias=False).to(cuda)
        assert not stem_fusable(c1, bn, pool, x)                                   # stride 1
        assert not stem_fusable(conv.cpu(), bn.cpu(), pool, x.cpu())
        conv.to(cuda), bn.to(cuda)
        bt = nn.BatchNorm2d(64).to(cuda).train()
        assert not stem_fusable(conv, bt, pool, x)                                 # running-stat update
    assert not stem_fusable(conv, bn, pool, x)                                     # autograd


@pytest.mark.parametrize("shape", [(6, 3, 224, 224), (1, 3, 12, 8), (2, 3, 40, 64), (2, 3, 36, 44)])
@pytest.mark.parametrize("running", [False, True])
def test_stem_row_pooled_epilogue_bitwise(cuda, shape, running):
    """The 3 x 3 / 2 pool split into a horizontal half in the convolution epilogue and a vertical
    pass (negated channels where gamma < 0, zero gammas included) equals the unsplit pooling pass
    bit for bit (mcgmil_stem_args.flags = MCGMIL_STEM_POOL_UNSPLIT); full and partial 16-pixel
    fragments."""
    from mcgmil import _lib
    from mcgmil.features import stem
    N, C, H, W = shape
    conv, bn = _stem_layers(C, 7, 3, cuda, H + W, running)
    with torch.no_grad():
        bn.weight[3] = 0.0
        bn.weight[11] = -0.0
    pool = nn.MaxPool2d(3, 2, 1)
    g = torch.Generator(device=cuda).manual_seed(N + H)
    x = (torch.randn(N, C, H, W, device=cuda, generator=g) * 1.5).bfloat16()
    outs = {}
    for flag in (0, _lib.STEM_POOL_UNSPLIT):
        with torch.no_grad():
            outs[flag] = stem(conv, bn, True, pool, x, flags=flag)
    assert torch.equal(outs[0], outs[_lib.STEM_POOL_UNSPLIT])
