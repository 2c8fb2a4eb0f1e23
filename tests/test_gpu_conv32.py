"""GPU parity of the fp32 backbone convolution (include/mcgmil_features.h, mcgmil_conv2d_f32) --
the reference's ResNet convolutions (model.py:166-177) at the reference precision, fp32 operands
and fp32 accumulation, as config 5's fp32 line runs them on every instance of a bag.

Reference: an fp64 convolution of the same fp32 input and weight. Bound: |y - ref| <=
2e-6 |ref| + 1e-5 * conv(|x|, |w|) (fp32 rounding of each product and of sums of up to 4,608
terms, in the kernel's order), and nrel <= 1e-5 over the tensor. MIOpen's fp32 convolution of the
same input is held to the same bound, so both are compared on equal terms."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# (N, Cin, H, W, Cout, k, stride, pad): ResNet-18's block convolutions, then odd sizes (pixel
# counts that are not a multiple of the 128 / 256-pixel tile, Cin = 16 and 48, 192 output
# channels = 128 + 64, 5x5 and 7x7 windows, stride 3)
SHAPES = [
    (3, 64, 56, 56, 64, 3, 1, 1),
    (2, 64, 56, 56, 128, 3, 2, 1),
    (2, 64, 56, 56, 128, 1, 2, 0),
    (3, 128, 28, 28, 128, 3, 1, 1),
    (2, 128, 28, 28, 256, 3, 2, 1),
    (2, 256, 14, 14, 512, 3, 2, 1),
    (2, 512, 7, 7, 512, 3, 1, 1),
    (5, 64, 9, 11, 192, 3, 1, 1),
    (2, 16, 10, 10, 64, 5, 1, 2),
    (1, 48, 8, 13, 128, 7, 3, 3),
    (7, 32, 3, 5, 64, 1, 1, 0),
    # gather mode (in_channels not a multiple of 16): the ResNet stem (7x7/2 from 3 channels, K =
    # 147 padded to 160), an odd 5x5 from 5 channels, 1x1 from 24 channels
    (3, 3, 64, 52, 64, 7, 2, 3),
    (2, 5, 17, 9, 128, 5, 1, 2),
    (4, 24, 6, 7, 64, 1, 1, 0),
]


def _layer(cin, cout, k, s, p, dev, seed):
    g = torch.Generator().manual_seed(seed)
    conv = nn.Conv2d(cin, cout, k, s, p, bias=False)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * (2.0 / (cin * k * k)) ** 0.5)
    return conv.to(dev).eval()


def _check(y, x, conv):
    x64, w64 = x.double(), conv.weight.double()
    ref = F.conv2d(x64, w64, stride=conv.stride, padding=conv.padding)
    mag = F.conv2d(x64.abs(), w64.abs(), stride=conv.stride, padding=conv.padding)
    err = (y.double() - ref).abs()
    assert bool((err <= 2e-6 * ref.abs() + 1e-5 * mag + 1e-30).all()), float((err - 2e-6 * ref.abs() - 1e-5 * mag).max())
    nrel = float(err.max() / ref.abs().max())
    assert nrel <= 1e-5, nrel
    return nrel


@pytest.mark.parametrize("shape", SHAPES)
def test_conv2d_f32_matches_fp64(cuda, shape):
    from mcgmil.features import conv2d_f32, conv32_fusable
    N, Cin, H, W, Cout, k, s, p = shape
    conv = _layer(Cin, Cout, k, s, p, cuda, Cin + Cout + k)
    g = torch.Generator(device=cuda).manual_seed(N * H + W)
    x = torch.randn(N, Cin, H, W, device=cuda, generator=g)
    x = x.contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        assert conv32_fusable(conv, x)
        y = conv2d_f32(conv, x)
        torch.cuda.synchronize()
        assert y.is_contiguous(memory_format=torch.channels_last) and y.dtype == torch.float32
        _check(y, x, conv)
        _check(conv(x), x, conv)                   # MIOpen's fp32 convolution, the same bound
        # repeatable: the same bits from a second launch
        assert torch.equal(conv2d_f32(conv, x), y)


def test_conv32_gates_and_repack(cuda):
    """Where the torch layer stays (bf16 / autocast, NCHW, odd channel counts, bias, autograd), and
    a changed weight is repacked."""
    from mcgmil.features import conv2d_f32, conv32_fusable, run_conv
    import os
    conv = _layer(64, 64, 3, 1, 1, cuda, 3)
    x = torch.randn(2, 64, 12, 12, device=cuda).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        assert conv32_fusable(conv, x)
        assert not conv32_fusable(conv, x.contiguous())                       # NCHW
        assert not conv32_fusable(conv, x.bfloat16())
        with torch.autocast("cuda", dtype=torch.bfloat16):
            assert not conv32_fusable(conv, x)
        odd = _layer(64, 96, 3, 1, 1, cuda, 4)
        assert not conv32_fusable(odd, x)                                     # 96 % 64
        x72 = torch.randn(2, 72, 12, 12, device=cuda).contiguous(memory_format=torch.channels_last)
        assert not conv32_fusable(_layer(72, 64, 5, 1, 2, cuda, 5), x72)     # 5*5*72 > 1024, 72 % 16
        biased = nn.Conv2d(64, 64, 3, 1, 1, bias=True).to(cuda)
        assert not conv32_fusable(biased, x)
        os.environ["MCGMIL_NATIVE_CONV32"] = "0"
        try:
            assert not conv32_fusable(conv, x)
            ref = run_conv(conv, x)                                           # the torch layer
        finally:
            os.environ.pop("MCGMIL_NATIVE_CONV32", None)
        y = run_conv(conv, x)
        assert (y - ref).abs().max() <= 1e-5 * ref.abs().max()
        conv.weight.mul_(2.0)                                                 # in-place change: repack
        y2 = conv2d_f32(conv, x)
        assert torch.allclose(y2, 2 * y, rtol=1e-6, atol=1e-6)
    assert not conv32_fusable(conv, x)                                        # grad enabled, weight needs grad


def _combine(part):
    """fp64 Chan combination of [parts, 3, C] (count, mean, M2) blocks -> (count, mean, var)."""
    p = part.double()
    n, m, M2 = p[:, 0], p[:, 1], p[:, 2]
    N = n.sum(0)
    mean = (n * m).sum(0) / N
    var = (M2 + n * (m - mean) ** 2).sum(0) / N
    return N, mean, var


# (N, Cin, H, W, Cout, k, stride, pad): both tile shapes (Cout 64: 64 x 256, else 128 x 128), a
# last pixel tile that is partly empty, the gather-mode stem, a 1x1 stride-2 downsample
STATS_SHAPES = [
    (1, 64, 3, 3, 64, 3, 1, 1),          # 9 pixels: three of the tile's four waves have none
    (3, 64, 20, 20, 64, 3, 1, 1),
    (2, 64, 17, 13, 128, 3, 2, 1),
    (2, 3, 40, 36, 64, 7, 2, 3),
    (3, 128, 9, 9, 256, 1, 2, 0),
]


@pytest.mark.parametrize("shape", STATS_SHAPES)
def test_conv2d_f32_stats(cuda, shape):
    """The epilogue's (count, mean, M2) blocks combine to the fp64 mean / variance of the fp32
    outputs themselves, over every output pixel; y is unchanged by computing them."""
    from mcgmil.features import conv2d_f32
    N, Cin, H, W, Cout, k, s, p = shape
    conv = _layer(Cin, Cout, k, s, p, cuda, 11 + Cin)
    x = torch.randn(N, Cin, H, W, device=cuda, generator=torch.Generator(device=cuda).manual_seed(H))
    x = x.contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y, part = conv2d_f32(conv, x, stats=True)
        torch.cuda.synchronize()
        assert torch.equal(y, conv2d_f32(conv, x))
    cnt, mean, var = _combine(part)
    yd = y.double().permute(0, 2, 3, 1).reshape(-1, Cout)
    assert bool((cnt == yd.shape[0]).all())
    rmean, rvar = yd.mean(0), yd.var(0, unbiased=False)
    scale = rvar.sqrt() + rmean.abs()
    assert float(((mean - rmean).abs() / scale).max()) <= 1e-6
    assert float(((var - rvar).abs() / rvar).max()) <= 1e-5


@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("shape", [(3, 64, 15, 11, 64, 3, 1, 1), (2, 128, 9, 9, 256, 3, 2, 1),
                                   (2, 64, 12, 12, 128, 1, 2, 0)])
def test_conv2d_f32_input_bn_bitwise(cuda, shape, relu):
    """conv(relu?(bn(x))) with the BatchNorm applied while staging (in_ab) is bit-identical to
    mcgmil_batchnorm_act followed by the plain convolution -- padding stays zero."""
    from mcgmil.features import batchnorm_act, batchnorm_coefficients, conv2d_f32, conv32_input_bn
    N, Cin, H, W, Cout, k, s, p = shape
    conv = _layer(Cin, Cout, k, s, p, cuda, 5 + Cout)
    g = torch.Generator(device=cuda).manual_seed(N + W)
    x = (torch.randn(N, Cin, H, W, device=cuda, generator=g) * 3 + 1).contiguous(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(Cin).to(cuda)
    with torch.no_grad():
        bn.weight.copy_(torch.randn(Cin, device=cuda, generator=g))
        bn.bias.copy_(torch.randn(Cin, device=cuda, generator=g))
    bn.eval()
    bn.running_mean, bn.running_var = None, None          # batch statistics, as the reference
    bn.track_running_stats = False
    with torch.no_grad():
        assert conv32_input_bn(conv, x)
        ab = batchnorm_coefficients(x, bn)
        y_in = conv2d_f32(conv, x, in_ab=ab, in_relu=relu)
        y_ref = conv2d_f32(conv, batchnorm_act(x, bn, relu))
        torch.cuda.synchronize()
    assert torch.equal(y_in, y_ref)


def test_bn_many_partials(cuda):
    """More than 1024 statistics blocks (an fp32 layer-1 convolution's one block per 256-pixel
    tile) are combined in chunks first: the result matches a statistics pass over y, through
    both mcgmil_batchnorm_act and mcgmil_batchnorm_coefficients."""
    from mcgmil.features import batchnorm_act, batchnorm_coefficients, conv2d_f32
    conv = _layer(64, 64, 3, 1, 1, cuda, 21)
    x = torch.randn(90, 64, 56, 56, device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
    x = x.contiguous(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(64, track_running_stats=False).to(cuda).eval()
    with torch.no_grad():
        y, part = conv2d_f32(conv, x, stats=True)
        assert part.shape[0] > 1024
        a1 = batchnorm_act(y, bn, True, partials=part)
        a2 = batchnorm_act(y, bn, True)
        c1 = batchnorm_coefficients(y, bn, part)
        c2 = batchnorm_coefficients(y, bn)
        torch.cuda.synchronize()
    assert float((a1 - a2).abs().max()) <= 1e-5 * float(a2.abs().max())
    assert float(((c1 - c2).abs() / c2.abs().clamp_min(1e-3)).max()) <= 1e-5


def test_backbone_f32_input_bn_bitwise(cuda):
    """The fp32 backbone with the BatchNorms folded into the next convolution (and the downsample
    BN into the residual add) is bit-identical to the one that materialises every BN output."""
    from mcgmil.resnet import build_backbone, deactivate_batchnorm, Identity
    import os
    outs = []
    for fold in ("1", "0"):
        os.environ["MCGMIL_FUSE_INPUT_BN"] = fold
        try:
            torch.manual_seed(0)
            net = build_backbone("r18", pretrained=False)
            net.fc = Identity()
            net.apply(deactivate_batchnorm)
            net = net.to(cuda).eval().to(memory_format=torch.channels_last)
            x = torch.rand(6, 3, 80, 80, device=cuda, generator=torch.Generator(device=cuda).manual_seed(1))
            with torch.no_grad():
                outs.append(net(x.contiguous(memory_format=torch.channels_last)))
            torch.cuda.synchronize()
        finally:
            os.environ.pop("MCGMIL_FUSE_INPUT_BN", None)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("parts", [1, 1024, 1025, 3000])
def test_bn_partials_combination(cuda, parts):
    """(count, mean, M2) blocks -> BatchNorm coefficients, directly (<= 1024 blocks) or through the
    chunked pre-combination (more): a_c, b_c match the fp64 combination of the same blocks."""
    from mcgmil.features import batchnorm_coefficients
    C = 64
    g = torch.Generator(device=cuda).manual_seed(parts)
    cnt = torch.randint(1, 300, (parts, 1), device=cuda, generator=g).float().expand(parts, C)
    mean = torch.randn(parts, C, device=cuda, generator=g) * 0.5 + 3.0
    M2 = (torch.rand(parts, C, device=cuda, generator=g) + 0.1) * cnt
    part = torch.stack([cnt, mean, M2], 1).contiguous()
    bn = nn.BatchNorm2d(C, track_running_stats=False).to(cuda).eval()
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, device=cuda, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, device=cuda, generator=g))
    y = torch.zeros(8, C, 1, 1, device=cuda).contiguous(memory_format=torch.channels_last)   # not read
    with torch.no_grad():
        ab = batchnorm_coefficients(y, bn, part).double()
    _, m, var = _combine(part)
    a_ref = bn.weight.detach().double() / torch.sqrt(var + bn.eps)
    b_ref = bn.bias.detach().double() - m * a_ref
    assert float(((ab[0] - a_ref).abs() / a_ref.abs()).max()) <= 2e-6
    assert float((ab[1] - b_ref).abs().max()) <= 2e-6 * float(b_ref.abs().max() + a_ref.abs().max() * m.abs().max())
