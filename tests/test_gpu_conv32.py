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
