"""GPU parity of the implicit-GEMM backbone convolution (include/mcgmil_features.h,
mcgmil_conv2d) -- the reference's torchvision BasicBlock / Bottleneck convolutions
(model.py:166-177) as torch.autocast runs them in bf16 on every instance of a bag
(infer.py:191 -> model.py:275-277).

Reference: an fp64 convolution of the same bf16 input and bf16-rounded weight (what autocast
feeds MIOpen). The kernel accumulates in fp32 and rounds once to bf16, so
|y - ref| <= 2^-8 |ref| (half an ulp) + 1e-5 * conv(|x|, |w|) (fp32 summation of up to 4608
terms, a bound far above its typical size).
"""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# (N, Cin, H, W, Cout, k, stride, pad): ResNet-18's block convolutions at small batch, then odd
# sizes (pixel count not a multiple of the 128-pixel tile, 192 output channels -> 64-wide tiles,
# 5x5 / 7x7 windows, stride 3)
SHAPES = [
    (3, 64, 56, 56, 64, 3, 1, 1),
    (2, 64, 56, 56, 128, 3, 2, 1),
    (2, 64, 56, 56, 128, 1, 2, 0),
    (3, 128, 28, 28, 128, 3, 1, 1),
    (2, 256, 14, 14, 512, 3, 2, 1),
    (2, 512, 7, 7, 512, 3, 1, 1),
    (5, 64, 9, 11, 192, 3, 1, 1),
    (2, 128, 10, 10, 64, 5, 1, 2),
    (1, 64, 8, 13, 64, 7, 3, 3),
    # 3x3 / 64 -> 64 halo-tile kernel: tiles spanning several small images, odd widths, a tile
    # crossing image boundaries, and a width whose patch only just fits (62) or does not (70)
    (9, 64, 8, 6, 64, 3, 1, 1),
    (3, 64, 30, 17, 64, 3, 1, 1),
    (2, 64, 20, 62, 64, 3, 1, 1),
    (1, 64, 5, 70, 64, 3, 1, 1),
]


def _layer(cin, cout, k, s, p, dev, seed):
    g = torch.Generator().manual_seed(seed)
    conv = nn.Conv2d(cin, cout, k, s, p, bias=False)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * (2.0 / (cin * k * k)) ** 0.5)
    return conv.to(dev).eval()


@pytest.mark.parametrize("shape", SHAPES)
def test_conv2d_matches_fp64(cuda, shape):
    from mcgmil.features import conv2d, conv_fusable
    N, Cin, H, W, Cout, k, s, p = shape
    conv = _layer(Cin, Cout, k, s, p, cuda, Cin + Cout + k)
    g = torch.Generator(device=cuda).manual_seed(N * H + W)
    x = torch.randn(N, Cin, H, W, device=cuda, generator=g).relu_().bfloat16()
    x = x.contiguous(memory_format=torch.channels_last)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        assert conv_fusable(conv, x)
        y = conv2d(conv, x)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    wb = conv.weight.detach().bfloat16().double()
    with torch.no_grad():
        ref = F.conv2d(x.double(), wb, None, s, p)
        mag = F.conv2d(x.double().abs(), wb.abs(), None, s, p)
    assert y.shape == ref.shape
    err = (y.double() - ref).abs()
    assert torch.all(err <= 2.0 ** -8 * ref.abs() + 1e-5 * mag), float((err / (ref.abs() + 1e-30)).max())


def test_conv2d_bf16_weights_and_repack(cuda):
    """A bf16 module runs without autocast; an in-place weight update is picked up (the packed
    weight cache is keyed by the tensor version)."""
    from mcgmil.features import conv2d
    conv = _layer(64, 128, 3, 1, 1, cuda, 3).bfloat16()
    x = torch.randn(2, 64, 12, 12, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y1 = conv2d(conv, x)
        ref1 = F.conv2d(x.double(), conv.weight.double(), None, 1, 1)
        conv.weight.mul_(-2.0)
        y2 = conv2d(conv, x)
    assert torch.all((y1.double() - ref1).abs() <= 2.0 ** -8 * ref1.abs() + 1e-3)
    assert torch.equal(y2, (-2.0 * y1.float()).bfloat16())


def test_conv_fusable_gates(cuda):
    """Where torch's convolution stays: CPU, NCHW, fp32 without autocast, the 3-channel stem,
    grouped / biased / dilated convolutions, autograd."""
    from mcgmil.features import conv_fusable
    conv = _layer(64, 64, 3, 1, 1, cuda, 1)
    x = torch.randn(1, 64, 8, 8, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            assert conv_fusable(conv, x)
            assert not conv_fusable(conv, x.contiguous())                          # NCHW
            assert not conv_fusable(conv.cpu(), x.cpu())
            conv.to(cuda)
            assert not conv_fusable(_layer(3, 64, 7, 2, 3, cuda, 2),
                                    torch.randn(1, 3, 32, 32, device=cuda).bfloat16()
                                    .contiguous(memory_format=torch.channels_last))
            assert not conv_fusable(nn.Conv2d(64, 64, 3, 1, 1, groups=2, bias=False).to(cuda), x)
            assert not conv_fusable(nn.Conv2d(64, 64, 3, 1, 1, bias=True).to(cuda), x)
            assert not conv_fusable(nn.Conv2d(64, 64, 3, 1, 2, dilation=2, bias=False).to(cuda), x)
        assert not conv_fusable(conv, x.float().contiguous(memory_format=torch.channels_last))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert not conv_fusable(conv, x)                      # grad enabled, weight needs grad
