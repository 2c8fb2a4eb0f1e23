"""GPU parity of the fused backbone BatchNorm (include/mcgmil_features.h) against torch's own
batch_norm -- the layer the reference runs (BatchNorm2d on the bag's batch statistics after
deactivate_batchnorm, infer.py:105-109) -- and of the whole ResNet backbone with and without it.

Tolerances: the fused layer computes y = x * a_c + b_c (+ residual) in fp32 from fp64-combined
statistics and rounds once; against an fp64 evaluation of the same formula that is
|dy| <= 2^-8 |y| + 1e-6 for bf16 outputs (half an ulp + the fp32 path) and 2e-6 |y| + 1e-6 for
fp32. The fp32 backbone matches the torch layers to nrel 1e-4; under bf16 autocast both paths
drift from the fp32 features and the fused one must drift no more than the torch layers.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(x, bn, relu, res, batch):
    xd = x.double()
    if batch:
        y = F.batch_norm(xd, None, None, bn.weight.double(), bn.bias.double(), True, 0.0, bn.eps)
    else:
        y = F.batch_norm(xd, bn.running_mean.double(), bn.running_var.double(), bn.weight.double(),
                         bn.bias.double(), False, 0.0, bn.eps)
    if res is not None:
        y = y + res.double()
    return torch.relu(y) if relu else y


def _bn(C, dev, seed):
    g = torch.Generator().manual_seed(seed)
    bn = nn.BatchNorm2d(C)
    with torch.no_grad():
        bn.weight.copy_(torch.randn(C, generator=g) * 0.5 + 1.0)
        bn.weight[::7] *= -1.0                      # negative scales too
        bn.bias.copy_(torch.randn(C, generator=g) * 0.3)
        bn.running_mean.copy_(torch.randn(C, generator=g))
        bn.running_var.copy_(torch.rand(C, generator=g) + 0.5)
    return bn.to(dev)


SHAPES = [(4, 64, 56, 56), (3, 128, 28, 28), (2, 512, 7, 7), (5, 8, 3, 5), (1, 2048, 2, 3)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", SHAPES)
def test_bn_act_matches_torch_batch_stats(cuda, shape, dtype):
    from mcgmil.features import batchnorm_act
    N, C, H, W = shape
    g = torch.Generator(device=cuda).manual_seed(N * C + H)
    bn = _bn(C, cuda, C)
    from mcgmil.resnet import deactivate_batchnorm
    deactivate_batchnorm(bn)
    bn.eval()
    # a large common offset per channel: the shifted statistics must not cancel
    x = (torch.randn(shape, device=cuda, generator=g) * 2 + 30).to(dtype)
    x = x.contiguous(memory_format=torch.channels_last)
    res = torch.randn(shape, device=cuda, generator=g).to(dtype).contiguous(memory_format=torch.channels_last)
    tol_r = 2.0 ** -8 if dtype == torch.bfloat16 else 2e-6
    with torch.no_grad():
        for relu in (False, True):
            for r in (None, res):
                y = batchnorm_act(x, bn, relu, r)
                assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
                ref = _ref(x, bn, relu, r, True)
                err = (y.double() - ref).abs()
                assert torch.all(err <= tol_r * ref.abs() + 1e-5), float(err.max())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_bn_act_running_stats(cuda, dtype):
    """A BN that keeps running statistics (no deactivate_batchnorm) in eval mode uses them."""
    from mcgmil.features import batchnorm_act, fusable
    bn = _bn(64, cuda, 3).eval()
    x = torch.randn(2, 64, 9, 11, device=cuda).to(dtype).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        assert fusable(x, bn)
        y = batchnorm_act(x, bn, True)
        ref = _ref(x, bn, True, None, False)
    tol_r = 2.0 ** -8 if dtype == torch.bfloat16 else 2e-6
    assert torch.all((y.double() - ref).abs() <= tol_r * ref.abs() + 1e-5)


def test_bn_act_many_rows_deterministic(cuda):
    """1.2M rows (the 1024-workgroup statistics path): matches torch and is bitwise repeatable."""
    from mcgmil.features import batchnorm_act
    from mcgmil.resnet import deactivate_batchnorm
    bn = _bn(64, cuda, 9)
    deactivate_batchnorm(bn)
    x = torch.randn(96, 64, 112, 112, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y1 = batchnorm_act(x, bn, True)
        y2 = batchnorm_act(x, bn, True)
        ref = _ref(x, bn, True, None, True)
    assert torch.equal(y1, y2)
    assert torch.all((y1.double() - ref).abs() <= 2.0 ** -8 * ref.abs() + 1e-5)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape,kpd", [((3, 64, 112, 112), (3, 2, 1)), ((2, 64, 7, 9), (3, 2, 1)),
                                       ((2, 16, 8, 6), (2, 2, 0)), ((1, 32, 5, 5), (3, 1, 1))])
def test_bn_act_maxpool_matches_torch(cuda, shape, kpd, dtype):
    """The stem: maxpool(relu(bn(x))) fused equals torch's pooling of the rounded activations."""
    from mcgmil.features import batchnorm_act
    from mcgmil.resnet import deactivate_batchnorm
    k, st, pd = kpd
    bn = _bn(shape[1], cuda, 11)
    deactivate_batchnorm(bn)
    pool = nn.MaxPool2d(k, st, pd)
    x = torch.randn(shape, device=cuda).to(dtype).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y = batchnorm_act(x, bn, True, pool=pool)
        act = batchnorm_act(x, bn, True)
        ref = F.max_pool2d(act, k, st, pd)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(y, ref)


def test_fusable_gates(cuda):
    """Where the torch layers stay: CPU, channels-first, odd C, autograd, running-stat updates."""
    from mcgmil.features import fusable
    bn = _bn(64, cuda, 1)
    x = torch.randn(2, 64, 4, 4, device=cuda).contiguous(memory_format=torch.channels_last)
    bn.eval()
    with torch.no_grad():
        assert fusable(x, bn)
        assert not fusable(x.cpu(), bn)
        assert not fusable(x.contiguous(), bn)                                 # NCHW
        assert not fusable(x.half(), bn)
        bn.train()
        assert not fusable(x, bn)                                              # would update stats
    bn.eval()
    assert not fusable(x, bn)                                                  # grad enabled, params need grad


def _backbone_features(cuda, fused, dtype):
    from mcgmil.resnet import build_backbone, deactivate_batchnorm, Identity
    os.environ["MCGMIL_FUSED_BN"] = "1" if fused else "0"
    os.environ["MCGMIL_NATIVE_CONV"] = "1" if fused else "0"
    os.environ["MCGMIL_NATIVE_STEM"] = "1" if fused else "0"
    try:
        torch.manual_seed(0)
        net = build_backbone("r18", pretrained=False)
        net.fc = Identity()
        net.apply(deactivate_batchnorm)
        net = net.to(cuda).eval().to(memory_format=torch.channels_last)
        g = torch.Generator(device=cuda).manual_seed(5)
        x = torch.rand(12, 3, 96, 96, device=cuda, generator=g)
        x = ((x - 0.45) / 0.25).contiguous(memory_format=torch.channels_last)
        with torch.no_grad():
            if dtype == torch.bfloat16:
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    return net(x).float()
            return net(x)
    finally:
        os.environ.pop("MCGMIL_FUSED_BN", None)
        os.environ.pop("MCGMIL_NATIVE_CONV", None)
        os.environ.pop("MCGMIL_NATIVE_STEM", None)


def test_backbone_fused_bn_matches_torch_layers(cuda):
    """fp32: the fused backbone equals the torch layers to 1e-4 nrel. bf16 autocast: both paths
    drift from the fp32 features through 17 bf16 convolutions; the fused one (implicit-GEMM
    convolutions, one rounding per BN layer, fp64-combined statistics) must be no further from
    them than the torch layers are."""
    ref = _backbone_features(cuda, False, torch.float32)
    f32 = _backbone_features(cuda, True, torch.float32)
    nrel = lambda a, b: float((a - b).abs().max() / b.abs().max())  # noqa: E731
    assert nrel(f32, ref) <= 1e-4, nrel(f32, ref)
    fused = _backbone_features(cuda, True, torch.bfloat16)
    torch_bf16 = _backbone_features(cuda, False, torch.bfloat16)
    d_fused, d_torch = nrel(fused, ref), nrel(torch_bf16, ref)
    print(f"bf16 drift vs fp32: fused {d_fused:.4f}, torch layers {d_torch:.4f}")
    assert d_fused <= 1.25 * d_torch + 1e-3, (d_fused, d_torch)
    assert np.isfinite(fused.cpu().numpy()).all()
