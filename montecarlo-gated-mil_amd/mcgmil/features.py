"""Fused BatchNorm + residual add + ReLU of the channels-last backbone on the GPU
(include/mcgmil_features.h, mcgmil_batchnorm_act).

The reference runs its ResNet's BatchNorm2d layers on the statistics of the bag itself
(infer.py:105-109 deactivate_batchnorm: running stats None, so torch.nn.functional.batch_norm
normalises with the batch mean and biased variance in eval mode too). `batchnorm_act` computes
exactly that layer -- plus the residual add and ReLU that follow it in BasicBlock / Bottleneck --
in three HBM-bound HIP kernels instead of MIOpen's training-mode BN and PyTorch's separate add and
clamp kernels. Layers that keep running statistics (no deactivate_batchnorm, eval mode) are
normalised with them.

`fusable` tells the backbone when the fused path applies: a CUDA(HIP) channels-last bf16/fp32
activation with C % 8 == 0 and C <= 2048, no autograd, and no running-statistics update pending
(a BN in training mode that tracks running stats keeps the torch path, which updates them).
MCGMIL_FUSED_BN=0 switches the backbone back to the torch layers (A/B timing and parity tests).
"""
import ctypes
import os
from typing import Optional

import torch
import torch.nn as nn

from . import _lib

_DT = {torch.float32: _lib.MCGMIL_F32, torch.bfloat16: _lib.MCGMIL_BF16}


def enabled() -> bool:
    return os.environ.get("MCGMIL_FUSED_BN", "1") != "0"


def fusable(x: torch.Tensor, bn: nn.BatchNorm2d, residual: Optional[torch.Tensor] = None) -> bool:
    if not (enabled() and x.is_cuda and x.dim() == 4 and x.dtype in _DT):
        return False
    C = x.shape[1]
    if C % 8 or C > 2048 or C != bn.num_features or x.numel() == 0:
        return False
    if not x.is_contiguous(memory_format=torch.channels_last):
        return False
    if residual is not None and (residual.shape != x.shape or residual.dtype != x.dtype or
                                 not residual.is_contiguous(memory_format=torch.channels_last)):
        return False
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in bn.parameters())):
        return False
    if bn.training and bn.track_running_stats and bn.running_mean is not None:
        return False                       # torch would update the running statistics
    return True


def _f32(t: Optional[torch.Tensor], dev) -> Optional[torch.Tensor]:
    if t is None:
        return None
    t = t.detach()
    if t.dtype != torch.float32 or t.device != dev or not t.is_contiguous():
        t = t.to(device=dev, dtype=torch.float32).contiguous()
    return t


def _pool_params(pool) -> Optional[tuple]:
    """(k, stride, pad) of a plain square nn.MaxPool2d the kernel can fuse, else None."""
    if not isinstance(pool, nn.MaxPool2d) or pool.ceil_mode or pool.return_indices:
        return None
    sq = lambda v: v if isinstance(v, int) else (v[0] if len(set(v)) == 1 else None)  # noqa: E731
    k, st = sq(pool.kernel_size), sq(pool.stride if pool.stride is not None else pool.kernel_size)
    pd, dil = sq(pool.padding), sq(pool.dilation)
    if None in (k, st, pd, dil) or dil != 1 or k < 1 or st < 1 or pd < 0 or 2 * pd > k:
        return None
    return k, st, pd


def batchnorm_act(x: torch.Tensor, bn: nn.BatchNorm2d, relu: bool,
                  residual: Optional[torch.Tensor] = None,
                  pool: Optional[nn.MaxPool2d] = None) -> torch.Tensor:
    """relu?(bn(x) [+ residual]) for a channels-last [N, C, H, W] activation (see fusable), or
    pool(relu?(bn(x))) with a fusable max-pool (the ResNet stem) without materialising the
    activation."""
    if not fusable(x, bn, residual):
        raise ValueError("batchnorm_act needs a CUDA channels-last bf16/fp32 activation with "
                         "C % 8 == 0, C <= 2048 and no autograd (see mcgmil.features.fusable)")
    pp = None
    if pool is not None:
        pp = _pool_params(pool)
        if pp is None or residual is not None:
            raise ValueError("only a square nn.MaxPool2d (dilation 1, floor mode), without a "
                             "residual, is fused")
    L = _lib.load()
    dev = x.device
    N, C, H, W = x.shape
    use_batch = bn.training or bn.running_mean is None or bn.running_var is None
    gamma = _f32(bn.weight, dev) if bn.affine else None
    beta = _f32(bn.bias, dev) if bn.affine else None
    rmean = None if use_batch else _f32(bn.running_mean, dev)
    rvar = None if use_batch else _f32(bn.running_var, dev)
    a = _lib.BnArgs()
    a.rows, a.channels, a.dtype = N * H * W, C, _DT[x.dtype]
    a.batch, a.height, a.width = N, H, W
    if pp is None:
        y = torch.empty_like(x, memory_format=torch.channels_last)
    else:
        k, st, pd = pp
        Ho, Wo = (H + 2 * pd - k) // st + 1, (W + 2 * pd - k) // st + 1
        y = torch.empty((N, C, Ho, Wo), dtype=x.dtype, device=dev, memory_format=torch.channels_last)
        a.pool_kernel, a.pool_stride, a.pool_pad = k, st, pd
    p = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    a.x, a.y, a.residual = p(x), p(y), p(residual)
    a.gamma, a.beta, a.running_mean, a.running_var = p(gamma), p(beta), p(rmean), p(rvar)
    a.eps, a.relu = float(bn.eps), int(bool(relu))
    n = ctypes.c_size_t()
    _lib.check(L.mcgmil_bn_workspace_size(ctypes.byref(a), ctypes.byref(n)), "mcgmil_bn_workspace_size")
    ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
    a.workspace, a.workspace_bytes = p(ws), n.value
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(L.mcgmil_batchnorm_act(ctypes.byref(a), stream), "mcgmil_batchnorm_act")
    return y


def bn_act(bn: nn.BatchNorm2d, x: torch.Tensor, relu: bool,
           residual: Optional[torch.Tensor] = None, pool: Optional[nn.Module] = None) -> torch.Tensor:
    """The backbone's `pool?(relu?(bn(x) [+ residual]))`: fused on the GPU when `fusable`, else
    the torch layers (CPU, autograd, training with running-stat updates, odd layouts)."""
    if fusable(x, bn, residual):
        if pool is None or (residual is None and _pool_params(pool) is not None):
            return batchnorm_act(x, bn, relu, residual, pool)
        return pool(batchnorm_act(x, bn, relu, residual))
    y = bn(x)
    if residual is not None:
        y = y + residual
    y = torch.relu(y) if relu else y
    return y if pool is None else pool(y)
