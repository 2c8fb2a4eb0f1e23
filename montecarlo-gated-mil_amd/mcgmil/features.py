"""The channels-last backbone's layers on the GPU (include/mcgmil_features.h): fused BatchNorm +
residual add + ReLU (mcgmil_batchnorm_act) and the implicit-GEMM convolution (mcgmil_conv2d).

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

`conv2d` runs a 3x3 / 1x1 torch.nn.Conv2d of the blocks (bias-free, groups 1, dilation 1, zero
padding, 64k input and output channels) on a channels-last bf16 activation as one MFMA
implicit-GEMM kernel -- the arithmetic of torch.autocast's bf16 convolution (bf16 operands, fp32
accumulation, one rounding) without MIOpen's per-convolution output fill. `conv_fusable` says when
it applies. MCGMIL_NATIVE_CONV=0 switches it off.

`stem` runs the torchvision stem maxpool(relu(bn1(conv1(x)))) (7x7/2 convolution of the 3-channel
instances) as one library call (mcgmil_stem_forward): an MFMA implicit GEMM straight from the NCHW
bf16 instances the patcher writes, with the BatchNorm statistics accumulated in its epilogue, then
the fused normalise + ReLU + max-pool pass. `stem_fusable` says when it applies (else the torch
layers run); MCGMIL_NATIVE_STEM=0 switches it off.
"""
import ctypes
import os
from typing import NamedTuple, Optional

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


def conv_enabled() -> bool:
    return os.environ.get("MCGMIL_NATIVE_CONV", "1") != "0"


def _square(v):
    return v if isinstance(v, int) else (v[0] if len(set(v)) == 1 else None)


def conv_fusable(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """A CUDA channels-last activation that torch would convolve in bf16 (bf16 input, or autocast
    to bf16), with a convolution the kernel implements, and no autograd."""
    if not (conv_enabled() and isinstance(conv, nn.Conv2d) and x.is_cuda and x.dim() == 4):
        return False
    if conv.groups != 1 or conv.bias is not None or conv.padding_mode != "zeros":
        return False
    if _square(conv.dilation) != 1 or _square(conv.stride) is None or \
            not isinstance(conv.padding, tuple) or _square(conv.padding) is None:
        return False
    kh, kw = conv.kernel_size
    if not (1 <= kh <= 7 and 1 <= kw <= 7):
        return False
    if conv.in_channels % 64 or conv.out_channels % 64 or x.shape[1] != conv.in_channels:
        return False
    bf16 = x.dtype == torch.bfloat16 and (
        conv.weight.dtype == torch.bfloat16 or
        (torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16))
    if not bf16 or not x.is_contiguous(memory_format=torch.channels_last):
        return False
    if torch.is_grad_enabled() and (x.requires_grad or conv.weight.requires_grad):
        return False
    return x.numel() * 2 < 2 ** 31


def _conv_args(conv: nn.Conv2d, x: torch.Tensor):
    a = _lib.ConvArgs()
    a.batch, _, a.height, a.width = x.shape
    a.in_channels, a.out_channels = conv.in_channels, conv.out_channels
    a.kernel_h, a.kernel_w = conv.kernel_size
    a.stride, a.pad = _square(conv.stride), _square(conv.padding)
    return a


def packed_conv_weight(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """The weight as bf16 [out, kh, kw, in] (torch's autocast cast, then channels-last), cached on
    the module until the weight changes."""
    w = conv.weight.detach()
    key = (w.data_ptr(), w._version, w.dtype, x.device)
    cached = getattr(conv, "_mcgmil_packed", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    L = _lib.load()
    if w.device != x.device or w.dtype not in (torch.float32, torch.bfloat16):
        w = w.to(device=x.device, dtype=torch.float32)
    w = w.contiguous()
    packed = torch.empty(w.numel(), dtype=torch.bfloat16, device=x.device)
    a = _conv_args(conv, x)
    stream = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    _lib.check(L.mcgmil_pack_conv_weights(ctypes.byref(a), ctypes.c_void_p(w.data_ptr()),
                                          _DT[w.dtype], ctypes.c_void_p(packed.data_ptr()), stream),
               "mcgmil_pack_conv_weights")
    conv._mcgmil_packed = (key, packed)
    return packed


def fold_enabled() -> bool:
    """MCGMIL_FUSE_INPUT_BN=0 materialises every BatchNorm output (no DeferredBN)."""
    return os.environ.get("MCGMIL_FUSE_INPUT_BN", "1") != "0"


def conv_input_bn(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """Whether conv2d(conv, x, in_ab=...) can apply an input BatchNorm inside the convolution
    (mcgmil_conv_input_bn: the 3x3 / stride 1 halo kernels); False with MCGMIL_FUSE_INPUT_BN=0."""
    if not fold_enabled():
        return False
    L = _lib.load()
    ok = ctypes.c_int32()
    _lib.check(L.mcgmil_conv_input_bn(ctypes.byref(_conv_args(conv, x)), ctypes.byref(ok)), "mcgmil_conv_input_bn")
    return bool(ok.value)


def split_enabled() -> bool:
    """MCGMIL_CONV_SPLIT=0: no K split of the last pixel tiles (mcgmil_conv_args.workspace NULL)."""
    return os.environ.get("MCGMIL_CONV_SPLIT", "1") != "0"


def conv2d(conv: nn.Conv2d, x: torch.Tensor, stats: bool = False,
           in_ab: Optional[torch.Tensor] = None, in_relu: bool = True, flags: int = 0):
    """conv(x) for a channels-last bf16 activation (see conv_fusable) on the MFMA kernel; returns a
    channels-last bf16 tensor, or with stats=True (y, partials): the BatchNorm statistics of y
    as [parts, 3, Cout] (count, mean, M2) blocks for batchnorm_act(..., partials=...), or None
    where the layer's kernel emits none (256 x 256 tiles). With in_ab ([2, Cin] fp32 from
    batchnorm_coefficients) the convolution reads relu?(bn(x)) instead of x (conv_input_bn).
    flags: mcgmil_conv_args.flags (the tile policy, MCGMIL_CONV_TILE_*; 0 = auto).
    Layers whose plan takes a K split of its last tiles get their workspace from the caching
    allocator (mcgmil_conv_workspace_size); MCGMIL_CONV_SPLIT=0 runs them on whole tiles."""
    if not conv_fusable(conv, x):
        raise ValueError("conv2d needs a CUDA channels-last bf16 activation, a bias-free groups=1 "
                         "convolution with 64k channels and no autograd (see conv_fusable)")
    L = _lib.load()
    a = _conv_args(conv, x)
    a.flags = int(flags)
    if in_ab is not None:
        if in_ab.shape != (2, a.in_channels) or in_ab.dtype != torch.float32 or \
                in_ab.device != x.device or not in_ab.is_contiguous():
            raise ValueError("in_ab must be a contiguous fp32 [2, in_channels] tensor on x's device")
        a.in_ab, a.in_relu = ctypes.c_void_p(in_ab.data_ptr()), int(bool(in_relu))
    oh = (a.height + 2 * a.pad - a.kernel_h) // a.stride + 1
    ow = (a.width + 2 * a.pad - a.kernel_w) // a.stride + 1
    y = torch.empty((a.batch, a.out_channels, oh, ow), dtype=torch.bfloat16, device=x.device,
                    memory_format=torch.channels_last)
    w = packed_conv_weight(conv, x)
    a.x, a.w, a.y = (ctypes.c_void_p(t.data_ptr()) for t in (x, w, y))
    ws = None
    if split_enabled():
        nb = ctypes.c_size_t()
        _lib.check(L.mcgmil_conv_workspace_size(ctypes.byref(a), ctypes.byref(nb)), "mcgmil_conv_workspace_size")
        if nb.value:
            ws = torch.empty(nb.value, dtype=torch.uint8, device=x.device)   # freed after the launch,
            a.workspace, a.workspace_bytes = ctypes.c_void_p(ws.data_ptr()), nb.value   # stream-ordered
    part = None
    if stats:
        n = ctypes.c_int32()
        _lib.check(L.mcgmil_conv_stats_parts(ctypes.byref(a), ctypes.byref(n)), "mcgmil_conv_stats_parts")
        if n.value > 0:          # 0: this layer's kernel emits no statistics
            part = torch.empty((n.value, 3, a.out_channels), dtype=torch.float32, device=x.device)
            a.stats = ctypes.c_void_p(part.data_ptr())
    stream = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    _lib.check(L.mcgmil_conv2d(ctypes.byref(a), stream), "mcgmil_conv2d")
    return (y, part) if stats else y


def conv32_enabled() -> bool:
    """MCGMIL_NATIVE_CONV32=0 keeps fp32 convolutions on the torch layers (MIOpen)."""
    return os.environ.get("MCGMIL_NATIVE_CONV32", "1") != "0" and conv_enabled()


def conv32_fusable(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """A CUDA channels-last fp32 activation (no autocast) and a convolution the fp32 kernel
    implements (mcgmil_conv2d_f32: out_channels % 64, kernel <= 7, and in_channels % 16 or
    kh * kw * in_channels <= 1024 -- the 3-channel stem), no autograd."""
    if not (conv32_enabled() and isinstance(conv, nn.Conv2d) and x.is_cuda and x.dim() == 4):
        return False
    if x.dtype != torch.float32 or torch.is_autocast_enabled("cuda"):
        return False
    if conv.groups != 1 or conv.bias is not None or conv.padding_mode != "zeros":
        return False
    if _square(conv.dilation) != 1 or _square(conv.stride) is None or \
            not isinstance(conv.padding, tuple) or _square(conv.padding) is None:
        return False
    kh, kw = conv.kernel_size
    if not (1 <= kh <= 7 and 1 <= kw <= 7):
        return False
    if conv.out_channels % 64 or x.shape[1] != conv.in_channels:
        return False
    if conv.in_channels % 16 and kh * kw * conv.in_channels > 1024:
        return False
    if not x.is_contiguous(memory_format=torch.channels_last):
        return False
    if torch.is_grad_enabled() and (x.requires_grad or conv.weight.requires_grad):
        return False
    oh = (x.shape[2] + 2 * _square(conv.padding) - kh) // _square(conv.stride) + 1
    ow = (x.shape[3] + 2 * _square(conv.padding) - kw) // _square(conv.stride) + 1
    return x.shape[0] * oh * ow < 2 ** 31 - 256


def packed_conv_weight_f32(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """The fp32 weight in mcgmil_conv2d_f32's packed layout, cached on the module until it changes."""
    w = conv.weight.detach()
    key = (w.data_ptr(), w._version, w.dtype, x.device, "f32")
    cached = getattr(conv, "_mcgmil_packed32", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    L = _lib.load()
    w32 = w.to(device=x.device, dtype=torch.float32).contiguous()
    a = _conv_args(conv, x)
    n = ctypes.c_size_t()
    _lib.check(L.mcgmil_conv_packed_size_f32(ctypes.byref(a), ctypes.byref(n)), "mcgmil_conv_packed_size_f32")
    packed = torch.empty(n.value, dtype=torch.float32, device=x.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    _lib.check(L.mcgmil_pack_conv_weights_f32(ctypes.byref(a), ctypes.c_void_p(w32.data_ptr()),
                                              ctypes.c_void_p(packed.data_ptr()), stream),
               "mcgmil_pack_conv_weights_f32")
    conv._mcgmil_packed32 = (key, packed)
    return packed


def conv32_input_bn(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """Whether conv2d_f32(conv, x, in_ab=...) can apply an input BatchNorm (in_channels a multiple
    of 16, <= 2048: every fp32 kernel but the gather mode); False with MCGMIL_FUSE_INPUT_BN=0."""
    return fold_enabled() and conv32_fusable(conv, x) and conv.in_channels % 16 == 0 and \
        conv.in_channels <= 2048


def conv2d_f32(conv: nn.Conv2d, x: torch.Tensor, stats: bool = False,
               in_ab: Optional[torch.Tensor] = None, in_relu: bool = True):
    """conv(x) in fp32 on the MFMA kernel (fp32 operands and accumulation) for a channels-last fp32
    activation (see conv32_fusable); returns a channels-last fp32 tensor, or with stats=True
    (y, partials): the BatchNorm statistics of y as [pixel tiles, 3, Cout] (count, mean, M2)
    blocks for batchnorm_act(..., partials=...). With in_ab ([2, Cin] fp32 from
    batchnorm_coefficients) the convolution reads relu?(bn(x)) instead of x (conv32_input_bn)."""
    if not conv32_fusable(conv, x):
        raise ValueError("conv2d_f32 needs a CUDA channels-last fp32 activation and a bias-free groups=1 "
                         "convolution with out_channels % 64 == 0 (conv32_fusable)")
    L = _lib.load()
    a = _conv_args(conv, x)
    if in_ab is not None:
        if in_ab.shape != (2, a.in_channels) or in_ab.dtype != torch.float32 or \
                in_ab.device != x.device or not in_ab.is_contiguous():
            raise ValueError("in_ab must be a contiguous fp32 [2, in_channels] tensor on x's device")
        a.in_ab, a.in_relu = ctypes.c_void_p(in_ab.data_ptr()), int(bool(in_relu))
    oh = (a.height + 2 * a.pad - a.kernel_h) // a.stride + 1
    ow = (a.width + 2 * a.pad - a.kernel_w) // a.stride + 1
    y = torch.empty((a.batch, a.out_channels, oh, ow), dtype=torch.float32, device=x.device,
                    memory_format=torch.channels_last)
    w = packed_conv_weight_f32(conv, x)
    a.x, a.w, a.y = (ctypes.c_void_p(t.data_ptr()) for t in (x, w, y))
    part = None
    if stats:
        n = ctypes.c_int32()
        _lib.check(L.mcgmil_conv_stats_parts_f32(ctypes.byref(a), ctypes.byref(n)), "mcgmil_conv_stats_parts_f32")
        part = torch.empty((n.value, 3, a.out_channels), dtype=torch.float32, device=x.device)
        a.stats = ctypes.c_void_p(part.data_ptr())
    stream = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    _lib.check(L.mcgmil_conv2d_f32(ctypes.byref(a), stream), "mcgmil_conv2d_f32")
    return (y, part) if stats else y


def _native_conv(conv: nn.Module, x: torch.Tensor) -> Optional[str]:
    """"bf16" (conv2d), "f32" (conv2d_f32) or None (the torch layer) for conv on x."""
    if isinstance(conv, nn.Conv2d):
        if conv_fusable(conv, x):
            return "bf16"
        if conv32_fusable(conv, x):
            return "f32"
    return None


def _takes_input_bn(conv: nn.Module, x: torch.Tensor) -> bool:
    kind = _native_conv(conv, x)
    return (kind == "bf16" and conv_input_bn(conv, x)) or (kind == "f32" and conv32_input_bn(conv, x))


def torch_conv(layer: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """The torch layer, with fp32 convolutions on the GPU split along the batch so that no call's
    input or output reaches 2^31 bytes (MCGMIL_FP32_CONV_CHUNK=0: unsplit). On some MI355X boxes
    the unsplit fp32 stem convolution of a config-5 bag (1,507 instances: a 4.85 GB output) came
    back wrong from MIOpen -- features nrel 1.68 against the CPU, with this build's kernels off --
    while other boxes matched the CPU to 2e-6 (scripts/probe_cfg5_drift.py)."""
    if not (isinstance(layer, nn.Conv2d) and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
            and x.shape[0] > 1 and os.environ.get("MCGMIL_FP32_CONV_CHUNK", "1") != "0"):
        return layer(x)
    oh = (x.shape[2] + 2 * layer.padding[0] - layer.dilation[0] * (layer.kernel_size[0] - 1) - 1) \
        // layer.stride[0] + 1
    ow = (x.shape[3] + 2 * layer.padding[1] - layer.dilation[1] * (layer.kernel_size[1] - 1) - 1) \
        // layer.stride[1] + 1
    per = 4 * max(x[0].numel(), layer.out_channels * oh * ow)
    n = max(1, ((1 << 31) - 1) // per)
    if n >= x.shape[0]:
        return layer(x)
    mf = torch.channels_last if x.is_contiguous(memory_format=torch.channels_last) else torch.contiguous_format
    return torch.cat([layer(x[i:i + n]) for i in range(0, x.shape[0], n)]).contiguous(memory_format=mf)


def run_conv(layer: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """The backbone's convolution: the bf16 MFMA kernel when `conv_fusable`, the fp32 one when
    `conv32_fusable`, else the torch layer."""
    if isinstance(layer, nn.Conv2d) and conv_fusable(layer, x):
        return conv2d(layer, x)
    if isinstance(layer, nn.Conv2d) and conv32_fusable(layer, x):
        return conv2d_f32(layer, x)
    return torch_conv(layer, x)


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
                  pool: Optional[nn.MaxPool2d] = None,
                  partials: Optional[torch.Tensor] = None,
                  residual_ab: Optional[torch.Tensor] = None) -> torch.Tensor:
    """relu?(bn(x) [+ residual]) for a channels-last [N, C, H, W] activation (see fusable), or
    pool(relu?(bn(x))) with a fusable max-pool (the ResNet stem) without materialising the
    activation. `partials` ([parts, 3, C] from conv2d(..., stats=True)) supplies the batch
    statistics of x, so x is read once. `residual_ab` ([2, C] from batchnorm_coefficients) is the
    residual's own BatchNorm, applied on the fly (bit-identical to normalising it first)."""
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
    if residual_ab is not None:
        if residual is None or residual_ab.shape != (2, C) or residual_ab.dtype != torch.float32 or \
                residual_ab.device != dev or not residual_ab.is_contiguous():
            raise ValueError("residual_ab needs a residual and a contiguous fp32 [2, C] tensor on x's device")
        a.residual_ab = p(residual_ab)
    if partials is not None and use_batch:
        if partials.dim() != 3 or partials.shape[1:] != (3, C) or not partials.is_contiguous() or \
                partials.dtype != torch.float32 or partials.device != dev:
            raise ValueError("partials must be a contiguous fp32 [parts, 3, C] tensor on x's device")
        a.partials, a.num_partials = p(partials), partials.shape[0]
    n = ctypes.c_size_t()
    _lib.check(L.mcgmil_bn_workspace_size(ctypes.byref(a), ctypes.byref(n)), "mcgmil_bn_workspace_size")
    ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
    a.workspace, a.workspace_bytes = p(ws), n.value
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(L.mcgmil_batchnorm_act(ctypes.byref(a), stream), "mcgmil_batchnorm_act")
    return y


def batchnorm_coefficients(x: torch.Tensor, bn: nn.BatchNorm2d,
                           partials: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The [2, C] fp32 (a_c, b_c) that batchnorm_act(x, bn, ...) would apply
    (mcgmil_batchnorm_coefficients), for a consumer that applies them itself (conv2d's in_ab)."""
    if not fusable(x, bn, None):
        raise ValueError("batchnorm_coefficients needs what batchnorm_act needs (see fusable)")
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
    p = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    a.x = p(x)
    a.gamma, a.beta, a.running_mean, a.running_var = p(gamma), p(beta), p(rmean), p(rvar)
    a.eps = float(bn.eps)
    ws = None
    if partials is not None and use_batch:
        if partials.dim() != 3 or partials.shape[1:] != (3, C) or not partials.is_contiguous() or \
                partials.dtype != torch.float32 or partials.device != dev:
            raise ValueError("partials must be a contiguous fp32 [parts, 3, C] tensor on x's device")
        a.partials, a.num_partials = p(partials), partials.shape[0]
    if use_batch:     # the statistics pass, or more than 1024 partials combined in chunks first
        n = ctypes.c_size_t()
        a.y = a.x
        _lib.check(L.mcgmil_bn_workspace_size(ctypes.byref(a), ctypes.byref(n)), "mcgmil_bn_workspace_size")
        ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
        a.workspace, a.workspace_bytes = p(ws), n.value
    ab = torch.empty((2, C), dtype=torch.float32, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(L.mcgmil_batchnorm_coefficients(ctypes.byref(a), p(ab), stream), "mcgmil_batchnorm_coefficients")
    return ab


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


def stem_enabled() -> bool:
    return os.environ.get("MCGMIL_NATIVE_STEM", "1") != "0"


def stem_fusable(conv: nn.Module, bn: nn.Module, pool: Optional[nn.Module], x: torch.Tensor) -> bool:
    """A CUDA [N, C<=4, H, W] activation that torch would convolve in bf16, a bias-free
    Conv2d(C, 64, k, stride 2) with k + (pad & 1) <= 8 and OW <= 125, a BatchNorm2d(64) the fused
    BN handles (see fusable), and a plain max-pool (or none); no autograd."""
    if not (stem_enabled() and isinstance(conv, nn.Conv2d) and isinstance(bn, nn.BatchNorm2d)):
        return False
    if not (x.is_cuda and x.dim() == 4 and x.dtype in _DT and x.numel() > 0):
        return False
    if conv.groups != 1 or conv.bias is not None or conv.padding_mode != "zeros":
        return False
    if _square(conv.dilation) != 1 or _square(conv.stride) != 2 or not isinstance(conv.padding, tuple) \
            or _square(conv.padding) is None or _square(conv.kernel_size) is None:
        return False
    k, pad = conv.kernel_size[0], conv.padding[0]
    N, C, H, W = x.shape
    if C != conv.in_channels or not 1 <= C <= 4 or conv.out_channels != 64 or bn.num_features != 64:
        return False
    if k + (pad & 1) > 8 or W % 2 or H + 2 * pad < k or W + 2 * pad < k or (W + 2 * pad - k) // 2 + 1 > 125:
        return False
    if pool is not None and _pool_params(pool) is None:
        return False
    bf16 = x.dtype == torch.bfloat16 or conv.weight.dtype == torch.bfloat16 or \
        (torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16)
    if not bf16:
        return False
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in conv.parameters())
                                    or any(p.requires_grad for p in bn.parameters())):
        return False
    if bn.training and bn.track_running_stats and bn.running_mean is not None:
        return False
    return True


def _stem_args(conv: nn.Conv2d, x: torch.Tensor) -> "_lib.StemArgs":
    a = _lib.StemArgs()
    a.batch, a.in_channels, a.height, a.width = x.shape
    a.out_channels, a.kernel = conv.out_channels, conv.kernel_size[0]
    a.stride, a.pad = conv.stride[0], conv.padding[0]
    return a


def packed_stem_weight(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """The stem weight in the kernel's MFMA fragment order (bf16), cached on the module and keyed
    by the weight's version."""
    w = conv.weight.detach()
    key = (w.data_ptr(), w._version, w.dtype, x.device)
    cached = getattr(conv, "_mcgmil_stem_packed", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    L = _lib.load()
    a = _stem_args(conv, x)
    n = ctypes.c_size_t()
    _lib.check(L.mcgmil_stem_packed_size(ctypes.byref(a), ctypes.byref(n)), "mcgmil_stem_packed_size")
    wc = w.to(device=x.device).contiguous()
    if wc.dtype not in _DT:
        wc = wc.float()
    packed = torch.empty(n.value, dtype=torch.uint8, device=x.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    _lib.check(L.mcgmil_pack_stem_weights(ctypes.byref(a), ctypes.c_void_p(wc.data_ptr()), _DT[wc.dtype],
                                          ctypes.c_void_p(packed.data_ptr()), stream),
               "mcgmil_pack_stem_weights")
    conv._mcgmil_stem_packed = (key, packed)
    return packed


def stem(conv: nn.Conv2d, bn: nn.BatchNorm2d, relu: bool, pool: Optional[nn.MaxPool2d],
         x: torch.Tensor, flags: int = 0) -> torch.Tensor:
    """pool?(relu?(bn(conv(x)))) of NCHW instances (see stem_fusable) -> channels-last bf16.
    flags: mcgmil_stem_args.flags (MCGMIL_STEM_POOL_UNSPLIT: one pooling pass; 0 = the split)."""
    if not stem_fusable(conv, bn, pool, x):
        raise ValueError("stem needs a CUDA [N, C<=4, H, W] bf16 (or autocast) input, a bias-free "
                         "stride-2 Conv2d(C, 64) with k + (pad & 1) <= 8 and OW <= 125, a "
                         "BatchNorm2d(64) and a square max-pool, without autograd (see stem_fusable)")
    L = _lib.load()
    dev = x.device
    xb = x.to(torch.bfloat16).contiguous()
    a = _stem_args(conv, xb)
    N, _, H, W = xb.shape
    OH = (H + 2 * a.pad - a.kernel) // 2 + 1
    OW = (W + 2 * a.pad - a.kernel) // 2 + 1
    PH, PW = OH, OW
    if pool is not None:
        k, st, pd = _pool_params(pool)
        a.pool_kernel, a.pool_stride, a.pool_pad = k, st, pd
        PH, PW = (OH + 2 * pd - k) // st + 1, (OW + 2 * pd - k) // st + 1
    use_batch = bn.training or bn.running_mean is None or bn.running_var is None
    gamma = _f32(bn.weight, dev) if bn.affine else None
    beta = _f32(bn.bias, dev) if bn.affine else None
    rmean = None if use_batch else _f32(bn.running_mean, dev)
    rvar = None if use_batch else _f32(bn.running_var, dev)
    w = packed_stem_weight(conv, xb)
    y = torch.empty((N, 64, PH, PW), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
    p = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    a.x, a.w, a.y = p(xb), p(w), p(y)
    a.gamma, a.beta, a.running_mean, a.running_var = p(gamma), p(beta), p(rmean), p(rvar)
    a.eps, a.relu = float(bn.eps), int(bool(relu))
    a.flags = int(flags)
    n = ctypes.c_size_t()
    _lib.check(L.mcgmil_stem_workspace_size(ctypes.byref(a), ctypes.byref(n)), "mcgmil_stem_workspace_size")
    ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
    a.workspace, a.workspace_bytes = p(ws), n.value
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(L.mcgmil_stem_forward(ctypes.byref(a), stream), "mcgmil_stem_forward")
    return y


def run_stem(conv: nn.Module, bn: nn.Module, pool: Optional[nn.Module], x: torch.Tensor) -> torch.Tensor:
    """The backbone's stem: the fused kernel when `stem_fusable`, else conv + bn_act (on the GPU
    with a channels-last activation, so the blocks after it stay on the fused path)."""
    if stem_fusable(conv, bn, pool, x):
        return stem(conv, bn, True, pool, x)
    if x.is_cuda and x.dim() == 4:
        x = x.contiguous(memory_format=torch.channels_last)
    if isinstance(conv, nn.Conv2d) and conv32_fusable(conv, x) and isinstance(bn, nn.BatchNorm2d) \
            and _use_batch(bn):
        y, part = conv2d_f32(conv, x, stats=True)    # statistics from the convolution's epilogue
        if fusable(y, bn) and (pool is None or _pool_params(pool) is not None):
            return batchnorm_act(y, bn, True, pool=pool, partials=part)
        return bn_act(bn, y, True, pool=pool)
    return bn_act(bn, run_conv(conv, x), True, pool=pool)


class DeferredBN(NamedTuple):
    """relu?(bn(y)) left unapplied: the next convolution applies it to its input (conv2d's
    in_ab), so the activation is neither written nor read a second time."""
    y: torch.Tensor
    ab: torch.Tensor                    # [2, C] fp32 (a_c, b_c) from batchnorm_coefficients
    relu: bool
    bn: nn.BatchNorm2d
    partials: Optional[torch.Tensor]    # the statistics ab came from (None: running statistics)

    def materialise(self) -> torch.Tensor:
        return batchnorm_act(self.y, self.bn, self.relu, partials=self.partials)


def _use_batch(bn: nn.BatchNorm2d) -> bool:
    return bn.training or bn.running_mean is None or bn.running_var is None


def conv_bn_act(conv: nn.Module, bn: nn.Module, x, relu: bool, residual=None,
                consumer: Optional[nn.Module] = None, as_residual: bool = False):
    """The blocks' `relu?(bn(conv(x)) [+ residual])`: on the GPU the MFMA convolution (bf16 or
    fp32) also emits the BatchNorm batch statistics of its output (when the BN normalises with
    them), and the fused BN consumes them -- the activation is written once and read once. Else
    run_conv + bn_act.
    x may be a DeferredBN (its BN runs inside this convolution). With `consumer` (the convolution
    that reads the result) and no residual, the result may come back as a DeferredBN when that
    convolution can apply the BN itself (conv_input_bn); pass it on to conv_bn_act. With
    as_residual (the downsample branch) a ReLU-free result may come back as a DeferredBN too; pass
    it as conv_bn_act's residual, whose fused BN applies it while adding."""
    res_ab, res_deferred = None, None
    if isinstance(residual, DeferredBN):
        if residual.relu:
            residual = residual.materialise()
        else:
            res_deferred, residual, res_ab = residual, residual.y, residual.ab
    kw = {}
    if isinstance(x, DeferredBN):
        if _takes_input_bn(conv, x.y):
            kw = {"in_ab": x.ab, "in_relu": x.relu}
            x = x.y
        else:
            x = x.materialise()
    kind = _native_conv(conv, x)
    if kind is not None:
        native = conv2d if kind == "bf16" else conv2d_f32
        if isinstance(bn, nn.BatchNorm2d) and _use_batch(bn):
            y, part = native(conv, x, stats=True, **kw)
        else:
            y, part = native(conv, x, **kw), None
        if not (isinstance(bn, nn.BatchNorm2d) and fusable(y, bn, residual)):
            return bn_act(bn, y, relu, res_deferred.materialise() if res_deferred else residual)
        if residual is None and ((isinstance(consumer, nn.Conv2d) and _takes_input_bn(consumer, y))
                                 or (as_residual and not relu and fold_enabled())):
            return DeferredBN(y, batchnorm_coefficients(y, bn, part), relu, bn, part)
        return batchnorm_act(y, bn, relu, residual, partials=part, residual_ab=res_ab)
    return bn_act(bn, run_conv(conv, x), relu, res_deferred.materialise() if res_deferred else residual)
