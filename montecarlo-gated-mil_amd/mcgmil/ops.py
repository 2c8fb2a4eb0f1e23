"""torch-facing wrappers of the C ABI: device buffers from PyTorch's caching allocator, launches
on torch's current HIP stream, results as torch tensors. Every function runs the gfx950 kernels;
none has a CPU path.

Reference semantics served: MultiHeadGatedAttentionMIL.mc_inference (reference model.py:256-328)
from the extracted features H on, for a whole batch of bags at once.
"""
import ctypes
import weakref
from typing import NamedTuple, Optional, Sequence, Union

import torch

from . import _lib

_DT = {torch.float32: _lib.MCGMIL_F32, torch.bfloat16: _lib.MCGMIL_BF16}


class HeadTensors(NamedTuple):
    """MIL head parameters, fp32, torch nn.Linear layout (reference model.py:182-203)."""
    Wv: torch.Tensor  # [G, D, L]
    bv: torch.Tensor  # [G, D]
    Wu: torch.Tensor  # [G, D, L]
    bu: torch.Tensor  # [G, D]
    wa: torch.Tensor  # [C, D]
    ba: torch.Tensor  # [C]
    wk: torch.Tensor  # [C, L]

    @property
    def G(self):
        return self.Wv.shape[0]

    @property
    def C(self):
        return self.wa.shape[0]

    @property
    def D(self):
        return self.Wv.shape[1]

    @property
    def L(self):
        return self.Wv.shape[2]

    def to(self, device):
        return HeadTensors(*[t.detach().to(device=device, dtype=torch.float32).contiguous()
                             for t in self])


def _p(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_cuda(name, t, dtype=None):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA(HIP) tensor")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")


# heads already validated (per-call host time): id(head) -> (weak references to its tensors, the
# device, each tensor's (data_ptr, stride)). No strong reference: a dropped model's GPU weights are
# freed. A hit needs the same tensor objects at the same storage and layout, so rebinding a field
# with `t.data = other` is validated again.
_CHECKED_HEADS: dict = {}


def _head_fingerprint(head: HeadTensors):
    return tuple((t.data_ptr(), t.stride()) for t in head)


def _check_head(head: HeadTensors, device):
    hit = _CHECKED_HEADS.get(id(head))
    if hit is not None and hit[1] == device and all(r() is t for r, t in zip(hit[0], head)) and \
            hit[2] == _head_fingerprint(head):
        return                    # same tensors, storage and layout: dtype and device unchanged
    for name, t in zip(head._fields, head):
        _require_cuda(name, t, torch.float32)
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
        if t.device != device:
            raise ValueError(f"{name} is on {t.device}, H on {device}")
    if len(_CHECKED_HEADS) > 16:
        _CHECKED_HEADS.clear()
    _CHECKED_HEADS[id(head)] = (tuple(weakref.ref(t) for t in head), device, _head_fingerprint(head))


class BagOffsets(torch.Tensor):
    """int32 CSR offsets [B+1] on the device that remember, from the host-side sizes they were
    built from, whether every bag has the same size (`uniform_rows`, 0 if ragged). No torch-function
    override: methods dispatch as on a plain tensor (and return plain tensors), so the subclass
    costs the per-call path nothing."""
    uniform_rows: int = 0
    __torch_function__ = torch._C._disabled_torch_function_impl


def uniform_offsets(n: int, bags: int, device) -> torch.Tensor:
    """CSR offsets of `bags` bags of n instances each, made on the device (no host->device copy,
    no synchronisation: the single-bag caller of infer.py:187-191 pays nothing for them)."""
    if n < 1 or bags < 1 or n * bags >= 2**31:
        raise ValueError("uniform bags need n >= 1, bags >= 1 and n * bags < 2^31")
    t = torch.arange(0, n * (bags + 1), n, dtype=torch.int32, device=device).as_subclass(BagOffsets)
    t.uniform_rows = n
    return t


def bag_offsets_tensor(sizes_or_offsets: Union[Sequence[int], torch.Tensor], device,
                       are_sizes: bool = True) -> torch.Tensor:
    """Build the int32 CSR offsets [B+1] on `device` from bag sizes (or offsets). The host copy
    is pinned and copied asynchronously, so a caller with queued GPU work is not stalled."""
    x = torch.as_tensor(sizes_or_offsets, dtype=torch.int64).cpu()
    if are_sizes:
        x = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(x, 0)])
    if x.numel() < 2 or x[0] != 0 or bool((x[1:] < x[:-1]).any()):
        raise ValueError("bag offsets must start at 0 and be non-decreasing")
    if int(x[-1]) >= 2**31:
        raise ValueError("total rows must fit int32")
    d = x[1:] - x[:-1]
    uniform = int(d[0]) if bool((d == d[0]).all()) and int(d[0]) > 0 else 0
    x = x.to(torch.int32)
    if torch.device(device).type == "cuda":
        x = x.pin_memory()
    t = x.to(device=device, non_blocking=True).as_subclass(BagOffsets)
    t.uniform_rows = uniform
    return t


def make_args(H: Optional[torch.Tensor], bag_offsets: torch.Tensor, head: Optional[HeadTensors],
              T: int, C: int, G: int, D: int, p_feat: float, p_att: float, seed: int,
              bag_id_base: int = 0, t_base: int = 0, L: Optional[int] = None,
              total_rows: Optional[int] = None,
              bag_ids: Optional[torch.Tensor] = None, path: str = "auto",
              gate: str = "auto") -> _lib.Args:
    """Fill struct mcgmil_args. With H=None, L and total_rows describe the (absent) features.
    path: "auto" | "fused" | "two_kernel", gate: "auto" | "pipe" | "pp" (mcgmil_args.flags)."""
    if path not in _lib.PATH_FLAGS or gate not in _lib.GATE_FLAGS:
        raise ValueError(f"path must be one of {list(_lib.PATH_FLAGS)}, gate one of {list(_lib.GATE_FLAGS)}")
    a = _lib.Args()
    a.flags = _lib.PATH_FLAGS[path] | _lib.GATE_FLAGS[gate]
    a.L = H.shape[1] if H is not None else int(L)
    a.D = D
    a.C = C
    a.G = G
    a.T = int(T)
    a.num_bags = bag_offsets.numel() - 1
    a.total_rows = H.shape[0] if H is not None else int(total_rows)
    a.h_dtype = _DT[H.dtype] if H is not None else _lib.MCGMIL_F32
    if H is not None:
        a.H = _p(H)
        a.ldh = H.stride(0) if H.shape[0] > 0 else H.shape[1]
    else:
        a.ldh = a.L
    a.bag_offsets = _p(bag_offsets)
    a.uniform_bag_rows = int(getattr(bag_offsets, "uniform_rows", 0))
    if head is not None:
        a.Wv, a.bv, a.Wu, a.bu = _p(head.Wv), _p(head.bv), _p(head.Wu), _p(head.bu)
        a.wa, a.ba, a.wk = _p(head.wa), _p(head.ba), _p(head.wk)
    a.p_feat = float(p_feat)
    a.p_att = float(p_att)
    a.seed = int(seed) & (2**64 - 1)
    a.bag_id_base = int(bag_id_base) & 0xFFFFFFFF
    a.t_base = int(t_base)
    if bag_ids is not None:
        _require_cuda("bag_ids", bag_ids, torch.int32)
        if bag_ids.numel() != a.num_bags or not bag_ids.is_contiguous():
            raise ValueError("bag_ids must be a contiguous int32 vector with one entry per bag")
        a.bag_ids = _p(bag_ids)
    return a


def _validate_inputs(H, bag_offsets):
    _require_cuda("H", H)
    if H.dtype not in _DT:
        raise ValueError(f"H must be float32 or bfloat16, got {H.dtype}")
    if H.dim() != 2 or (H.shape[0] > 0 and H.stride(1) != 1):
        raise ValueError("H must be a row-major [rows, L] matrix")
    _require_cuda("bag_offsets", bag_offsets, torch.int32)
    if bag_offsets.dim() != 1 or bag_offsets.numel() < 2 or not bag_offsets.is_contiguous():
        raise ValueError("bag_offsets must be a contiguous int32 vector of length B+1")


def packed_weights(head: HeadTensors, dtype: torch.dtype) -> torch.Tensor:
    """Re-lay the head's GEMM weights out as gfx950 MFMA operand tiles (mcgmil_pack_weights)."""
    L = _lib.load()
    dev = head.Wv.device
    _check_head(head, dev)
    a = make_args(None, torch.zeros(2, dtype=torch.int32, device=dev), head, 1, head.C, head.G,
                  head.D, 0.0, 0.0, 0, L=head.L, total_rows=0)
    a.h_dtype = _DT[dtype]
    n = ctypes.c_size_t()
    _lib.check(L.mcgmil_packed_weights_size(ctypes.byref(a), ctypes.byref(n)), "mcgmil_packed_weights_size")
    out = torch.empty(n.value, dtype=torch.uint8, device=dev)
    _lib.check(L.mcgmil_pack_weights(ctypes.byref(a), _p(out), _stream(dev)), "mcgmil_pack_weights")
    return out


def mcdo_forward(H: torch.Tensor, bag_offsets: torch.Tensor, head: HeadTensors, T: int, *,
                 p_feat: float, p_att: float, seed: int, bag_id_base: int = 0, t_base: int = 0,
                 keep_feat: Optional[torch.Tensor] = None, keep_att: Optional[torch.Tensor] = None,
                 return_attention: bool = True, return_stats: bool = False,
                 packed: Optional[torch.Tensor] = None,
                 bag_ids: Optional[torch.Tensor] = None, path: str = "auto",
                 gate: str = "auto") -> dict:
    """All T MC-dropout samples of every bag in one call (mcgmil_mcdo_forward).

    H: [total_rows, L] fp32/bf16 on the GPU, bags as CSR row ranges bag_offsets[B+1] (int32,
    same device, last entry = total_rows). Bag b draws the Philox stream of bag counter
    bag_ids[b] (int32 [B] on the device) if given, else bag_id_base + b. `path` / `gate` pick the
    launch path (mcgmil_args.flags; every path gives bitwise the same outputs). Returns a dict with
      Y      [B, T, C]            class logits        (reference Y[T,1,C] per bag)
      A      [T*C*total_rows]     attention, per bag [T, C, N_b] (reference A[T,1,C,N])
      A_mean, A_var [C*total_rows], per bag [C, N_b];  P_mean [B, C]   (if return_stats)
    """
    L = _lib.load()
    _validate_inputs(H, bag_offsets)
    dev = H.device
    _check_head(head, dev)
    if head.L != H.shape[1]:
        raise ValueError(f"H has L={H.shape[1]}, the head expects L={head.L}")
    a = make_args(H, bag_offsets, head, T, head.C, head.G, head.D, p_feat, p_att, seed,
                  bag_id_base, t_base, bag_ids=bag_ids, path=path, gate=gate)
    B, R, C = a.num_bags, a.total_rows, head.C
    if packed is not None:
        a.packed_w = _p(packed)
    if keep_feat is not None or keep_att is not None:
        if keep_feat is None or keep_att is None:
            raise ValueError("replay mode needs both keep_feat and keep_att")
        _require_cuda("keep_feat", keep_feat, torch.uint8)
        _require_cuda("keep_att", keep_att, torch.uint8)
        if keep_feat.numel() != T * R * (H.shape[1] // 8) or keep_att.numel() != T * C * R:
            raise ValueError("replay masks have the wrong size")
        if not (keep_feat.is_contiguous() and keep_att.is_contiguous()):
            raise ValueError("replay masks must be contiguous")
        a.keep_feat, a.keep_att = _p(keep_feat), _p(keep_att)
    out = {"Y": torch.empty(B, T, C, dtype=torch.float32, device=dev)}
    a.Y = _p(out["Y"])
    if return_attention or return_stats:
        out["A"] = torch.empty(T * C * R, dtype=torch.float32, device=dev)
        a.A = _p(out["A"])
    if return_stats:
        out["A_mean"] = torch.empty(C * R, dtype=torch.float32, device=dev)
        out["A_var"] = torch.empty(C * R, dtype=torch.float32, device=dev)
        out["P_mean"] = torch.empty(B, C, dtype=torch.float32, device=dev)
        a.A_mean, a.A_var, a.P_mean = _p(out["A_mean"]), _p(out["A_var"]), _p(out["P_mean"])
    n = ctypes.c_size_t()
    _lib.check(L.mcgmil_workspace_size(ctypes.byref(a), ctypes.byref(n)), "mcgmil_workspace_size")
    ws = torch.empty(max(n.value, 1), dtype=torch.uint8, device=dev)
    a.workspace, a.workspace_bytes = _p(ws), n.value
    _lib.check(L.mcgmil_mcdo_forward(ctypes.byref(a), _stream(dev)), "mcgmil_mcdo_forward")
    if not return_attention:
        out.pop("A", None)
    return out


def clock_record(device) -> torch.Tensor:
    """A zeroed MCGMIL_CLOCK_PROBE record (args.debug): int64 [MCGMIL_CLOCK_SLOTS, 4]."""
    return torch.zeros(_lib.CLOCK_SLOTS, 4, dtype=torch.int64, device=device)


def clock_mhz(record: torch.Tensor) -> Optional[dict]:
    """The shader clock a probed gate launch ran at: per workgroup d(s_memtime) / d(s_memrealtime)
    x 100 MHz (the realtime counter's rate) over the workgroups that wrote a record; the median
    and the spread. None when no workgroup wrote one."""
    r = record.cpu().double()
    dt, dr = r[:, 2] - r[:, 0], r[:, 3] - r[:, 1]
    ok = (dr > 0) & (dt > 0)
    if not bool(ok.any()):
        return None
    mhz = (dt[ok] / dr[ok] * 100.0).sort().values
    n = mhz.numel()
    return {"median": float(mhz[n // 2]), "p10": float(mhz[n // 10]), "p90": float(mhz[(9 * n) // 10]),
            "workgroups": n, "median_span_us": float((dr[ok] / 100.0).median())}


def split_bags(flat: torch.Tensor, sizes: Sequence[int], per_row: int):
    """Split a per-row flat output (A: per_row = T*C; A_mean: per_row = C) into bag views."""
    out, o = [], 0
    for n in sizes:
        out.append(flat[o:o + per_row * n])
        o += per_row * n
    return out


def feature_keep(bag_offsets: torch.Tensor, total_rows: int, T: int, L: int, p: float, seed: int,
                 bag_id_base: int = 0, t_base: int = 0,
                 bag_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The feature keep bits the kernel draws: uint8 [T*total_rows, L/8] (order bag, t, n)."""
    lib = _lib.load()
    dev = bag_offsets.device
    a = make_args(None, bag_offsets, None, T, 1, 1, 16, p, 0.0, seed, bag_id_base, t_base,
                  L=L, total_rows=total_rows, bag_ids=bag_ids)
    out = torch.empty(T * total_rows, L // 8, dtype=torch.uint8, device=dev)
    _lib.check(lib.mcgmil_feature_keep(ctypes.byref(a), _p(out), _stream(dev)), "mcgmil_feature_keep")
    return out


def attention_keep(bag_offsets: torch.Tensor, total_rows: int, T: int, C: int, p: float,
                   seed: int, bag_id_base: int = 0, t_base: int = 0,
                   bag_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The attention keep flags the kernel draws: uint8 [T*C*total_rows] (order bag, t, c, n)."""
    lib = _lib.load()
    dev = bag_offsets.device
    a = make_args(None, bag_offsets, None, T, C, 1, 16, 0.0, p, seed, bag_id_base, t_base,
                  L=32, total_rows=total_rows, bag_ids=bag_ids)
    out = torch.empty(T * C * total_rows, dtype=torch.uint8, device=dev)
    _lib.check(lib.mcgmil_attention_keep(ctypes.byref(a), _p(out), _stream(dev)), "mcgmil_attention_keep")
    return out
