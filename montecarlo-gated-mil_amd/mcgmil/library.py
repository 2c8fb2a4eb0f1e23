"""torch.library registration of the MCDO head ("register it with
torch.library.custom_op so it composes with torch.compile / autograd-free inference").

    torch.ops.mcgmil.mcdo_forward(H, bag_offsets, Wv, bv, Wu, bu, wa, ba, wk, T, p_feat, p_att,
                                  seed, bag_id_base=0, t_base=0) -> (Y [B, T, C], A [T*C*R])
    torch.ops.mcgmil.mcdo_forward_stats(...same...) -> (Y, A_mean [C*R], A_var [C*R], P_mean [B, C])

Same semantics as `mcgmil.ops.mcdo_forward` (reference model.py:256-328 for every bag of the
batch, bags as CSR row ranges of H). The ops are opaque to a graph capture: the fake (meta)
implementations below only derive output shapes, and the real ones run the gfx950 kernels
through the C ABI. There is no CPU kernel: called with CPU tensors they raise. `seed` is the
64-bit Philox key as a signed int64 (the schema's int); it is reinterpreted as unsigned.
"""
from typing import Tuple

import torch

from . import ops

__all__ = ["mcdo_forward", "mcdo_forward_stats"]


def _head(Wv, bv, Wu, bu, wa, ba, wk) -> ops.HeadTensors:
    return ops.HeadTensors(Wv, bv, Wu, bu, wa, ba, wk)


@torch.library.custom_op("mcgmil::mcdo_forward", mutates_args=())
def mcdo_forward(H: torch.Tensor, bag_offsets: torch.Tensor, Wv: torch.Tensor, bv: torch.Tensor,
                 Wu: torch.Tensor, bu: torch.Tensor, wa: torch.Tensor, ba: torch.Tensor,
                 wk: torch.Tensor, T: int, p_feat: float, p_att: float, seed: int,
                 bag_id_base: int = 0, t_base: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    out = ops.mcdo_forward(H, bag_offsets, _head(Wv, bv, Wu, bu, wa, ba, wk), T, p_feat=p_feat,
                           p_att=p_att, seed=seed & 0xFFFFFFFFFFFFFFFF, bag_id_base=bag_id_base,
                           t_base=t_base)
    return out["Y"], out["A"]


@mcdo_forward.register_fake
def _mcdo_forward_fake(H, bag_offsets, Wv, bv, Wu, bu, wa, ba, wk, T, p_feat, p_att, seed,
                       bag_id_base=0, t_base=0):
    B, C, R = bag_offsets.shape[0] - 1, wa.shape[0], H.shape[0]
    return (H.new_empty((B, T, C), dtype=torch.float32),
            H.new_empty((T * C * R,), dtype=torch.float32))


@torch.library.custom_op("mcgmil::mcdo_forward_stats", mutates_args=())
def mcdo_forward_stats(H: torch.Tensor, bag_offsets: torch.Tensor, Wv: torch.Tensor,
                       bv: torch.Tensor, Wu: torch.Tensor, bu: torch.Tensor, wa: torch.Tensor,
                       ba: torch.Tensor, wk: torch.Tensor, T: int, p_feat: float, p_att: float,
                       seed: int, bag_id_base: int = 0, t_base: int = 0
                       ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    out = ops.mcdo_forward(H, bag_offsets, _head(Wv, bv, Wu, bu, wa, ba, wk), T, p_feat=p_feat,
                           p_att=p_att, seed=seed & 0xFFFFFFFFFFFFFFFF, bag_id_base=bag_id_base,
                           t_base=t_base, return_attention=False, return_stats=True)
    return out["Y"], out["A_mean"], out["A_var"], out["P_mean"]


@mcdo_forward_stats.register_fake
def _mcdo_forward_stats_fake(H, bag_offsets, Wv, bv, Wu, bu, wa, ba, wk, T, p_feat, p_att, seed,
                             bag_id_base=0, t_base=0):
    B, C, R = bag_offsets.shape[0] - 1, wa.shape[0], H.shape[0]
    f = torch.float32
    return (H.new_empty((B, T, C), dtype=f), H.new_empty((C * R,), dtype=f),
            H.new_empty((C * R,), dtype=f), H.new_empty((B, C), dtype=f))
