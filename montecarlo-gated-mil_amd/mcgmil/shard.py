"""Bag sharding across the GPUs of a node (one process per GPU, torch.distributed).

The reference is single-process; bags are independent (bs=1, the
softmax is within a bag), so the batch is split by bag with no data-path collective. Each
rank runs the varlen kernel on its bags; the only exchange is one gather of the per-bag
predictions Y[T, C] (RCCL over xGMI with backend "nccl", gloo on CPU for tests).

Bags keep their global Philox bag counter (ops.mcdo_forward(bag_ids=...)), so results do not
depend on the number of ranks.
"""
from typing import Callable, List, Sequence

import torch
import torch.distributed as dist


def lpt_assign(costs: Sequence[float], world: int) -> List[List[int]]:
    """Longest-processing-time-first: bags sorted by cost (N_b * T), each to the least-loaded
    rank. Returns the global bag indices per rank, each list in ascending order."""
    load = [0.0] * world
    out: List[List[int]] = [[] for _ in range(world)]
    for b in sorted(range(len(costs)), key=lambda i: (-costs[i], i)):
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(b)
        load[r] += costs[b]
    return [sorted(x) for x in out]


def gather_predictions(Y_local: torch.Tensor, assignment: List[List[int]], rank: int,
                       group=None) -> torch.Tensor:
    """Gather per-rank Y [B_local, T, C] into the global Y [B, T, C] on every rank."""
    world = len(assignment)
    pad = max(len(a) for a in assignment)
    T, C = Y_local.shape[1:]
    buf = torch.zeros(pad, T, C, dtype=Y_local.dtype, device=Y_local.device)
    buf[:Y_local.shape[0]] = Y_local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    B = sum(len(a) for a in assignment)
    out = torch.empty(B, T, C, dtype=Y_local.dtype, device=Y_local.device)
    for r, idx in enumerate(assignment):
        if idx:
            out[torch.as_tensor(idx, device=out.device)] = parts[r][:len(idx)]
    return out


def run_sharded(bag_sizes: Sequence[int], T: int, compute: Callable[[List[int]], torch.Tensor],
                rank: int, world: int, group=None) -> torch.Tensor:
    """Split bags over ranks (LPT on N_b * T), call compute(local global-bag-indices) ->
    Y_local [B_local, T, C], and gather the global Y [B, T, C] on every rank."""
    assignment = lpt_assign([float(n) * T for n in bag_sizes], world)
    Y_local = compute(assignment[rank])
    return gather_predictions(Y_local, assignment, rank, group)
