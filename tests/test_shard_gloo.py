"""Multi-rank bag sharding (mcgmil.shard) on CPU with the gloo backend, world size 2 and 3.

Each rank computes only its LPT-assigned bags -- here with the CPU oracle as the per-rank
compute function (no GPU in this container) -- and one all_gather assembles Y[B, T, C]. The
result must equal the unsharded computation exactly, because every bag keeps its global
Philox stream (bag counter = global bag index)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_DIR, REPO

SIZES = [37, 5, 64, 200, 1, 90, 13]
T, C, L, SEED = 3, 2, 512, 11


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _bag_Y(b):
    from oracle import mcdo_ref
    from mcgmil import synthetic
    arrays = synthetic.head_arrays(synthetic.head_state_dict(1, C=C, shared=False), C, False)
    H = synthetic.bag_features(500 + b, SIZES[b], L)
    kF, kA = mcdo_ref.masks_for_bag(SEED, b, T, SIZES[b], L, C, 0.1, 0.1)
    Y, _ = mcdo_ref.mc_inference(H, mcdo_ref.HeadParams(arrays), kF, kA, 0.1, 0.1)
    return Y[:, 0]                                                  # [T, C]


def _worker(rank, world, port, out_path):
    import sys
    for p in (REPO, PKG_DIR):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mcgmil import shard
    seen = []

    def compute(idx):
        seen.extend(idx)
        if not idx:
            return torch.zeros(0, T, C)
        return torch.stack([_bag_Y(b) for b in idx])

    Y = shard.run_sharded(SIZES, T, compute, rank, world)
    gathered = [None] * world
    dist.all_gather_object(gathered, sorted(seen))
    if rank == 0:
        np.savez(out_path, Y=Y.numpy(), seen=np.array(sum(gathered, []), dtype=np.int64))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_equals_unsharded(tmp_path, world):
    out = str(tmp_path / "y.npz")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    z = np.load(out)
    ref = torch.stack([_bag_Y(b) for b in range(len(SIZES))]).numpy()
    assert np.array_equal(z["Y"], ref)
    assert sorted(z["seen"].tolist()) == list(range(len(SIZES)))   # each bag exactly once


def test_lpt_assignment():
    from mcgmil.shard import lpt_assign
    costs = [float(n) for n in SIZES]
    for world in (1, 2, 3, 8):
        a = lpt_assign(costs, world)
        assert sorted(sum(a, [])) == list(range(len(SIZES)))
        loads = [sum(costs[i] for i in r) for r in a]
        assert max(loads) <= sum(costs) / world + max(costs)       # LPT bound
    big = np.random.default_rng(0).integers(256, 2049, 4096).astype(float)
    loads = [sum(big[i] for i in r) for r in lpt_assign(list(big), 8)]
    assert max(loads) / min(loads) < 1.001                          # config 4 balances tightly
