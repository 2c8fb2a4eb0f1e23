"""Multi-rank bag sharding with the GPU kernels: two ranks on cuda:0 (one process each, gloo for
the gather: RCCL does not allow two ranks on one device), each running ops.mcdo_forward on its
LPT shard with the bags' global ids, then shard.gather_predictions. The gathered Y must equal
the single-process run bit for bit -- what makes the 1/2/4/8-GPU results of bench.py identical.
(The 8-GPU RCCL run itself is the driver's; this is the functional rehearsal of its data path.)"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_DIR, REPO

pytestmark = pytest.mark.gpu

SIZES = [300, 37, 2048, 512, 1, 999, 64, 1500, 128]
T, C, L, SEED = 20, 2, 512, 77


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _inputs(dev):
    from mcgmil import ops, synthetic
    arrays = synthetic.head_arrays(synthetic.head_state_dict(6, C=C, shared=False), C, False)
    head = ops.HeadTensors(*[torch.from_numpy(arrays[k]).to(dev) for k in ops.HeadTensors._fields])
    Hs = [torch.from_numpy(synthetic.bag_features(700 + b, n, L)).to(dev).bfloat16()
          for b, n in enumerate(SIZES)]
    return head, Hs


def _worker(rank, world, port, out_path):
    import sys
    for p in (REPO, PKG_DIR):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mcgmil import ops, shard
    head, Hs = _inputs(dev)
    assignment = shard.lpt_assign([float(n) * T for n in SIZES], world)
    mine = assignment[rank]
    ids = torch.tensor(mine, dtype=torch.int32, device=dev)
    out = ops.mcdo_forward(torch.cat([Hs[b] for b in mine]),
                           ops.bag_offsets_tensor([SIZES[b] for b in mine], dev), head, T,
                           p_feat=0.1, p_att=0.1, seed=SEED, bag_ids=ids)
    Y = shard.gather_predictions(out["Y"].cpu(), assignment, rank)
    if rank == 0:
        np.save(out_path, Y.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_on_one_gpu_match_single_process(cuda, tmp_path):
    from mcgmil import ops
    head, Hs = _inputs(cuda)
    full = ops.mcdo_forward(torch.cat(Hs), ops.bag_offsets_tensor(SIZES, cuda), head, T,
                            p_feat=0.1, p_att=0.1, seed=SEED)["Y"].cpu()
    out = str(tmp_path / "y.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert np.array_equal(np.load(out), full.numpy())
