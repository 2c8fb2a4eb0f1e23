"""Bitwise comparison of the MCDO outputs (Y, A, A_mean, A_var, P_mean) of two builds of
libmcgmil.so on the same inputs (MCGMIL_PROBE_LIBS=old.so,new.so): a refactor that must not
change results is checked with this before its timing is trusted."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))
sys.path.insert(0, REPO)


def run(path, bags, n, T, shared):
    from mcgmil import _lib, ops
    from mcgmil import synthetic
    _lib._lib = _lib.bind(path, mcdo_only=True)
    dev = torch.device("cuda", 0)
    C = 2
    sd = synthetic.head_state_dict(0, C=C, shared=shared)
    arrays = synthetic.head_arrays(sd, C, shared)
    head = ops.HeadTensors(*[torch.from_numpy(arrays[k]).to(dev) for k in ops.HeadTensors._fields])
    g = torch.Generator(device=dev).manual_seed(3)
    sizes = [n + 37 * b for b in range(bags)]
    H = torch.randn(sum(sizes), 512, device=dev, generator=g).abs_().bfloat16()
    out = ops.mcdo_forward(H, ops.bag_offsets_tensor(sizes, dev), head, T, p_feat=0.1, p_att=0.1,
                           seed=42, return_attention=True, return_stats=True)
    torch.cuda.synchronize()
    return {k: v.cpu() for k, v in out.items() if torch.is_tensor(v)}


def main():
    libs = os.environ["MCGMIL_PROBE_LIBS"].split(",")
    a = libs[0]
    for b in libs[1:]:      # every variant against the first
        for shared in (False, True):
            for bags, n, T in ((3, 2048, 100), (5, 300, 7), (2, 4000, 5), (1, 5000, 3)):
                ra, rb = run(a, bags, n, T, shared), run(b, bags, n, T, shared)
                same = all(bool(torch.equal(ra[k], rb[k])) for k in ra)
                print(json.dumps({"a": os.path.basename(a), "b": os.path.basename(b), "shared": shared,
                                  "bags": bags, "n": n, "T": T, "bitwise_equal": same}))


if __name__ == "__main__":
    main()
