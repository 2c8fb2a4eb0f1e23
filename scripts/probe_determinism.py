"""Run the gate-score launch repeatedly on identical inputs (config 3 shape) and report which
logits / z values differ between runs: count, and their positions within a 64- and 128-row
tile, class and sample t. Diagnostic for races in the gate kernels."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "montecarlo-gated-mil_amd")]


def main():
    from mcgmil import _lib, ops
    from mcgmil import synthetic
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from probe_gate import load_variant
    _lib.load()
    paths = [p for p in os.environ.get("MCGMIL_PROBE_LIBS", "").split(",") if p]
    libs = {os.path.basename(p): load_variant(p) for p in paths} or {"libmcgmil.so": _lib.load()}
    dev = torch.device("cuda", 0)
    for name, lib in libs.items():
        run(lib, name, dev, _lib, ops, synthetic)


def run(lib, name, dev, _lib, ops, synthetic):
    N, T, L, D, C = 2048, 100, 512, 128, 2
    B = int(os.environ.get("PROBE_BAGS", "4"))
    for shared in (False, True):
        G = 1 if shared else C
        arrays = synthetic.head_arrays(synthetic.head_state_dict(0, C=C, shared=shared), C, shared)
        head = ops.HeadTensors(*[torch.from_numpy(arrays[k]).to(dev) for k in ops.HeadTensors._fields])
        H = torch.randn(B * N, L, device=dev).abs_().bfloat16()
        offs = ops.bag_offsets_tensor([N] * B, dev)
        packed = ops.packed_weights(head, torch.bfloat16)
        a = ops.make_args(H, offs, head, T, C, G, D, 0.1, 0.1, seed=1)
        a.packed_w = ctypes.c_void_p(packed.data_ptr())
        n = ctypes.c_size_t()
        _lib.check(lib.mcgmil_workspace_size(ctypes.byref(a), ctypes.byref(n)), "ws")
        ws = torch.zeros(n.value, dtype=torch.uint8, device=dev)
        a.workspace, a.workspace_bytes = ctypes.c_void_p(ws.data_ptr()), n.value
        sh = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        rows = B * N * T
        outs = []
        for rep in range(4):
            ws.zero_()
            _lib.check(lib.mcgmil_gate_scores(ctypes.byref(a), sh), "gate")
            torch.cuda.synchronize()
            # logits then zz, [rows, C] each, at the start of the workspace after packed weights
            outs.append(ws.clone())
        base = outs[0].view(torch.int32)
        diffs = [(o.view(torch.int32) != base).nonzero().flatten().cpu().numpy() for o in outs[1:]]
        allw = np.unique(np.concatenate(diffs)) if diffs else np.array([], dtype=np.int64)
        n_el = rows * C
        res = {"lib": name, "shared": shared, "kernel_env": os.environ.get("MCGMIL_GATE", "default"),
               "mismatch_words": int(len(allw)), "per_rep": [int(len(d)) for d in diffs]}
        if len(allw):
            # workspace words: [packed? no: packed_w supplied] logits [rows*C], zz [rows*C]
            which = np.where(allw < n_el, "logit", "zz")
            idx = np.where(allw < n_el, allw, allw - n_el)
            r, c = idx // C, idx % C
            res["which"] = {k: int((which == k).sum()) for k in ("logit", "zz")}
            res["row_mod64_hist"] = np.bincount(r % 64, minlength=64).tolist()
            res["class_hist"] = np.bincount(c, minlength=C).tolist()
            res["first_rows"] = r[:12].tolist()
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
