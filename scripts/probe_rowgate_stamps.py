"""Phase cycles of the row-gate kernel (rowgate_scores_kernel) from the diagnostic stamp build
(-DMCGMIL_STAMPS): per (tile, wave) s_memtime at 0 tile start | 1 next-tile rows decoded |
2 K loop done | 3 epilogue + stores done. Read shares and medians; stamps perturb the schedule."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from mcgmil import _lib, ops, synthetic
    path = os.environ.get("STAMP_LIB", os.path.join(REPO, "abvar", "stamps.so"))
    _lib.load()
    lib = _lib.bind(path, mcdo_only=True)
    dev = torch.device("cuda", 0)
    N, T, L, D, C = 2048, 100, 512, 128, 2
    B = int(os.environ.get("PROBE_BAGS", "16"))
    for shared in (False, True):
        G = 1 if shared else C
        arrays = synthetic.head_arrays(synthetic.head_state_dict(0, C=C, shared=shared), C, shared)
        head = ops.HeadTensors(*[torch.from_numpy(arrays[k]).to(dev) for k in ops.HeadTensors._fields])
        H = torch.randn(B * N, L, device=dev).abs_().bfloat16()
        offs = ops.bag_offsets_tensor([N] * B, dev)
        packed = ops.packed_weights(head, torch.bfloat16)
        a = ops.make_args(H, offs, head, T, C, G, D, 0.1, 0.1, seed=1, gate="row", path="two_kernel")
        a.packed_w = ctypes.c_void_p(packed.data_ptr())
        n = ctypes.c_size_t()
        lib.mcgmil_workspace_size(ctypes.byref(a), ctypes.byref(n))
        ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
        a.workspace, a.workspace_bytes = ctypes.c_void_p(ws.data_ptr()), n.value
        tiles = (B * N * T + 127) // 128
        st = torch.zeros(tiles * 4 * 8, dtype=torch.int64, device=dev)
        a.debug = ctypes.c_void_p(st.data_ptr())
        sh = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for _ in range(3):
            assert lib.mcgmil_gate_scores(ctypes.byref(a), sh) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert lib.mcgmil_gate_scores(ctypes.byref(a), sh) == 0
        e1.record()
        torch.cuda.synchronize()
        s = st.view(tiles * 4, 8).cpu().numpy().astype(np.int64)[:, :4]
        s = s[s[:, 3] != 0]
        d = np.diff(s, axis=1)
        tot = s[:, 3] - s[:, 0]
        names = ["decode", "k_loop", "epilogue"]
        print(json.dumps({"shared": shared, "kernel_ms": round(e0.elapsed_time(e1), 4), "wave_tiles": len(s),
                          "tile_cycles_median": int(np.median(tot)),
                          "phase_cycles_median": {k: int(np.median(d[:, i])) for i, k in enumerate(names)},
                          "phase_share": {k: round(float(d[:, i].sum() / tot.sum()), 3) for i, k in enumerate(names)}}),
              flush=True)


if __name__ == "__main__":
    main()
