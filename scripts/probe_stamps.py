"""Phase breakdown of the pipelined gate kernel from the diagnostic stamp build
(libmcgmil_stamps.so, -DMCGMIL_STAMPS). Stamps (s_memtime, shader cycles) per tile:
  0 start | 1 row table | 2 prologue staged | 3 K loop done | 4 epilogue folded |
  5 partials in LDS | 6 after the finish barrier | 7 end
Read the SHARES, not the absolute length (stamps add fences; guide §7)."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


PHASES = ["row_table", "prologue", "k_loop", "epilogue", "partials", "barrier", "scores"]


def main():
    from mcgmil import _build, _lib, ops
    from mcgmil import synthetic
    path = os.path.join(REPO, "montecarlo-gated-mil_amd", "mcgmil", "libmcgmil_stamps.so")
    extra = [d for d in os.environ.get("STAMP_DEFINES", "").split(",") if d]
    if extra:
        path = path.replace(".so", "_" + "_".join(x.replace("=", "") for x in extra) + ".so")
    _build.build(out=path, defines=["MCGMIL_STAMPS"] + extra)   # rebuilt when stale
    _lib.load()
    lib = ctypes.CDLL(path)
    for f in ("mcgmil_gate_scores", "mcgmil_workspace_size"):
        getattr(lib, f).restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    N, T, L, D, C = 2048, 100, 512, 128, 2
    B = int(os.environ.get("PROBE_BAGS", "16"))
    for shared in ((False,) if os.environ.get("PROBE_FUSED") == "1" else (False, True)):
        G = 1 if shared else C
        arrays = synthetic.head_arrays(synthetic.head_state_dict(0, C=C, shared=shared), C, shared)
        head = ops.HeadTensors(*[torch.from_numpy(arrays[k]).to(dev) for k in ops.HeadTensors._fields])
        H = torch.randn(B * N, L, device=dev).abs_().bfloat16()
        offs = ops.bag_offsets_tensor([N] * B, dev)
        packed = ops.packed_weights(head, torch.bfloat16)
        a = ops.make_args(H, offs, head, T, C, G, D, 0.1, 0.1, seed=1)
        a.packed_w = ctypes.c_void_p(packed.data_ptr())
        n = ctypes.c_size_t()
        lib.mcgmil_workspace_size(ctypes.byref(a), ctypes.byref(n))
        ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
        a.workspace, a.workspace_bytes = ctypes.c_void_p(ws.data_ptr()), n.value
        tiles = (B * N * T + 15) // 16          # enough for any kernel's tile size (>= 16 rows)
        st = torch.zeros(tiles * 8, dtype=torch.int64, device=dev)
        a.debug = ctypes.c_void_p(st.data_ptr())
        sh = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        # PROBE_FUSED=1: the fused single launch (MCGMIL_FUSED=1; a region's last tile's stamps)
        fused = os.environ.get("PROBE_FUSED") == "1"
        if fused:
            os.environ["MCGMIL_FUSED"] = "1"
            lib.mcgmil_gate_softmax_pool.restype = ctypes.c_int
            Y = torch.empty(B, T, C, device=dev)
            a.Y = ctypes.c_void_p(Y.data_ptr())
        launch = lib.mcgmil_gate_softmax_pool if fused else lib.mcgmil_gate_scores
        for _ in range(3):
            assert launch(ctypes.byref(a), sh) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert launch(ctypes.byref(a), sh) == 0
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        s = st.view(tiles, 8).cpu().numpy().astype(np.int64)
        s = s[s[:, 7] != 0]                      # the tiles the launch actually had
        tiles = len(s)
        d = np.diff(s, axis=1)
        tot = s[:, 7] - s[:, 0]
        span = s[:, 7].max() - s[:, 0].min()
        res = {"shared": shared, "kernel_ms": round(ms, 4), "tiles": tiles,
               "tile_cycles_median": int(np.median(tot)),
               "phase_cycles_median": {k: int(np.median(d[:, i])) for i, k in enumerate(
                   PHASES)},
               "phase_share": {k: round(float(d[:, i].sum() / tot.sum()), 3) for i, k in enumerate(
                   PHASES)},
               }
        print(json.dumps(res))


if __name__ == "__main__":
    main()
