"""Time the gate-score kernel under variants, interleaved in one process (guide §5.4 rule 24).

  philox   : masks drawn in-register (the product path)
  replay   : masks read from a precomputed bit buffer (isolates the RNG cost)
  p0       : p_feat = p_att = 0 (Philox still runs; compare to see the select cost)
Prints one JSON line per variant with median kernel ms and TFLOP/s (algorithmic).
"""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def load_variant(path):
    from mcgmil import _lib
    return _lib.bind(path, mcdo_only=True)


def main():
    from mcgmil import _lib, ops
    from mcgmil import synthetic
    _lib.load()
    # MCGMIL_PROBE_LIBS=a.so,b.so: A/B variant builds of the library in one process
    paths = [p for p in os.environ.get("MCGMIL_PROBE_LIBS", "").split(",") if p]
    libs = {os.path.basename(p): load_variant(p) for p in paths} or {"libmcgmil.so": _lib.load()}
    only = os.environ.get("PROBE_ONLY", "")
    dev = torch.device("cuda", 0)
    N, T, L, D, C = 2048, 100, 512, 128, 2
    B = int(os.environ.get("PROBE_BAGS", "16"))
    rounds = int(os.environ.get("PROBE_ROUNDS", "7"))
    iters = 5
    variants = []
    for name in libs:
        sep_only = os.environ.get("PROBE_SEP_ONLY") == "1"      # bf16 separate heads only
        for dtype in ((torch.bfloat16,) if sep_only else (torch.bfloat16, torch.float32)):
            for shared in ((False,) if sep_only else (False, True)):
                for mode in ("philox", "replay", "p0"):
                    if dtype == torch.float32 and mode != "philox":
                        continue
                    if only and mode not in only.split(","):
                        continue
                    variants.append((name, dtype, shared, mode))
    setups = {}
    g = torch.Generator(device=dev).manual_seed(0)
    Hf = torch.randn(B * N, L, device=dev, generator=g).abs_()
    offs = ops.bag_offsets_tensor([N] * B, dev)
    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)
    keep_f = keep_a = None
    for v in variants:
        name, dtype, shared, mode = v
        G = 1 if shared else C
        Bv = B if dtype == torch.bfloat16 else max(1, B // 4)
        H = Hf[:Bv * N].to(dtype).contiguous()
        offv = offs[:Bv + 1].contiguous()
        arrays = synthetic.head_arrays(synthetic.head_state_dict(0, C=C, shared=shared), C, shared)
        head = ops.HeadTensors(*[torch.from_numpy(arrays[k]).to(dev) for k in ops.HeadTensors._fields])
        packed = ops.packed_weights(head, dtype)
        p = 0.0 if mode == "p0" else 0.1
        a = ops.make_args(H, offv, head, T, C, G, D, p, p, seed=1)
        a.packed_w = ctypes.c_void_p(packed.data_ptr())
        if mode == "replay":
            if keep_f is None:
                keep_f = ops.feature_keep(offs, B * N, T, L, 0.1, 1)
                keep_a = ops.attention_keep(offs, B * N, T, C, 0.1, 1)
            a.keep_feat = ctypes.c_void_p(keep_f.data_ptr())
            a.keep_att = ctypes.c_void_p(keep_a.data_ptr())
        n = ctypes.c_size_t()
        lib = libs[name]
        _lib.check(lib.mcgmil_workspace_size(ctypes.byref(a), ctypes.byref(n)), "ws")
        ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
        a.workspace, a.workspace_bytes = ctypes.c_void_p(ws.data_ptr()), n.value
        flops = Bv * T * (2 * N * L * D * 2 * G + 2 * N * D * C + 2 * N * L * C + 2 * L * C)
        setups[v] = (a, ws, H, head, packed, flops, Bv, lib)
    times = {v: [] for v in variants}
    for _ in range(rounds):
        for v in variants:
            a, lib = setups[v][0], setups[v][7]
            _lib.check(lib.mcgmil_gate_scores(ctypes.byref(a), sh), "gate")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(iters):
                lib.mcgmil_gate_scores(ctypes.byref(a), sh)
            e1.record(stream)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / iters)
    for v in variants:
        name, dtype, shared, mode = v
        ms = statistics.median(times[v])
        flops, Bv = setups[v][5], setups[v][6]
        print(json.dumps({"lib": name, "dtype": str(dtype).split(".")[-1], "shared": shared, "mode": mode,
                          "bags": Bv, "ms": round(ms, 4), "min_ms": round(min(times[v]), 4),
                          "tflops": round(flops / (ms * 1e-3) / 1e12, 1),
                          "bag_samples_per_s": round(Bv * T / (ms * 1e-3))}))


if __name__ == "__main__":
    main()
