"""A/B of the single-launch MCDO path (gate_fused_kernel) against the two-kernel path
(gate_pipe_kernel + softmax_pool_kernel), interleaved in one process, optionally over several
variant builds of the library (MCGMIL_PROBE_LIBS=a.so,b.so; scripts/build_variants.sh).

Config 3 shape (N=2048, T=100, bf16, separate heads; PROBE_N, PROBE_T and PROBE_DTYPE=f32 change
it), PROBE_BAGS bags per launch (default 128).
Per (library, path): median ms of the gate(+softmax) launch(es) by HIP events, algorithmic
TFLOP/s, and whether Y and A are bitwise equal to the first library's two-kernel path."""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    from mcgmil import _lib, ops, synthetic
    from bench import flops_per_bag
    base = _lib.load()
    paths = [p for p in os.environ.get("MCGMIL_PROBE_LIBS", "").split(",") if p]
    libs = {os.path.basename(p): _lib.bind(p, mcdo_only=True) for p in paths} or {"libmcgmil.so": base}
    dev = torch.device("cuda", 0)
    N, T, L, D, C = int(os.environ.get("PROBE_N", "2048")), int(os.environ.get("PROBE_T", "100")), 512, 128, 2
    dt = torch.float32 if os.environ.get("PROBE_DTYPE", "bf16") == "f32" else torch.bfloat16
    B = int(os.environ.get("PROBE_BAGS", str(128 * 2048 // N)))
    rounds = int(os.environ.get("PROBE_ROUNDS", "5"))
    g = torch.Generator(device=dev).manual_seed(0)
    H = torch.randn(B * N, L, device=dev, generator=g).abs_().to(dt)
    offs = ops.bag_offsets_tensor([N] * B, dev)
    sd = synthetic.head_state_dict(0, L=L, D=D, C=C, shared=False)
    arrays = synthetic.head_arrays(sd, C, False)
    head = ops.HeadTensors(*[torch.from_numpy(arrays[k]).to(dev) for k in ops.HeadTensors._fields])
    packed = ops.packed_weights(head, dt)
    a = ops.make_args(H, offs, head, T, C, C, D, 0.1, 0.1, seed=42)
    a.packed_w = ctypes.c_void_p(packed.data_ptr())
    Y = torch.empty(B, T, C, device=dev)
    A = torch.empty(T * C * B * N, device=dev)
    a.Y, a.A = ctypes.c_void_p(Y.data_ptr()), ctypes.c_void_p(A.data_ptr())
    n = ctypes.c_size_t()
    _lib.check(base.mcgmil_workspace_size(ctypes.byref(a), ctypes.byref(n)), "ws")
    ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
    a.workspace, a.workspace_bytes = ctypes.c_void_p(ws.data_ptr()), n.value
    pa = ctypes.byref(a)
    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)
    F = B * flops_per_bag(N, T, L, D, C, C)

    def launch(lib, fused):
        # the path through args.flags: MCGMIL_FUSED is read once per process
        a.flags = (a.flags & ~3) | (_lib.PATH_FLAGS["fused"] if fused else _lib.PATH_FLAGS["two_kernel"])
        if fused:
            _lib.check(lib.mcgmil_gate_softmax_pool(pa, sh), "gate_softmax_pool")
        else:
            _lib.check(lib.mcgmil_gate_scores(pa, sh), "gate_scores")
            _lib.check(lib.mcgmil_softmax_pool(pa, sh), "softmax_pool")

    variants = [(name, fused) for name in libs for fused in (False, True)]
    ref = None
    equal = {}
    for name, fused in variants:                       # warm-up + bitwise check
        launch(libs[name], fused)
        torch.cuda.synchronize()
        out = (Y.clone(), A.clone())
        if ref is None:
            ref = out
        equal[(name, fused)] = bool(torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1]))
    times = {v: [] for v in variants}
    for _ in range(rounds):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            launch(libs[v[0]], v[1])
            e1.record(stream)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1))
    for v in variants:
        ms = statistics.median(times[v])
        print(json.dumps({"lib": v[0], "path": "fused" if v[1] else "two-kernel", "bags": B,
                          "ms": ms, "tflops": F / (ms * 1e-3) / 1e12, "bitwise_equal": equal[v],
                          "all_ms": [round(t, 4) for t in times[v]]}), flush=True)


if __name__ == "__main__":
    main()
