"""Row-owner gate kernel (mcgmil_rowgate.h, MCGMIL_GATE_ROW) on the GPU: parity against the
reference restatement (oracle/mcdo_ref.py, model.py:280-316) with the kernel's own masks, then
timing against the current kernels interleaved in one process.

  PROBE_PARITY=0   skip the parity part
  PROBE_BAGS       bags per timed launch (default 64 of N = 2048, T = 100)
  PROBE_VARIANT    "gate:path" the variant libraries (MCGMIL_PROBE_LIBS) are timed on; path "pool2" is
                   the two-kernel path through mcgmil_gate_softmax_pool
Prints one JSON line per check / variant.
"""
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def head_on(arrays, dev):
    from mcgmil.ops import HeadTensors
    return HeadTensors(*[torch.from_numpy(np.ascontiguousarray(arrays[k])).to(dev) for k in HeadTensors._fields])


def parity(dev):
    from mcgmil import ops, synthetic
    from oracle import mcdo_ref
    L = 512
    cases = [("sep_uniform", [2048, 2048], 6, False, 0.1, 0.1),
             ("shared_uniform", [2048, 2048], 6, True, 0.1, 0.1),
             ("sep_ragged", [1, 37, 200, 513, 0, 130], 5, False, 0.1, 0.5),
             ("shared_ragged", [129, 3, 640], 7, True, 0.37, 0.1),
             ("sep_p0", [300], 3, False, 0.0, 0.0),
             ("sep_p1", [100], 2, False, 1.0, 1.0)]
    ok = True
    for name, sizes, T, shared, pf, pa in cases:
        C = 2
        seed = 77
        sd = synthetic.head_state_dict(seed, L=L, C=C, shared=shared)
        Hs = [synthetic.bf16_round(synthetic.bag_features(seed + 10 + b, n, L)) for b, n in enumerate(sizes)]
        head = head_on(synthetic.head_arrays(sd, C, shared), dev)
        H = torch.from_numpy(np.concatenate(Hs)).to(dev).to(torch.bfloat16).contiguous()
        offs = ops.bag_offsets_tensor(sizes, dev)
        kw = dict(p_feat=pf, p_att=pa, seed=seed, bag_id_base=5, return_stats=True, path="two_kernel")
        row = ops.mcdo_forward(H, offs, head, T, gate="row", **kw)
        old = ops.mcdo_forward(H, offs, head, T, gate="auto", **kw)
        torch.cuda.synchronize()
        prm = mcdo_ref.HeadParams(synthetic.head_arrays(synthetic.round_state_dict_bf16(sd), C, shared))
        Y = row["Y"].cpu().numpy()
        A = ops.split_bags(row["A"].cpu(), sizes, T * C)
        dy = da = 0.0
        for b, n in enumerate(sizes):
            if n == 0:
                dy = max(dy, float(np.abs(Y[b]).max()))
                continue
            kF, kA = mcdo_ref.masks_for_bag(seed, 5 + b, T, n, L, C, pf, pa)
            Yr, Ar = mcdo_ref.mc_inference(Hs[b], prm, kF, kA, pf, pa)
            dy = max(dy, float(np.abs(Y[b] - Yr[:, 0].numpy()).max()))
            Ar = Ar[:, 0].numpy()
            da = max(da, float(np.abs(A[b].numpy().reshape(T, C, n) - Ar).max() / max(np.abs(Ar).max(), 1e-30)))
        dyo = float((row["Y"] - old["Y"]).abs().max())
        good = dy <= 1e-4 and da <= 1e-4
        ok &= good
        print(json.dumps({"check": name, "max_dY_vs_oracle": dy, "nrel_A_vs_oracle": da,
                          "max_dY_vs_old_kernel": dyo, "ok": good}), flush=True)
    # replay masks through the row kernel == its own Philox
    sizes, T = [700, 33], 4
    sd = synthetic.head_state_dict(3, L=L, C=2, shared=False)
    head = head_on(synthetic.head_arrays(sd, 2, False), dev)
    H = torch.from_numpy(np.concatenate([synthetic.bag_features(9 + b, n, L) for b, n in enumerate(sizes)])) \
        .to(dev).to(torch.bfloat16).contiguous()
    offs = ops.bag_offsets_tensor(sizes, dev)
    R = sum(sizes)
    kf = ops.feature_keep(offs, R, T, L, 0.1, 11)
    ka = ops.attention_keep(offs, R, T, 2, 0.1, 11)
    kw = dict(p_feat=0.1, p_att=0.1, seed=11, path="two_kernel", gate="row")
    a = ops.mcdo_forward(H, offs, head, T, **kw)
    b = ops.mcdo_forward(H, offs, head, T, keep_feat=kf, keep_att=ka, **kw)
    eq = bool(torch.equal(a["Y"], b["Y"]) and torch.equal(a["A"], b["A"]))
    ok &= eq
    print(json.dumps({"check": "replay_equals_philox", "bitwise": eq}), flush=True)
    return ok


def timing(dev):
    from mcgmil import _lib, ops, synthetic
    lib = _lib.load()
    # MCGMIL_PROBE_LIBS=a.so,b.so: variant builds (scripts/build_variants.sh, GATE_ONLY=1), each timed
    # with gate="row" beside the product library's default kernel
    paths = [q for q in os.environ.get("MCGMIL_PROBE_LIBS", "").split(",") if q]
    libs = {"product": lib}
    libs.update({os.path.basename(q): _lib.bind(q, mcdo_only=True, any_abi=True) for q in paths})
    N, T, L, D, C = 2048, 100, 512, 128, 2
    B = int(os.environ.get("PROBE_BAGS", "64"))
    rounds, iters = 7, int(os.environ.get("PROBE_ITERS", "3"))
    g = torch.Generator(device=dev).manual_seed(0)
    H = torch.randn(B * N, L, device=dev, generator=g).abs_().bfloat16().contiguous()
    offs = ops.bag_offsets_tensor([N] * B, dev)
    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)
    setups = {}
    for shared in (False, True):
        G = 1 if shared else C
        head = head_on(synthetic.head_arrays(synthetic.head_state_dict(0, C=C, shared=shared), C, shared), dev)
        packed = ops.packed_weights(head, torch.bfloat16)
        # PROBE_VARIANT="gate:path" times the variant libraries on that launch (default row two-kernel)
        vg, vp = os.environ.get("PROBE_VARIANT", "row:two_kernel").split(":")
        combos = [(n, vg if n != "product" else "row", vp if n != "product" else "two_kernel") for n in libs]
        combos += [("product", "auto", "two_kernel")]
        combos += [("product", "row", "fused"), ("product", "auto", "fused"), ("product", "auto", "pool2")]
        if shared:   # the tile kernels: gate_pipe_kernel / gate_fused_kernel (one pair per wave)
            combos += [("product", "pipe", "two_kernel"), ("product", "pipe", "fused")]
        for name, gate, path in combos:
            if paths and shared and os.environ.get("PROBE_SHARED", "1") == "0":
                continue
            # path "pool2": the two-kernel path through mcgmil_gate_softmax_pool (gate + softmax launches)
            a = ops.make_args(H, offs, head, T, C, G, D, 0.1, 0.1, seed=1, gate=gate,
                              path="two_kernel" if path == "pool2" else path)
            a.packed_w = ctypes.c_void_p(packed.data_ptr())
            n = ctypes.c_size_t()
            _lib.check(lib.mcgmil_workspace_size(ctypes.byref(a), ctypes.byref(n)), "ws")
            ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
            a.workspace, a.workspace_bytes = ctypes.c_void_p(ws.data_ptr()), n.value
            flops = B * T * (2 * N * L * D * 2 * G + 2 * N * D * C + 2 * N * L * C + 2 * L * C)
            Y = torch.empty(B, T, C, device=dev)
            A = torch.empty(T * C * B * N, device=dev)
            a.Y, a.A = ctypes.c_void_p(Y.data_ptr()), ctypes.c_void_p(A.data_ptr())
            setups[(shared, gate, name, path)] = (a, ws, head, packed, flops, libs[name], Y, A)
    times = {k: [] for k in setups}
    for _ in range(rounds):
        for k, (a, *_rest) in setups.items():
            lb = setups[k][5]
            fn = lb.mcgmil_gate_softmax_pool if k[3] in ("fused", "pool2") else lb.mcgmil_gate_scores
            _lib.check(fn(ctypes.byref(a), sh), "gate")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(iters):
                fn(ctypes.byref(a), sh)
            e1.record(stream)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / iters)
    for (shared, gate, name, path), ts in times.items():
        ms = statistics.median(ts)
        flops = setups[(shared, gate, name, path)][4]
        print(json.dumps({"timing": "gate_softmax_pool" if path in ("fused", "pool2") else "gate_scores", "lib": name,
                          "shared": shared, "gate": gate, "path": path, "bags": B,
                          "ms": round(ms, 4),
                          "tflops": round(flops / (ms * 1e-3) / 1e12, 1),
                          "frac": round(flops / (ms * 1e-3) / 2.5e15, 4)}), flush=True)


def main():
    from mcgmil import _lib
    _lib.load()
    dev = torch.device("cuda", 0)
    ok = True
    if os.environ.get("PROBE_PARITY", "1") != "0":
        ok = parity(dev)
    timing(dev)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
