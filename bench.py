"""Headline benchmark: MCDO gated-attention MIL inference on MI355X.

Metric (BASELINE.json): bags/sec x MCDO-samples (T=100) at N=2048, d=512 -- BASELINE config 3
(N=2048 instances/bag, L=d=512, D=128, C=2 heads, separate attention as config.yml:8, T=100,
bf16 operands, fp32 accumulate / softmax / outputs). A step = one pass of the hot path over one
batch of --bags synthetic bags per GPU already resident in HBM: ONE launch of gate_fused_kernel
(all T samples' gate scores with in-register Philox masks, softmax over instances and attention
pooling; the two-kernel path gate_pipe_kernel + softmax_pool_kernel for batches too small to
fill the GPU region by region) + per-bag attention mean/var, and for N > 1 GPUs the gather of
the per-bag predictions Y[T, C] to every rank (weak scaling: every rank owns --bags bags).

Prints ONE JSON line (rank 0). `roofline` prices the dominant kernel (the gate kernel) with the
ALGORITHMIC FLOPs of the literal reference computation against the bf16 dense
MFMA peak; its time comes from HIP events around that kernel on the launch stream.
`cpu_baseline` times the reference op sequence (oracle/mcdo_ref.py, torch CPU, with its own
dropout RNG) on a bounded sample of the same workload on this host.
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "montecarlo-gated-mil_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "bags/sec × MCDO-samples (T=100) at N=2048,d=512; 1/2/4/8-GPU + %HBM roofline"
PEAK_TFLOPS = {"bf16": 2500.0, "f32": 157.3}   # MI355X dense MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
MAX_CLOCK_MHZ = 2400.0                          # the clock the spec peaks are quoted at


def flops_per_bag(N, T, L, D, C, G):
    # T * [2*N*L*D*2G + 2*N*D*C + 2*N*L*C + 2*L*C]
    return T * (2 * N * L * D * 2 * G + 2 * N * D * C + 2 * N * L * C + 2 * L * C)


def bytes_per_bag(N, T, L, C, esize):
    # features read once + A[T,C,N] written + Y[T,C] written (weights once per launch, added below)
    return N * L * esize + 4 * T * C * N + 4 * T * C


def measured_traffic(N, T, B, dtype, shared, path_kind):
    """HBM bytes per gate launch from the committed rocprofv3 PMC passes (profiles/*/
    gate_traffic*.json, newest round first) when they were taken on this exact workload and
    launch path ("fused": gate_fused_kernel; "pipe": gate_pipe_kernel). N is "U(256,2048)" for
    config 4's ragged batch."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "gate_traffic*.json")),
                       reverse=True):
        t = json.load(open(path))
        if t.get("config") == {"bags": B, "N": N, "T": T, "dtype": dtype, "shared": shared} and \
                t.get("path", "pipe") == path_kind:
            return t["hbm_bytes_per_launch"], os.path.relpath(path, REPO)
    return None, None


def measured_grbm_clock(workload, kernel):
    """The product launch's clock from the newest committed GRBM pass of this workload
    (profiles/r*/grbm_clock_<workload>.json, scripts/grbm_clock.py: GRBM_GUI_ACTIVE / 8 / dispatch
    wall, median over the timed dispatches of `kernel`, the unprobed instantiation)."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", f"grbm_clock_{workload}.json")), reverse=True):
        for name, rec in json.load(open(path)).items():
            if kernel in name and not name.endswith("true>(mcgmil::GateParams)") and "Lb1EEEv" not in name:
                return rec["grbm_clock_mhz_median"], os.path.relpath(path, REPO)
    return None, None


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores():
    """The CPUs this process may run on: its affinity mask, capped by the cgroup (v2 cpu.max or
    v1 cfs quota) CPU quota when there is one. Returns (count, provenance dict)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    n = aff if quota is None else max(1, min(aff, int(quota)))
    return n, {"affinity_cpus": aff, "cgroup_cpu_quota": quota, "os_cpu_count": os.cpu_count()}


def cpu_baseline(N, T, L, D, C, shared, budget_s):
    """The reference CPU path (torch op sequence incl. dropout RNG), bounded sample, on every CPU
    this process may use (affinity, capped by the cgroup quota) and on one thread (BASELINE.md's
    plan)."""
    from oracle import mcdo_ref
    from mcgmil import synthetic
    arrays = synthetic.head_arrays(synthetic.head_state_dict(0, L=L, D=D, C=C, shared=shared), C, shared)
    prm = mcdo_ref.HeadParams(arrays)
    H = synthetic.bag_features(42, N, L)

    def timed(budget, max_bags):
        with torch.no_grad():
            mcdo_ref.mc_inference_torch_rng(H, prm, T, 0.1, 0.1)   # warm-up
            n, t0 = 0, time.perf_counter()
            while True:
                mcdo_ref.mc_inference_torch_rng(H, prm, T, 0.1, 0.1)
                n += 1
                el = time.perf_counter() - t0
                if el >= budget or n >= max_bags:
                    return n, el

    before = torch.get_num_threads()
    threads, prov = host_cores()
    torch.set_num_threads(threads)
    try:
        n, el = timed(budget_s, 50)
        torch.set_num_threads(1)
        n1, el1 = timed(budget_s / 3, 10)
    finally:
        torch.set_num_threads(before)
    model = cpu_model()
    return {"value": n * T / el, "unit": "bag-samples/s", "cores": threads, "kind": "port",
            "cpu_model": model, "cores_provenance": prov,
            "single_thread": {"value": n1 * T / el1, "unit": "bag-samples/s", "cores": 1,
                              "ms_per_bag": el1 * 1e3 / n1, "bags": n1},
            "sample": f"{n} bags of N={N}, T={T}, fp32, {'shared' if shared else 'separate'} "
                      f"attention, torch {torch.__version__} CPU, {threads} threads on {model}, "
                      f"{el * 1e3 / n:.1f} ms/bag; 1 thread: {n1} bags, {el1 * 1e3 / n1:.1f} ms/bag"}


def spawn_ranks(n):
    """`bench.py --gpus N` outside a launcher: start N rank processes through torch.distributed.run
    (one per GPU, backend nccl = RCCL) and return their exit code. Runs before this process
    touches the GPU, and starts the ranks as children (no exec)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)]
    return subprocess.call(cmd + sys.argv[1:])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    # 512 bags of N=2048 per GPU per step: ~57 ms of kernels, so the driver's 20 timed steps
    # span > 1 s (a 16-bag step is 1.8 ms; the workload per bag is the same)
    ap.add_argument("--bags", type=int, default=512, help="bags per GPU per step")
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--T", type=int, default=100)
    ap.add_argument("--dtype", choices=["bf16", "f32"], default="bf16")
    ap.add_argument("--shared", type=int, default=0)
    ap.add_argument("--workload", choices=["cfg3", "cfg4", "cfg5", "single"], default="cfg3",
                    help="cfg3: --bags bags of N=--n per GPU (weak scaling, the headline); "
                         "cfg4: 4096 bags N~U(256,2048) LPT-sharded over the GPUs (strong scaling); "
                         "cfg5: end-to-end image -> patcher -> ResNet-18 -> head -> maps (bench_cfg5.py); "
                         "single: one bag per call through the drop-in module (infer.py:187-191)")
    ap.add_argument("--features", choices=["bf16", "fp32"], default="bf16",
                    help="cfg5 only: precision of the instances / ResNet / head operands")
    ap.add_argument("--dist-backend", default="nccl", help=argparse.SUPPRESS)   # rehearsal: gloo
    ap.add_argument("--same-device", action="store_true", help=argparse.SUPPRESS)  # ranks on cuda:0
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--busy-seconds", type=float, default=12.0,
                    help="keep stepping (untimed) after the warm-up until the GPU has been busy this long")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the fp32 reference-precision and single-bag lines")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-calibration", action="store_true",
                    help="skip the MFMA ceiling calibration (roofline.measured_peak_tflops)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            return spawn_ranks(args.gpus)
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE="
              f"{os.environ['WORLD_SIZE']} ranks", file=sys.stderr)
        return 2
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", 0 if args.same_device else local)
    torch.cuda.set_device(dev)          # before the process group, so RCCL binds this rank's GPU
    if world > 1:
        dist.init_process_group(args.dist_backend)

    if args.workload == "cfg5":
        import bench_cfg5
        from mcgmil import _lib
        _lib.load()
        if not args.no_calibration:
            CALIB["bf16" if args.features == "bf16" else "f32"] = \
                mfma_calibration(dev, "bf16" if args.features == "bf16" else "f32")
        out = bench_cfg5.run(args, world, rank, dev, PEAK_TFLOPS["bf16"],
                             calib=lambda a, dt: vs_measured(a, dt))
        if rank == 0:
            print(json.dumps(out))
        if world > 1:
            dist.destroy_process_group()
        return 0

    from mcgmil import _lib

    _lib.load()
    if args.workload == "single":
        if not args.no_calibration:
            CALIB["bf16"] = mfma_calibration(dev, "bf16")
        out = single_bag_line(args, dev)
        print(json.dumps(out))
        return 0

    N, T, L, D, C = args.n, args.T, 512, 128, 2
    G = 1 if args.shared else C
    if args.workload == "cfg4":
        # BASELINE config 4: 4096 bags, N_b = rng(0).integers(256, 2049, 4096), sharded LPT
        import numpy as np
        from mcgmil.shard import lpt_assign
        all_sizes = np.random.default_rng(0).integers(256, 2049, 4096).tolist()
        mine = lpt_assign([float(n) * T for n in all_sizes], world)[rank]
        sizes = [all_sizes[b] for b in mine]
        ids = mine
        total_bags = len(all_sizes)
    else:
        sizes = [N] * args.bags
        ids = list(range(rank * args.bags, (rank + 1) * args.bags))
        total_bags = world * args.bags

    # headline: W warm-up steps, then untimed steps until the GPU has been busy --busy-seconds
    # (the driver's utilisation sampler polls every few seconds), then K timed steps
    r = measure_batch(sizes, ids, T, args.dtype, bool(args.shared), dev, world, args.steps,
                      args.warmup, busy_s=args.busy_seconds, gather=True, seed_rank=rank)
    el, gate_ms, fused, nreg, nbytes_packed = r["el"], r["gate_ms"], r["fused"], r["regions"], r["packed_bytes"]
    # the box's own MFMA ceiling, measured right after the headline's timed steps (chip under load)
    if not args.no_calibration:
        CALIB["bf16"] = mfma_calibration(dev, "bf16")
        if world == 1 and args.workload == "cfg3" and not args.no_secondary:
            CALIB["f32"] = mfma_calibration(dev, "f32")
    esize = 2 if args.dtype == "bf16" else 4
    total_bag_samples = total_bags * T * args.steps
    value = total_bag_samples / el
    F = sum(flops_per_bag(n, T, L, D, C, G) for n in sizes)
    achieved = F / (gate_ms * 1e-3) / 1e12
    hbm_bytes = sum(bytes_per_bag(n, T, L, C, esize) for n in sizes) + nbytes_packed
    hbm_gbs = hbm_bytes / (gate_ms * 1e-3) / 1e9
    traffic, traffic_src = measured_traffic(N if args.workload == "cfg3" else "U(256,2048)", T, len(sizes),
                                            args.dtype, args.shared, "fused" if fused else "pipe")

    # the reference's precision at the metric's shape (model.py:280-316 computes in fp32), and the
    # one-bag-per-call caller (infer.py:187-191): N = 1 only, after the headline's timed steps
    fp32_line = single = shared_line = None
    if world == 1 and args.workload == "cfg3" and not args.no_secondary:
        if not args.shared:
            shared_line = shared_secondary(args, dev)
        fp32_line = fp32_secondary(args, dev)
        single = single_bag_line(args, dev, quiet=True)

    if rank == 0:
        # the CPU baseline is a rank-0, N=1 figure: at N > 1 it would only hold the other ranks
        cpu = None if args.no_cpu_baseline or world > 1 else cpu_baseline(N, T, L, D, C, bool(args.shared),
                                                                          args.cpu_budget)
        kernel = (f"gate_fused_kernel (gate scores + softmax + pooling, one launch, {nreg} regions)"
                  if fused else "gate_pipe_kernel")
        out = {
            "metric": METRIC, "value": value, "unit": "bag-samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "weak" if args.workload == "cfg3" else "strong",
            "vs_baseline": None,
            "dtype": args.dtype, "data": "synthetic (|N(0,1)| features, random-init head)",
            "config": {"workload": (f"BASELINE config 3: N={N} instances/bag" if args.workload == "cfg3"
                                    else "BASELINE config 4: 4096 bags, N~U(256,2048)") +
                                   f", d={L}, D={D}, C={C}, T={T} MCDO samples, "
                                   f"{'shared' if args.shared else 'separate'} attention, "
                                   f"{args.dtype} operands / fp32 accumulate",
                       "bags_per_gpu_per_step": len(sizes), "global_batch_bags": total_bags,
                       "rows_per_gpu": sum(sizes), "N": N if args.workload == "cfg3" else "U(256,2048)",
                       "L": L, "D": D, "C": C, "T": T,
                       "parallelism": f"bags over {world} GPU(s), LPT, RCCL all_gather of Y"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_TFLOPS[args.dtype],
                         "unit": "TFLOP/s", "frac": achieved / PEAK_TFLOPS[args.dtype],
                         "traffic": traffic, "traffic_unit": "HBM bytes per launch",
                         "traffic_source": traffic_src, "kernel": kernel,
                         # what the HIP events bracket: the whole path (gate scores + softmax +
                         # pooling) when fused, the gate GEMM kernel alone otherwise
                         "timed_path": "fused: gate+softmax+pooling" if fused else "two-kernel: gate only",
                         "kernel_ms": gate_ms, "algorithmic_tflop_per_launch": F / 1e12,
                         **at_clock(achieved, PEAK_TFLOPS[args.dtype], r["clock"], args.dtype),
                         **grbm_keys(achieved, PEAK_TFLOPS[args.dtype], args.workload, fused)},
            "roofline_hbm": {"achieved": hbm_gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": hbm_gbs / PEAK_HBM_GBS,
                             "algorithmic_bytes_per_launch": hbm_bytes},
            "busy_warmup_s": r["busy_s"],
            # the same K steps timed right after the W warm-up, before the --busy-seconds of load
            # (a cooler chip holds a higher clock); value / roofline above are the steady state
            "cold_start": None if r["cold"] is None else {
                "value": total_bag_samples / r["cold"][0], "ms_per_step": r["cold"][0] * 1e3 / args.steps,
                "kernel_ms": r["cold"][1],
                "frac": F / (r["cold"][1] * 1e-3) / 1e12 / PEAK_TFLOPS[args.dtype]},
            "mfma_calibration": {k: v for k, v in CALIB.items()},
            "shared_heads": shared_line,
            "fp32_reference_precision": fp32_line,
            "single_bag": single,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()
    return 0


def _head(dev, shared, L=512, D=128, C=2):
    from mcgmil import ops, synthetic
    sd = synthetic.head_state_dict(0, L=L, D=D, C=C, shared=shared)
    arrays = synthetic.head_arrays(sd, C, shared)
    return ops.HeadTensors(*[torch.from_numpy(arrays[k]).to(dev) for k in ops.HeadTensors._fields])


def measure_batch(sizes, ids, T, dtype, shared, dev, world, steps, warmup, busy_s=0.0, gather=False,
                  seed_rank=0, path="auto"):
    """Time `steps` passes of the hot path over one batch of bags resident in HBM: the gate
    launch(es) through the C ABI, per-bag statistics, and (N > 1 GPUs, gather) the all_gather of
    Y. HIP events on the launch stream bracket the gate kernel (the fused launch when it runs).
    Returns wall seconds (max over ranks), the events' mean ms, the launch path."""
    from mcgmil import _lib, ops
    lib = _lib.load()
    L, D, C = 512, 128, 2
    G = 1 if shared else C
    dt = torch.bfloat16 if dtype == "bf16" else torch.float32
    B, rows = len(sizes), sum(sizes)
    head = _head(dev, shared)
    g = torch.Generator(device=dev).manual_seed(1000 + seed_rank)
    H = torch.randn(rows, L, device=dev, generator=g).abs_().to(dt).contiguous()
    offs = ops.bag_offsets_tensor(sizes, dev)
    bag_ids = torch.tensor(ids, dtype=torch.int32, device=dev)
    packed = ops.packed_weights(head, dt)
    a = ops.make_args(H, offs, head, T, C, G, D, 0.1, 0.1, seed=42, bag_ids=bag_ids, path=path)
    a.packed_w = ctypes.c_void_p(packed.data_ptr())
    Y = torch.empty(B, T, C, device=dev)
    A = torch.empty(T * C * rows, device=dev)
    Am = torch.empty(C * rows, device=dev)
    Av = torch.empty(C * rows, device=dev)
    a.Y, a.A = ctypes.c_void_p(Y.data_ptr()), ctypes.c_void_p(A.data_ptr())
    a.A_mean, a.A_var = ctypes.c_void_p(Am.data_ptr()), ctypes.c_void_p(Av.data_ptr())
    n = ctypes.c_size_t()
    _lib.check(lib.mcgmil_workspace_size(ctypes.byref(a), ctypes.byref(n)), "workspace_size")
    ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
    a.workspace, a.workspace_bytes = ctypes.c_void_p(ws.data_ptr()), n.value
    pa = ctypes.byref(a)
    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)
    gat = None
    if gather and world > 1:
        pad = torch.zeros(1, dtype=torch.int64, device=dev) + B
        dist.all_reduce(pad, op=dist.ReduceOp.MAX)
        Ypad = torch.zeros(int(pad), T, C, device=dev)
        gat = [torch.empty_like(Ypad) for _ in range(world)]

    # ONE launch (gate_fused_kernel: gate scores + softmax + pooling) when the batch is large
    # enough, else gate_pipe_kernel + softmax_pool_kernel; the events bracket the gate kernel
    regions = ctypes.c_int64()
    _lib.check(lib.mcgmil_fused_regions(pa, ctypes.byref(regions)), "fused_regions")
    fused = regions.value > 0

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        if fused:
            _lib.check(lib.mcgmil_gate_softmax_pool(pa, sh), "gate_softmax_pool")
        else:
            _lib.check(lib.mcgmil_gate_scores(pa, sh), "gate_scores")
        if ev is not None:
            ev[1].record(stream)
        if not fused:
            _lib.check(lib.mcgmil_softmax_pool(pa, sh), "softmax_pool")
        _lib.check(lib.mcgmil_bag_stats(pa, sh), "bag_stats")
        if gat is not None:          # per-bag predictions to every rank (RCCL over xGMI)
            Ypad[:B].copy_(Y)
            dist.all_gather(gat, Ypad)

    def timed_pass():
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(steps)]
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(evs[i])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        gate_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / steps
        if world > 1:
            t = torch.tensor([el, gate_ms], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el, gate_ms = float(t[0]), float(t[1])
        return el, gate_ms

    t_busy = time.perf_counter()
    for _ in range(warmup):
        step()
    extra = 0
    cold = None
    if busy_s > 0:
        # the same K steps right after the W warm-up, before the GPU has been loaded for long: the
        # chip's clock under this load settles lower within seconds, so this
        # pass is reported beside the steady-state one, never as the value
        cold = timed_pass()
        # untimed steps until the GPU has been busy busy_s seconds; the count is agreed over the
        # ranks (each step ends in a collective)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        per = (time.perf_counter() - t1) / 2
        extra = max(0, math.ceil((busy_s - (time.perf_counter() - t_busy)) / max(per, 1e-4)))
        if world > 1:
            t = torch.tensor([extra], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            extra = int(t)
        for _ in range(extra):
            step()
    torch.cuda.synchronize()
    busy = time.perf_counter() - t_busy
    el, gate_ms = timed_pass()
    # the clock the gate launch runs at: the third of five back-to-back (untimed) steps right after
    # the timed ones, its workgroups stamping s_memtime / s_memrealtime at start and end
    # (MCGMIL_CLOCK_PROBE). Not the first step after a synchronize: the chip raises its clock in the
    # idle gap, and such a launch read ~7% above the steady state that GRBM_GUI_ACTIVE / 8 / wall
    # gives for the timed launches (profiles/r06/grbm_clock.json)
    rec = ops.clock_record(dev)
    for i in range(5):
        if i == 2:
            a.debug, a.flags = ctypes.c_void_p(rec.data_ptr()), a.flags | _lib.CLOCK_PROBE
        step()
        if i == 2:
            a.debug, a.flags = None, a.flags & ~_lib.CLOCK_PROBE
    torch.cuda.synchronize()
    clock = ops.clock_mhz(rec)
    if world > 1 and clock is not None:
        t = torch.tensor([clock["median"]], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)     # the slowest rank's clock
        clock["median_min_over_ranks"] = float(t)
    return {"el": el, "gate_ms": gate_ms, "fused": fused, "regions": regions.value,
            "packed_bytes": packed.numel(), "busy_s": busy, "busy_extra_steps": extra, "cold": cold,
            "clock": clock}


def at_clock(achieved, peak, clock, dtype="bf16"):
    """The roofline's clock keys: the shader clock the launch ran at and the fraction of the peak
    scaled to that clock (the spec peak assumes MAX_CLOCK_MHZ), plus the fractions of the box's
    measured MFMA ceiling (vs_measured)."""
    if clock is None:
        return {"clock_mhz": None, "frac_at_clock": None, **vs_measured(achieved, dtype)}
    return {"clock_mhz": round(clock["median"], 1), "clock_mhz_p10_p90": [round(clock["p10"], 1), round(clock["p90"], 1)],
            "frac_at_clock": achieved / (peak * clock["median"] / MAX_CLOCK_MHZ),
            "clock_source": f"in-kernel s_memtime/s_memrealtime x 100 MHz, median of {clock['workgroups']} "
                            f"workgroups of one probed launch, the 3rd of 5 back-to-back steps after the timed ones",
            **vs_measured(achieved, dtype, clock["median"])}


def mfma_calibration(dev, dtype, warm_s=2.0, timed_s=1.0, launch_ms=20.0):
    """The MFMA rate this box sustains (include/mcgmil_calib.h): a bare loop at the gate kernels'
    occupancy (one 512-thread workgroup per CU, two waves per SIMD), B fragments re-read from LDS
    by ds_read_b128 each step, random full-range operands. >= warm_s seconds of back-to-back
    launches first (the chip settles its clock under load, MI355X_MICROARCH.md 'DVFS give-back'
    item 6), then timed_s seconds timed by HIP events on the launch stream, then one launch
    clock-probed (s_memtime / s_memrealtime per workgroup)."""
    from mcgmil import _lib, ops
    lib = _lib.load()
    code = _lib.MCGMIL_BF16 if dtype == "bf16" else _lib.MCGMIL_F32
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    sink = torch.empty(cus * 512, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)
    fps = lib.mcgmil_mfma_calib_flops_per_step(code)

    def launch(steps, seed=1, rec=None):
        _lib.check(lib.mcgmil_mfma_calib(code, cus, steps, seed, ctypes.c_void_p(sink.data_ptr()),
                                         None if rec is None else ctypes.c_void_p(rec.data_ptr()), sh),
                   "mfma_calib")
    # size one launch to ~launch_ms from a short probe
    launch(200)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    launch(2000)
    e1.record(stream)
    torch.cuda.synchronize()
    steps = max(100, int(2000 * launch_ms / max(e0.elapsed_time(e1), 1e-3)))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        for i in range(10):
            launch(steps, seed=i + 2)
        torch.cuda.synchronize()
    n = max(5, int(timed_s * 1e3 / launch_ms))
    e0.record(stream)
    for i in range(n):
        launch(steps, seed=100 + i)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    rec = ops.clock_record(dev)
    for i in range(5):            # the probed launch in the middle of back-to-back launches
        launch(steps, seed=7 + i, rec=rec if i == 2 else None)
    torch.cuda.synchronize()
    clock = ops.clock_mhz(rec)
    tflops = fps * cus * steps / (ms * 1e-3) / 1e12
    return {"tflops": tflops, "clock_mhz": None if clock is None else round(clock["median"], 1),
            "launch_ms": ms, "launches_timed": n, "warm_s": round(time.perf_counter() - t0, 2),
            "workgroups": cus, "steps_per_launch": steps,
            "loop": ("v_mfma_f32_16x16x32_bf16 x 32 per wave-step" if dtype == "bf16"
                     else "v_mfma_f32_16x16x4_f32 x 128 per wave-step") +
                    ", 2 waves/SIMD, B via ds_read_b128 from LDS, random operands in [-1, 1)"}


CALIB = {}      # dtype -> mfma_calibration() of this process (bench.py fills it once per run)


def vs_measured(achieved, dtype, clock_mhz=None):
    """Roofline keys against the box's measured MFMA ceiling: frac_of_measured = achieved / the
    calibration loop's TFLOP/s (both wall rates on this GPU, this process); with the kernel's own
    clock, per_clock_frac_of_measured = (achieved / its clock) / (calibration / its clock)."""
    c = CALIB.get(dtype)
    if not c:
        return {"measured_peak_tflops": None, "frac_of_measured": None}
    out = {"measured_peak_tflops": round(c["tflops"], 1), "measured_peak_clock_mhz": c["clock_mhz"],
           "frac_of_measured": achieved / c["tflops"],
           "measured_peak_source": "mcgmil_mfma_calib (include/mcgmil_calib.h), same process, "
                                   f"{c['warm_s']} s of back-to-back launches before timing"}
    if clock_mhz and c["clock_mhz"]:
        out["per_clock_frac_of_measured"] = (achieved / clock_mhz) / (c["tflops"] / c["clock_mhz"])
    return out


def grbm_keys(achieved, peak, workload, fused):
    """The cross-check of the in-kernel clock: the probed launch runs the PROBE instantiation, whose
    code differs from the product kernel's (measured 11% slower, at a ~9% higher clock under
    rocprofv3, profiles/r06/grbm_clock_cfg3.json), so frac_at_clock uses a clock the product launch
    does not hold. The committed GRBM pass gives the product dispatches' own clock."""
    mhz, src = measured_grbm_clock(workload, "gate_fused_kernel" if fused else "gate_pipe_kernel")
    if mhz is None:
        return {}
    out = {"clock_mhz_grbm": mhz, "frac_at_grbm_clock": achieved / (peak * mhz / MAX_CLOCK_MHZ),
           "grbm_source": f"{src} (GRBM_GUI_ACTIVE / 8 / dispatch wall, timed dispatches, a committed "
                          f"rocprofv3 pass of this workload)"}
    c = CALIB.get("bf16" if peak == PEAK_TFLOPS["bf16"] else "f32")
    if c and c.get("clock_mhz"):
        out["per_clock_frac_of_measured_grbm"] = (achieved / mhz) / (c["tflops"] / c["clock_mhz"])
    return out


def shared_secondary(args, dev, steps=10, warmup=3):
    """The reference constructor's default head layout (shared_attention=True, model.py:144,
    182-184: one gate pair feeds every class) on the headline's workload: --bags bags of N=--n,
    T=--T, bf16, its own algorithmic FLOPs (G = 1) against the bf16 peak."""
    N, T, L, D, C = args.n, args.T, 512, 128, 2
    bags = args.bags
    r = measure_batch([N] * bags, list(range(bags)), T, args.dtype, True, dev, 1, steps, warmup)
    F = bags * flops_per_bag(N, T, L, D, C, 1)
    ach = F / (r["gate_ms"] * 1e-3) / 1e12
    return {"metric": "bag-samples/s, shared attention (the reference constructor's default)",
            "value": bags * T * steps / r["el"], "unit": "bag-samples/s", "dtype": args.dtype,
            "steps": steps, "warmup": warmup, "ms_per_step": r["el"] * 1e3 / steps,
            "config": f"{bags} bags of N={N}, d={L}, D={D}, C={C}, T={T}, shared attention, {args.dtype}",
            "gflop_per_bag": flops_per_bag(N, T, L, D, C, 1) / 1e9,
            "roofline": {"bound": "mfma", "achieved": ach, "peak": PEAK_TFLOPS[args.dtype], "unit": "TFLOP/s",
                         "frac": ach / PEAK_TFLOPS[args.dtype], "kernel_ms": r["gate_ms"],
                         "kernel": (f"fused launch ({r['regions']} regions)" if r["fused"]
                                    else "gate kernel (two-kernel path)"),
                         "timed_path": "fused: gate+softmax+pooling" if r["fused"] else "two-kernel: gate only",
                         "algorithmic_tflop_per_launch": F / 1e12,
                         **at_clock(ach, PEAK_TFLOPS[args.dtype], r["clock"])}}


def fp32_secondary(args, dev, bags=64, steps=10, warmup=2):
    """The same hot path at the reference's precision (fp32 operands and accumulation, model.py:
    280-316): `bags` bags of N=--n, T=--T, separate heads, priced against the fp32 MFMA peak."""
    N, T, L, D, C = args.n, args.T, 512, 128, 2
    r = measure_batch([N] * bags, list(range(bags)), T, "f32", False, dev, 1, steps, warmup)
    F = bags * flops_per_bag(N, T, L, D, C, C)
    ach = F / (r["gate_ms"] * 1e-3) / 1e12
    return {"metric": "bag-samples/s, fp32 operands (the reference precision)",
            "value": bags * T * steps / r["el"], "unit": "bag-samples/s", "dtype": "f32",
            "steps": steps, "warmup": warmup, "ms_per_step": r["el"] * 1e3 / steps,
            "config": f"{bags} bags of N={N}, d={L}, D={D}, C={C}, T={T}, separate attention, fp32",
            "roofline": {"bound": "mfma", "achieved": ach, "peak": PEAK_TFLOPS["f32"], "unit": "TFLOP/s",
                         "frac": ach / PEAK_TFLOPS["f32"], "kernel_ms": r["gate_ms"],
                         "kernel": (f"gate_fused_kernel ({r['regions']} regions)" if r["fused"]
                                    else "gate_pipe_kernel (fp32 MFMA 16x16x4)"),
                         "timed_path": "fused: gate+softmax+pooling" if r["fused"] else "two-kernel: gate only",
                         "algorithmic_tflop_per_launch": F / 1e12,
                         **at_clock(ach, PEAK_TFLOPS["f32"], r["clock"], "f32")}}


def _single_bag_entry(m, dev, N, T, L, D, C):
    g = torch.Generator(device=dev).manual_seed(7)
    H = torch.randn(N, L, device=dev, generator=g).abs_().bfloat16()
    call = lambda i: m.mc_inference_features(H, T=T, seed=100 + i, return_stats=True)  # noqa: E731
    for i in range(5):
        call(i)
    torch.cuda.synchronize()
    reps = 50
    # host time per call, nothing queued
    t0 = time.perf_counter()
    for i in range(reps):
        call(i)
    host = (time.perf_counter() - t0) / reps
    torch.cuda.synchronize()
    # device time per call: a busy kernel queued ahead (~0.1 s), so the host enqueues every
    # call before the GPU reaches them
    torch.cuda._sleep(int(2e8))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = torch.cuda.current_stream(dev)
    e0.record(s)
    for i in range(reps):
        call(i)
    e1.record(s)
    torch.cuda.synchronize()
    gpu = e0.elapsed_time(e1) / reps
    lat = []
    for i in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        call(i)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
    F = flops_per_bag(N, T, L, D, C, C)
    ach = F / (gpu * 1e-3) / 1e12
    return {"gpu_ms": gpu, "host_ms": host * 1e3, "sync_ms": sorted(lat)[len(lat) // 2] * 1e3,
            "achieved_tflops": ach, "frac": ach / PEAK_TFLOPS["bf16"],
            "bag_samples_per_s": T / (gpu * 1e-3), **vs_measured(ach, "bf16")}


def single_bag_line(args, dev, quiet=False):
    """The per-bag caller (infer.py:187-191 calls mc_inference once per bag): the drop-in module's
    mc_inference_features on ONE bag per call, N = --n (and config 5's k = 1,507), T = --T, bf16
    operands, separate heads, A_mean/A_var/P_mean included. Reports
      gpu_ms   device time per call: events around a run of calls queued behind a busy GPU, so
               host overhead is hidden and only kernels + on-device launch gaps count;
      host_ms  host time per call (the Python/ctypes path, no synchronisation);
      sync_ms  one call from an idle GPU to its results on the host side (latency).
    """
    from mcgmil import MultiHeadGatedAttentionMIL, synthetic
    L, D, C, T = 512, 128, 2, args.T
    m = MultiHeadGatedAttentionMIL(pretrained=False, shared_attention=False)
    sd = synthetic.head_state_dict(0, L=L, D=D, C=C, shared=False)
    own = m.state_dict()
    m.load_state_dict({k: torch.from_numpy(v).reshape(own[k].shape) for k, v in sd.items()}, strict=False)
    m.compute_dtype = torch.bfloat16
    m = m.to(dev).eval()
    by_t = {}
    # the headline's T and the reference caller's own sample count (infer.py:191 passes
    # N=config['N'], config.yml:12 sets 50)
    for T in dict.fromkeys((args.T, 50)):
        res = by_t[T] = {}
        for N in (args.n, 1507):
            res[f"N{N}"] = _single_bag_entry(m, dev, N, T, L, D, C)
    out = {"metric": "one bag per call (infer.py:187-191): head device time per bag",
           "unit": "ms", "dtype": "bf16", "T": args.T, "bags": by_t[args.T],
           **{f"T{t}": {"T": t, "bags": r} for t, r in by_t.items() if t != args.T},
           "path": "MultiHeadGatedAttentionMIL.mc_inference_features -> mcgmil_mcdo_forward "
                   "(two-kernel path + bag statistics)"}
    return out


if __name__ == "__main__":
    sys.exit(main())
