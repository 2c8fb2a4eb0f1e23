# Round-6 call: the N > 1 bench path with every default leg (2 ranks on cuda:0 over gloo, the
# one-GPU rehearsal of the driver's scaling run), then the config-5 kernel trace of the final tree.
set -u
timeout -k 10 600 python3 bench.py --gpus 2 --same-device --dist-backend gloo --steps 3 --warmup 1 --bags 64 --busy-seconds 2 > gpurun_out/bench_2ranks.log 2>&1 || { tail -20 gpurun_out/bench_2ranks.log; exit 1; }
grep '^{' gpurun_out/bench_2ranks.log | cut -c1-300
STEPS="profcfg5" bash scripts/gpu_round6.sh
