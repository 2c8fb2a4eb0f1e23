# Round-6 call: the one-bag-per-call path with the two-workgroups-per-CU tile (MCGMIL_GATE=pp:
# gate_pp_kernel, 64-row tiles for separate heads) against the default gate_pipe_kernel, alternating.
set -u
for i in 1 2; do
  for g in pipe pp; do
    timeout -k 10 300 env MCGMIL_GATE=$g python3 bench.py --workload single --no-calibration > gpurun_out/ab_single_gate_${g}_$i.log 2>&1 || exit 1
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/ab_single_gate_${g}_$i.log') if l.startswith('{')][0])
print('$g', {k: round(v['gpu_ms'], 4) for k, v in d['bags'].items()}, {k: round(v['gpu_ms'], 4) for k, v in d['T50']['bags'].items()})"
  done
done
