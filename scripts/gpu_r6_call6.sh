# Round-6 call: the XCD-aware tile order on the one-bag-per-call path (B = 1), A/B in alternating
# processes (bench.py --workload single: N = 2,048 and 1,507 at T = 100 and 50).
set -u
for i in 1 2; do
  for v in xcd noxcd; do
    timeout -k 10 300 env MCGMIL_LIB=abvar/$v.so python3 bench.py --workload single --no-calibration > gpurun_out/ab_xcd_single_${v}_$i.log 2>&1 || exit 1
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/ab_xcd_single_${v}_$i.log') if l.startswith('{')][0])
print('$v', {k: round(v['gpu_ms'], 4) for k, v in d['bags'].items()}, {k: round(v['gpu_ms'], 4) for k, v in d['T50']['bags'].items()})"
  done
done
