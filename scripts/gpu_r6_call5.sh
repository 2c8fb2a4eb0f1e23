# Round-6 call: XCD-aware tile order of the two-kernel gate launches, A/B in alternating processes
# (config 4 ragged batch; shared heads), then config 4's traffic with the new order.
set -u
for i in 1 2; do
  for v in xcd noxcd; do
    timeout -k 10 300 env MCGMIL_LIB=abvar/$v.so python3 bench.py --workload cfg4 --steps 5 --warmup 2 --busy-seconds 4 --no-cpu-baseline --no-calibration > gpurun_out/ab_xcd_cfg4_${v}_$i.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_xcd_cfg4_${v}_$i.log') if l.startswith('{')][0]); print('$v', d['value'], d['roofline']['kernel_ms'], d['roofline']['clock_mhz'])"
  done
done
for i in 1 2; do
  for v in xcd noxcd; do
    timeout -k 10 300 env MCGMIL_LIB=abvar/$v.so python3 bench.py --shared 1 --steps 10 --warmup 2 --busy-seconds 4 --no-cpu-baseline --no-calibration --no-secondary > gpurun_out/ab_xcd_shared_${v}_$i.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_xcd_shared_${v}_$i.log') if l.startswith('{')][0]); print('shared $v', d['value'], d['roofline']['kernel_ms'], d['roofline']['clock_mhz'])"
  done
done
STEPS="pmc4" bash scripts/gpu_round6.sh
