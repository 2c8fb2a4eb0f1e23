# Round-6 call: conv_dma_kernel with per-piece offsets and tap masks precomputed per tile and a
# uniform wave index (LDS-DMA bases by SALU), and the halo kernel's uniform wave index: bitwise
# against the previous build on the layer-3/4 shapes, timed interleaved; then config 5 end to end,
# alternating the two builds.
set -u
timeout -k 10 600 env AB_LIBS=abvar/old.so,abvar/new.so,abvar/old.so,abvar/new.so python -u scripts/ab_conv_libs.py > gpurun_out/ab_conv_tapmask.log 2>&1; rc=$?
grep -h "layers_3_4\|bitwise_equal_all" gpurun_out/ab_conv_tapmask.log
[ $rc -le 1 ] || exit $rc
for i in 1 2; do
  for v in old new; do
    timeout -k 10 400 env MCGMIL_LIB=abvar/$v.so python3 bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline --no-calibration > gpurun_out/ab_cfg5_${v}_$i.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab_cfg5_${v}_$i.log') if l.startswith('{')][0]); print('$v', round(d['value']), {k: round(x, 3) for k, x in d['config']['stage_ms'].items()})"
  done
done
