# probe_conv (config-5 bag, k = 1507) under the default tile policy and MCGMIL_CONV_TILE=small, interleaved
set -o pipefail
mkdir -p gpurun_out/abtile
for r in 1 2; do
    PROBE_K=1507 timeout -k 10 200 python scripts/probe_conv.py > gpurun_out/abtile/default_$r.log 2>&1 || exit 1
    MCGMIL_CONV_TILE=small PROBE_K=1507 timeout -k 10 200 python scripts/probe_conv.py > gpurun_out/abtile/small_$r.log 2>&1 || exit 1
done
