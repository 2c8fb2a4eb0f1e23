# probe_conv (config-5 bag, k = 1507) over the abvar/ builds named in $VARS, interleaved, $ROUNDS rounds
set -o pipefail
mkdir -p gpurun_out/abvar
for r in $(seq 1 ${ROUNDS:-2}); do for v in ${VARS:-base cur}; do
    MCGMIL_LIB=abvar/$v.so PROBE_K=1507 timeout -k 10 200 python scripts/probe_conv.py > gpurun_out/abvar/probe_${v}_$r.log 2>&1 || exit 1
done; done
