# BN apply / vertical-pool variants (abvar/*.so): the stem tests on the column-pool build, then
# probe_bn (apply, apply + residual) and probe_stem over the builds in one process each, twice
set -o pipefail
mkdir -p gpurun_out/abbn
MCGMIL_LIB=abvar/col.so timeout -k 10 300 python -u -m pytest tests/test_gpu_stem.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/abbn/pytest_stem_col.log 2>&1 && \
for r in 1 2; do
    MCGMIL_PROBE_LIBS=abvar/u2.so,abvar/u4.so,abvar/u4b8.so,abvar/u2b2.so timeout -k 10 300 python scripts/probe_bn.py > gpurun_out/abbn/bn_$r.log 2>&1 || exit 1
    MCGMIL_PROBE_LIBS=abvar/u2.so,abvar/col.so timeout -k 10 200 python scripts/probe_stem.py > gpurun_out/abbn/stem_$r.log 2>&1 || exit 1
done
