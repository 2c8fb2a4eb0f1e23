# A/B of two conv/stem builds (abvar/base.so vs abvar/$VAR.so): bitwise conv/feature/stem tests on the tree
# build, probe_conv and probe_stem interleaved, config 5, then an LDS counter pass on the probe
set -o pipefail
VAR=${VAR:-new}
mkdir -p gpurun_out/abconv
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_features.py tests/test_gpu_stem.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/abconv/pytest.log 2>&1 && \
for r in 1 2; do for v in base $VAR; do MCGMIL_LIB=abvar/$v.so PROBE_K=916 timeout -k 10 200 python scripts/probe_conv.py > gpurun_out/abconv/probe_${v}_$r.log 2>&1 || exit 1; done; done && \
for r in 1 2; do for v in base $VAR; do MCGMIL_LIB=abvar/$v.so timeout -k 10 200 python scripts/probe_stem.py > gpurun_out/abconv/stem_${v}_$r.log 2>&1 || exit 1; done; done && \
timeout -k 10 400 python bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/abconv/cfg5.log 2>&1 && \
PMC_OUT=gpurun_out/abconv/pmc PROBE_K=1507 PMC_CMD="python3 scripts/probe_conv.py" PASSES="lds" timeout -k 10 400 bash scripts/pmc_passes.sh > gpurun_out/abconv/pmc.log 2>&1
