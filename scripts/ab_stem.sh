# Stem: GPU stem/feature/pipeline tests on the tree build, then A/B (abvar/base.so vs abvar/new.so in
# one process, twice) and config 5
set -o pipefail
mkdir -p gpurun_out/abstem
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_features.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/abstem/pytest.log 2>&1 && \
for r in 1 2; do MCGMIL_PROBE_LIBS=abvar/base.so,abvar/new.so timeout -k 10 200 python scripts/probe_stem.py > gpurun_out/abstem/stem_$r.log 2>&1 || exit 1; done && \
timeout -k 10 400 python bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/abstem/cfg5.log 2>&1
