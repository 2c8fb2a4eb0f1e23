# Stem A/B (abvar/base.so vs abvar/new.so in one process, twice) and a config-5 kernel trace of the tree build
set -o pipefail
mkdir -p gpurun_out/abstem
export TMPDIR=/tmp
for r in 1 2; do MCGMIL_PROBE_LIBS=abvar/base.so,abvar/new.so timeout -k 10 200 python scripts/probe_stem.py > gpurun_out/abstem/stem_$r.log 2>&1 || exit 1; done && \
rm -rf gpurun_out/abstem/prof && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/abstem/prof -o run --output-format csv -- python3 bench.py --workload cfg5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abstem/prof.log 2>&1
