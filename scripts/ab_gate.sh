#!/bin/bash
# Gate-kernel A/B session on the GPU box: bitwise comparison of the variant libraries in abvar/,
# interleaved timing (scripts/probe_gate.py), then the MCDO GPU parity tests on the in-tree build.
# Usage: bash scripts/ab_gate.sh [tests]
set -u
OUT=gpurun_out
mkdir -p $OUT
LIBS=$(ls -1 abvar/*.so | paste -sd, -)
export TMPDIR=/tmp
if [ -z "${SKIP_COMPARE:-}" ]; then
    timeout -k 10 240 env MCGMIL_PROBE_LIBS="$LIBS" python scripts/compare_libs.py > $OUT/ab_compare.log 2>&1
    rc=$?; echo "compare rc=$rc"; cat $OUT/ab_compare.log | grep -v amdgpu.ids
    [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 env MCGMIL_PROBE_LIBS="$LIBS" PROBE_ONLY=${PROBE_ONLY:-philox} python scripts/probe_gate.py > $OUT/ab_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu.ids $OUT/ab_probe.log
[ $rc -ne 0 ] && exit $rc
if [ "${1:-}" = tests ]; then
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/ab_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -5 $OUT/ab_tests.log
fi
exit $rc
