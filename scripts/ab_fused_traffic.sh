#!/bin/bash
# Fused-kernel A/B (n-major region order vs linear) and the fused launch's HBM traffic (PMC).
export TMPDIR=/tmp
timeout -k 10 300 env MCGMIL_PROBE_LIBS=abvar/fz.so,abvar/fzn.so PROBE_BAGS=128 PROBE_ROUNDS=7 python -u scripts/probe_fused.py > gpurun_out/ab_fused5.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_fused5.log
MCGMIL_FUSED=1 PASSES="fetch write tcc" bash scripts/pmc_passes.sh > gpurun_out/pmc_fz.log 2>&1 || exit $?
grep -A4 '"void mcgmil::gate_fused' gpurun_out/pmc/*.json
