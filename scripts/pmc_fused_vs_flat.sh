#!/bin/bash
# L2 hit rate and HBM traffic of the headline bench, two-kernel path vs the fused single launch
# (MCGMIL_FUSED=1), one rocprofv3 counter pass per group (scripts/pmc_passes.sh).
set -u
export TMPDIR=/tmp
PASSES="tcc fetch write tcp" bash scripts/pmc_passes.sh || exit $?
mkdir -p gpurun_out/pmc_flat && mv gpurun_out/pmc/*.json gpurun_out/pmc_flat/
MCGMIL_FUSED=1 PASSES="tcc fetch write tcp" bash scripts/pmc_passes.sh || exit $?
mkdir -p gpurun_out/pmc_fused && mv gpurun_out/pmc/*.json gpurun_out/pmc_fused/
echo "== done"
