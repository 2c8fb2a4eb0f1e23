#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the headline bench command per library variant,
# then one interleaved timing A/B of the same variants. Usage:
#   VARIANTS="base nt rev" bash scripts/ab_traffic_variants.sh      (libraries abvar/<name>.so)
set -u
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
    echo "== variant $v"
    MCGMIL_LIB=abvar/$v.so PASSES="fetch write" bash scripts/pmc_passes.sh > gpurun_out/pmc_$v.log 2>&1 || {
        echo "pmc failed for $v"; tail -5 gpurun_out/pmc_$v.log; exit 1; }
    for p in fetch write; do
        mkdir -p gpurun_out/pmc_$v && cp gpurun_out/pmc/$p.json gpurun_out/pmc_$v/
        grep -A4 '"void mcgmil::gate_fused' gpurun_out/pmc/$p.json | grep -i 'size\|calls' || true
    done
done
libs=$(for v in ${VARIANTS:-base}; do printf "abvar/%s.so," "$v"; done)
timeout -k 10 300 env MCGMIL_PROBE_LIBS=${libs%,} PROBE_BAGS=128 PROBE_ROUNDS=7 python -u scripts/probe_fused.py \
    > gpurun_out/ab_traffic_timing.log 2>&1 || { tail -5 gpurun_out/ab_traffic_timing.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_traffic_timing.log
