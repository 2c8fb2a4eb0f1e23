#!/bin/bash
# Round-6 GPU session (steps chosen by STEPS): tests, benches, rocprof summaries, counter passes.
set -u
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    grep -v "amdgpu.ids" "$OUT/$name.log" | tail -n 30
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "== stopping"; exit $rc; fi
}
for s in ${STEPS:-smoke calib all bench}; do
    case $s in
        fused) step pytest_fused 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q -rf --timeout 120 --timeout-method thread ;;
        all) step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ;;
        cfg5) step bench_cfg5 600 python bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline ;;
        profcfg5) rm -rf "$OUT/prof_cfg5"; step rocprof_cfg5 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cfg5" -o run --output-format csv -- python3 bench.py --workload cfg5 --steps 2 --warmup 1 --no-cpu-baseline --no-calibration
              find "$OUT/prof_cfg5" -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace_cfg5.csv" \;
              find "$OUT/prof_cfg5" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_cfg5.csv" \;
              python3 scripts/cfg5_phase_table.py "$OUT/kernel_trace_cfg5.csv" "$OUT/cfg5_phases.json" ;;
        pmcconv) step pmc_conv 1100 env PROBE_K=1507 PMC_CMD="python3 scripts/probe_conv.py" PASSES="sq lds coex" bash scripts/pmc_passes.sh ;;
        parity) step pytest_parity 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py -m gpu -x -q -rf --timeout 300 --timeout-method thread ;;
        bench) step bench 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
        bench16) step bench16 600 python bench.py --bags 16 --no-cpu-baseline ;;
        cfg4) step bench_cfg4 600 python3 bench.py --workload cfg4 --steps 10 --warmup 3 --no-cpu-baseline ;;
        cfg4two) step bench_cfg4_twokernel 600 env MCGMIL_FUSED=0 python3 bench.py --workload cfg4 --steps 10 --warmup 3 --no-cpu-baseline ;;
        benchtwo) step bench_twokernel 600 env MCGMIL_FUSED=0 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ;;
        abfused) step ab_fused 300 env MCGMIL_PROBE_LIBS="$(ls -1 abvar/*.so abvar2/*.so 2>/dev/null | paste -sd, -)" python -u scripts/probe_fused.py ;;
        abfused128) step ab_fused128 300 env PROBE_N=128 MCGMIL_PROBE_LIBS="$(ls -1 abvar/*.so abvar2/*.so 2>/dev/null | paste -sd, -)" python -u scripts/probe_fused.py ;;
        stamps) step stamps_flat 300 env PROBE_BAGS=128 python -u scripts/probe_stamps.py
                step stamps_fused 300 env PROBE_BAGS=128 PROBE_FUSED=1 python -u scripts/probe_stamps.py ;;
        listpmc) step list_pmc 120 rocprofv3 --list-avail ;;
        drift) step probe_drift 600 env PROBE_CPU=1 python -u scripts/probe_cfg5_drift.py bf16 fp32 fp32nochunk fp32torch ;;
        pmc) step pmc 1100 env PMC_CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --busy-seconds 0 --no-secondary" PASSES="fetch write sq coex" bash scripts/pmc_passes.sh ;;
        pmcab) step pmc_ab 1200 env PROBE_ROUNDS=1 PMC_CMD="python3 scripts/probe_fused.py" bash scripts/pmc_passes.sh ;;
        conv32) step pytest_conv32 600 python -u -m pytest tests/test_gpu_conv32.py tests/test_gpu_features.py tests/test_gpu_pipeline.py -m gpu -x -q -rf --timeout 300 --timeout-method thread ;;
        probe32) step probe_conv32 600 python -u scripts/probe_conv32.py ;;
        cfg5f32) step bench_cfg5_fp32 900 python bench.py --workload cfg5 --features fp32 --steps 3 --warmup 1 --no-cpu-baseline ;;
        calib) step pytest_calib 300 python -u -m pytest tests/test_gpu_calib.py -m gpu -x -q -rf --timeout 120 --timeout-method thread ;;
        benchq) step bench 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ;;
        grbm) rm -rf "$OUT/grbm"; step grbm 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d "$OUT/grbm" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary --busy-seconds 4
              python3 scripts/grbm_clock.py "$OUT/grbm" > "$OUT/grbm_clock.json"; head -30 "$OUT/grbm_clock.json" ;;
        grbm4) rm -rf "$OUT/grbm4"; step grbm4 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d "$OUT/grbm4" -o run --output-format csv -- python3 bench.py --workload cfg4 --steps 5 --warmup 2 --no-cpu-baseline --busy-seconds 4
              python3 scripts/grbm_clock.py "$OUT/grbm4" > "$OUT/grbm4_clock.json"; head -30 "$OUT/grbm4_clock.json" ;;
        cfg5drift) step pytest_cfg5drift 400 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q -s -rf --timeout 300 --timeout-method thread -k cfg5 ;;
        pmcfinal) step pmc_final 700 env PMC_OUT=gpurun_out/pmc_final PMC_CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --busy-seconds 0 --no-secondary --no-calibration" PASSES="fetch write" bash scripts/pmc_passes.sh
              python3 scripts/traffic_json.py gpurun_out/pmc_final gpurun_out/gate_traffic.json cfg3 "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE --kernel-trace -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --busy-seconds 0 --no-secondary --no-calibration (scripts/pmc_passes.sh PASSES='fetch write')" ;;
        pmc4) step pmc_cfg4 700 env PMC_OUT=gpurun_out/pmc_cfg4 PMC_CMD="python3 bench.py --workload cfg4 --steps 2 --warmup 1 --no-cpu-baseline --busy-seconds 0 --no-calibration" PASSES="fetch write" bash scripts/pmc_passes.sh
              python3 scripts/traffic_json.py gpurun_out/pmc_cfg4 gpurun_out/gate_traffic_cfg4.json cfg4 "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE --kernel-trace -- python3 bench.py --workload cfg4 --steps 2 --warmup 1 --no-cpu-baseline --busy-seconds 0 --no-calibration (scripts/pmc_passes.sh PASSES='fetch write')" ;;
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        fusednew) step pytest_fusednew 600 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -v --timeout 300 --timeout-method thread -k "xcd or bench_step or path_flag" ;;
        cfg4full) step pytest_cfg4full 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread -k "cfg4_full" ;;
        single) step bench_single 300 python bench.py --workload single ;;
        profsingle) rm -rf "$OUT/prof_single"; step rocprof_single 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_single" -o run --output-format csv -- python3 bench.py --workload single
              find "$OUT/prof_single" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_single.csv" \; ;;
        ab512) step ab_fused512 400 env PROBE_BAGS=512 MCGMIL_PROBE_LIBS="$(ls -1 abvar/*.so 2>/dev/null | paste -sd, -)" python -u scripts/probe_fused.py ;;
        prof) rm -rf "$OUT/prof"; step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5
              find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \; ;;
    esac
done
echo "== done"
