#!/bin/bash
# One gpurun session: smoke -> GPU parity tests -> bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit. A plain failure (exit 1: a failed assertion) lets the
# next step run; any other non-zero exit (fault/abort/segfault/timeout) ends the script.
# Usage: bash scripts/gpu_check.sh [tag] [steps...]   (steps: smoke tests bench prof)
set -u
TAG=${1:-r01}
shift || true
STEPS=${*:-smoke tests bench prof}
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "== $name (limit ${secs}s): $*"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 25 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "== stopping: $name exited with $rc"
        exit $rc
    fi
    return 0
}

for s in $STEPS; do
    case $s in
        smoke) run smoke 420 python -c "import __graft_entry__ as g; g.build(); g.smoke()" ;;
        tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread ;;
        bench) run bench 600 python bench.py ;;
        imgtests) run pytest_gpu_image 600 python -m pytest tests/test_gpu_image.py -m gpu -q -rf ;;
        imgprobe) run probe_image 300 python scripts/probe_image.py ;;
        e2etests) run pytest_gpu_pipeline 600 python -m pytest tests/test_gpu_pipeline.py -m gpu -q -rf ;;
        resnet) run probe_resnet 600 python scripts/probe_resnet.py ;;
        cfg5) run bench_cfg5 900 python bench.py --workload cfg5 --steps 5 --warmup 2 ;;
        cfg4) run bench_cfg4 600 python bench.py --workload cfg4 ;;
        dist1) run bench_dist1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
                --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 2 ;;
        probe) run probe 300 python scripts/probe_gate.py ;;
        determ) run determinism 300 python scripts/probe_determinism.py && \
                run determinism_pipe 300 env MCGMIL_GATE=pipe python scripts/probe_determinism.py ;;
        probepipe) run probe_pipe 300 env MCGMIL_GATE=pipe python scripts/probe_gate.py ;;
        stamps) run stamps 300 python scripts/probe_stamps.py ;;
        ab) run ab 300 env MCGMIL_PROBE_LIBS="$(ls -1 abvar/*.so 2>/dev/null | paste -sd, -)" \
                PROBE_ONLY=philox python scripts/probe_gate.py ;;
        prof)
            rm -rf "$OUT/prof_$TAG"
            run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run \
                --output-format csv -- python3 bench.py
            find "$OUT/prof_$TAG" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_$TAG.csv" \;
            ;;
        pmcsq)
            rm -rf "$OUT/pmc_${TAG}_sq"
            run pmc_sq 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
                SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace \
                -d "$OUT/pmc_${TAG}_sq" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
            f=$(find "$OUT/pmc_${TAG}_sq" -name "*counter_collection.csv" | head -1)
            python3 scripts/pmc_summary.py "$f" > "$OUT/pmc_sq_summary_$TAG.json"
            ;;
        profcfg5)
            rm -rf "$OUT/prof_cfg5_$TAG"
            run rocprof_cfg5 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cfg5_$TAG" -o run \
                --output-format csv -- python3 bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline
            find "$OUT/prof_cfg5_$TAG" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_cfg5_$TAG.csv" \;
            ;;
        pmc)
            for ctr in FETCH_SIZE WRITE_SIZE; do
                rm -rf "$OUT/pmc_${TAG}_$ctr"
                run pmc_$ctr 600 rocprofv3 --pmc $ctr --kernel-trace -d "$OUT/pmc_${TAG}_$ctr" -o run \
                    --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
                find "$OUT/pmc_${TAG}_$ctr" -name "*counter_collection.csv" -exec cp {} "$OUT/pmc_${TAG}_$ctr.csv" \;
            done
            ;;
    esac
done
echo "== done"
