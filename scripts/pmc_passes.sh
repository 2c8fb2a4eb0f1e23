#!/bin/bash
# rocprofv3 counter passes on the headline bench command (python3 bench.py: 512 config-3 bags per
# step), one pass per block group as MI355X_MICROARCH.md prescribes (<= 8 SQ, 4 TCC, 4 TCP, 2 GRBM
# counters each; no tracing besides --kernel-trace). Each pass under its own hard time limit; the
# script stops at the first pass that does not exit 0. Summaries: scripts/pmc_summary.py.
set -u
OUT=gpurun_out/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD=${PMC_CMD:-"python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"}
pass() {  # name counters...
    local name=$1
    shift
    rm -rf "$OUT/$name"
    echo "== pass $name: $*"
    timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run --output-format csv -- $CMD \
        > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== pass $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; exit $rc; fi
    f=$(find "$OUT/$name" -name "*counter_collection.csv" | head -1)
    python3 scripts/pmc_summary.py "$f" > "$OUT/$name.json"
    grep -A12 '"_ZN6mcgmil' "$OUT/$name.json" | head -30
}
for p in ${PASSES:-sq lds mem tcp tcc fetch write}; do
    case $p in
        sq)    pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
                    SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES ;;
        lds)   pass lds SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU \
                    SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES ;;
        mem)   pass mem SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM \
                    SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT ;;
        tcp)   pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum \
                    TCP_PENDING_STALL_CYCLES_sum ;;
        tcc)   pass tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum ;;
        fetch) pass fetch FETCH_SIZE ;;
        write) pass write WRITE_SIZE ;;
    esac
done
echo "== pmc done"
