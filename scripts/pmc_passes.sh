#!/bin/bash
# rocprofv3 counter passes on the headline bench command (python3 bench.py: 512 config-3 bags per
# step), one pass per block group as MI355X_MICROARCH.md prescribes (<= 8 SQ, 4 TCC, 4 TCP, 2 TA,
# 2 TD, 2 GRBM counters each; no tracing besides --kernel-trace). Each pass under its own hard time
# limit; the script stops at the first pass that does not exit 0. A pass whose counters are not in
# `rocprofv3 --list-avail` (taken once into $OUT/avail.txt) is skipped, not run.
# Summaries: scripts/pmc_summary.py.
set -u
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD=${PMC_CMD:-"python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"}
if [ ! -s "$OUT/avail.txt" ]; then
    timeout -s KILL 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
fi
have() {  # every counter's base name (without _sum/_avr/_min/_max) listed?
    local c
    for c in "$@"; do
        c=${c%_sum}; c=${c%_avr}; c=${c%_max}; c=${c%_min}
        grep -q -w "$c" "$OUT/avail.txt" || { echo "== skip: $c not listed"; return 1; }
    done
}
pass() {  # name counters...
    local name=$1
    shift
    have "$@" || return 0
    rm -rf "$OUT/$name"
    echo "== pass $name: $*"
    timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run --output-format csv -- $CMD \
        > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== pass $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; exit $rc; fi
    f=$(find "$OUT/$name" -name "*counter_collection.csv" | head -1)
    python3 scripts/pmc_summary.py "$f" > "$OUT/$name.json"
    grep -A14 '"_ZN6mcgmil16gate' "$OUT/$name.json" | head -32
}
for p in ${PASSES:-sq lds mem tcp tcc fetch write}; do
    case $p in
        sq)    pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
                    SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES ;;
        lds)   pass lds SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU \
                    SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES ;;
        mem)   pass mem SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM \
                    SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT ;;
        coex)  pass coex SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
                    SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY ;;
        tcp)   pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum \
                    TCP_PENDING_STALL_CYCLES_sum ;;
        tcp2)  pass tcp2 TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum \
                    TCP_TCC_READ_REQ_LATENCY_sum TCP_GATE_EN1_sum ;;
        ta)    pass ta TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum ;;
        ta2)   pass ta2 TA_FLAT_READ_WAVEFRONTS_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum ;;
        td)    pass td TD_TD_BUSY_sum TD_TC_STALL_sum ;;
        tcc)   pass tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum ;;
        fetch) pass fetch FETCH_SIZE ;;
        write) pass write WRITE_SIZE ;;
    esac
done
echo "== pmc done"
