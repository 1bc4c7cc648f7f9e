#!/bin/bash
# Counter evidence for the bench line: rocprofv3 --pmc passes of the bench
# command itself (never combined with tracing; one counter group per pass),
# summarised by tools/pmc_summary.py into OUT/pmc.json.
#   busy   issue/busy counters        fetch  FETCH_SIZE     write  WRITE_SIZE
#   stall  wave-cycle split + memory instruction mix     cache  L2 hits/misses
#   tex    texture address/data unit busy (TA, TD) and flat read wavefronts
# usage: tools/pmc_bench.sh OUTDIR [bench args...]
OUT=${1:-gpurun_out/pmcb}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
pass() {
    name=$1; shift
    timeout -k 10 600 rocprofv3 --pmc "$@" -d "$OUT/$name" -o $name --output-format csv -- python3 "$ROOT/bench.py" --no-cpu "${BENCH_ARGS[@]}" > "$OUT/$name.log" 2>&1
    rc=$?; echo "$name rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}
BENCH_ARGS=("$@")
pass busy SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_SMEM
pass cache TCC_HIT_sum TCC_MISS_sum
pass tex TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/pmc.json" && cat "$OUT/pmc.json"
