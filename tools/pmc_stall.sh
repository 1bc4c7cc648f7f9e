#!/bin/bash
# Instruction-cache and VALU-mix counters of the C3 probe (one rocprofv3 run per pass).
# usage: tools/pmc_stall.sh OUTDIR [SPP]
OUT=${1:-gpurun_out/stall}; SPP=${2:-32}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
i=0
run() {
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/p$i" -o p$i --output-format csv -- python3 "$ROOT/tools/perf_probe.py" "$SPP" > "$OUT/p$i.log" 2>&1
    rc=$?; echo "pass $i: rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}
run SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU
run SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VSKIPPED
python3 "$ROOT/tools/sum_pmc.py" pt_render_fast "$OUT/p1" "$OUT/p2"
