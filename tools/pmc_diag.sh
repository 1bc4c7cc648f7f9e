#!/bin/bash
# Where the C3 kernel's wave-cycles go: instruction cache, issue stalls, LDS.
# One rocprofv3 --pmc run per counter group (<= 8 SQ counters a pass).
# usage: tools/pmc_diag.sh OUTDIR [SPP]
OUT=${1:-gpurun_out/diag}; SPP=${2:-32}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
i=0
run() {
    i=$((i + 1))
    timeout -s KILL 150 rocprofv3 --pmc "$@" -d "$OUT/p$i" -o p$i --output-format csv -- python3 "$ROOT/tools/perf_probe.py" "$SPP" fast > "$OUT/p$i.log" 2>&1
    rc=$?; echo "pass $i: rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}
run SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS
run SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
run SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_BUSY_CYCLES
python3 "$ROOT/tools/sum_pmc.py" pt_render_fast "$OUT/p1" "$OUT/p2" "$OUT/p3"
