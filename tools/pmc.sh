#!/bin/bash
# PMC passes for the render kernel (one rocprofv3 run per counter group; no
# tracing domains combined with --pmc).  usage: tools/pmc.sh OUTDIR [spp]
# Each pass is time-limited; a timeout/abort/segfault stops the script.
OUT=${1:-gpurun_out/pmc}
SPP=${2:-16}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
run() {
    i=$((i + 1))
    timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/p$i" -o p$i --output-format csv -- python3 "$ROOT/tools/perf_probe.py" "$SPP" > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "pass $i ($*): rc=$rc"
    case $rc in 124|137|134|139) echo "stopping after rc=$rc"; exit $rc;; esac
    return 0
}
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE
run SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH
run SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_IFETCH SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT
run FETCH_SIZE
run WRITE_SIZE
exit 0
