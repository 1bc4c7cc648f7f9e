#!/bin/bash
# Two PMC passes (issue mix + memory instructions) of tools/cfg_probe.py.
# usage: tools/pmc_cfg.sh OUTDIR CONFIG NPIX SPP [probe options]
OUT=${1:-gpurun_out/pmcc}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
i=0
run() {
    i=$((i + 1))
    timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/p$i" -o p$i --output-format csv -- python3 "$ROOT/tools/cfg_probe.py" $ARGS > "$OUT/p$i.log" 2>&1
    rc=$?; echo "pass $i: rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}
ARGS="$*"
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE
run SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_FLAT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU
python3 "$ROOT/tools/sum_pmc.py" pt_render_fast "$OUT/p1" "$OUT/p2"
