#!/bin/bash
# Dynamic instruction counts of the render kernel per device-code variant.
# usage: tools/pmc_variants.sh OUTDIR SPP "" "PT_LEAF_STUB=1" ...
OUT=$1; SPP=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
    i=$((i + 1))
    PT_DEVICE_DEFINES="$v" timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$OUT/v$i" -o v$i --output-format csv -- python3 "$ROOT/tools/perf_probe.py" "$SPP" > "$OUT/v$i.log" 2>&1
    rc=$?
    echo "variant $i [$v]: rc=$rc"
    case $rc in 124|137|134|139) exit $rc;; esac
done
