#!/bin/bash
# PC sampling of one bench.py frame (rocprofv3 beta: --pc-sampling-method stochastic
# records the wave's issue state and stall reason per sample; host_trap only the PC),
# summarised on the box by tools/pc_summary.py.   usage: tools/pc_sample.sh OUTDIR METHOD INTERVAL [bench args]
OUT=$1; METHOD=$2; IV=$3; shift 3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
UNIT=cycles; [ "$METHOD" = host_trap ] && UNIT=time
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method "$METHOD" --pc-sampling-unit "$UNIT" \
    --pc-sampling-interval "$IV" -d /tmp/pcs_raw -o pcs --output-format csv -- python3 "$ROOT/bench.py" --no-cpu "$@" \
    > "$OUT/pcs_${METHOD}.log" 2>&1
rc=$?
if [ $rc -ne 0 ]; then echo "FAILED rc=$rc (rocprofv3 pc sampling)"; tail -30 "$OUT/pcs_${METHOD}.log"; exit $rc; fi
python3 "$ROOT/tools/pc_summary.py" /tmp/pcs_raw 600 > "$OUT/pc_summary_${METHOD}.txt" 2>&1
head -40 "$OUT/pc_summary_${METHOD}.txt"
