#!/bin/bash
# Interleaved A/B of PT_DEVICE_DEFINES variants on one box.
# usage: tools/ab/defs.sh SPP REPS "defs1" "defs2" ...   ("-" = none)
SPP=$1; REPS=$2; shift 2
for r in $(seq "$REPS"); do
  for d in "$@"; do
    if [ "$d" = "-" ]; then unset PT_DEVICE_DEFINES; else export PT_DEVICE_DEFINES="$d"; fi
    out=$(timeout -k 10 300 python tools/perf_probe.py "$SPP" 2>/dev/null) || exit $?
    python -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('%-28s %7.2f Msamples/s  kernel %8.1f ms  waves-only %7.2f' % (sys.argv[2], d['Msamples_per_s'], d['kernel_ms'], d['Msamples_per_s_waves'] or 0))" "$out" "$d"
  done
done
