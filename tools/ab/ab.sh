#!/bin/bash
# Interleaved A/B of device-library texts on one box (clock and tail vary
# between boxes, so only same-box comparisons count).
# usage: tools/ab/ab.sh SPP REPS header... ("-" = the built-in library)
SPP=$1; REPS=$2; shift 2
for r in $(seq "$REPS"); do
  for h in "$@"; do
    if [ "$h" = "-" ]; then unset PT_DEVICE_HEADER; else export PT_DEVICE_HEADER=$h; fi
    out=$(timeout -k 10 300 python tools/perf_probe.py "$SPP" 2>/dev/null) || exit $?
    python -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('%-22s %7.2f Msamples/s  kernel %8.1f ms  waves-only %7.2f' % (sys.argv[2], d['Msamples_per_s'], d['kernel_ms'], d['Msamples_per_s_waves'] or 0))" "$out" "$h"
  done
done
