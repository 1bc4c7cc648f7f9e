#!/bin/bash
# Interleaved A/B of device-library texts on the C2 probe (640x360x16).
# usage: tools/ab/c2_hdr.sh REPS header1 [header2 ...]   ("-" = built-in library, "D:defs" = PT_DEVICE_DEFINES)
REPS=$1; shift
for r in $(seq "$REPS"); do
  for h in "$@"; do
    unset PT_DEVICE_HEADER PT_DEVICE_DEFINES
    case "$h" in -) ;; D:*) export PT_DEVICE_DEFINES="${h#D:}" ;; *) export PT_DEVICE_HEADER="$h" ;; esac
    out=$(timeout -k 10 300 python tools/probe_cfg.py C2 640 360 16 2>/dev/null) || exit $?
    python -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('C2 640x360x16 %-18s %8.3f Msamples/s  kernel %8.1f ms  mid %d slow %d' % (sys.argv[2], d['Msamples_per_s'], d['kernel_ms'], d['mid_queries'], d['slow_queries']))" "$out" "$h"
  done
done
