#!/bin/bash
# A/B of PT_DEVICE_DEFINES variants on tools/cfg_probe.py.
# usage: tools/ab/cfg_ab.sh "CONFIG NPIX SPP [opt]" REPS "defs1" "defs2" ...   ("-" = none)
ARGS=$1; REPS=$2; shift 2
for r in $(seq "$REPS"); do
  for d in "$@"; do
    if [ "$d" = "-" ]; then unset PT_DEVICE_DEFINES; else export PT_DEVICE_DEFINES="$d"; fi
    out=$(timeout -k 10 300 python tools/cfg_probe.py $ARGS 2>/dev/null) || exit $?
    python -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('%-12s %-24s %8.2f Msamples/s  kernel %8.1f ms  waves-only %8.1f ms' % (d['config'], sys.argv[2], d['Msamples_per_s'], d['kernel_ms'], d['wave_ms']))" "$out" "$d"
  done
done
