#!/bin/bash
# Interleaved A/B of environment settings (runtime experiment hooks) on one box.
# usage: tools/ab/env_ab.sh SPP REPS "VAR=val ..." "-" ...   ("-" = no extra env)
SPP=$1; REPS=$2; shift 2
for r in $(seq "$REPS"); do
  for d in "$@"; do
    if [ "$d" = "-" ]; then envs=(); else read -ra envs <<< "$d"; fi
    out=$(env "${envs[@]}" timeout -k 10 300 python tools/perf_probe.py "$SPP" 2>/dev/null) || exit $?
    python -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('%-28s %7.2f Msamples/s  kernel %8.1f ms  reduce %6.1f ms  waves-only %7.2f' % (sys.argv[2], d['Msamples_per_s'], d['kernel_ms'], d['reduce_ms'], d['Msamples_per_s_waves'] or 0))" "$out" "$d"
  done
done
