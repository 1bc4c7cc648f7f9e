#!/bin/bash
# Interleaved A/B of compiler-option variants on C2 (probe_cfg, reduced frame) and C5 (bench.py subset line).
# usage: tools/ab/cfg_opt.sh REPS "opts1" "opts2" ...   ("-" = none)
REPS=$1; shift
for r in $(seq "$REPS"); do
  for o in "$@"; do
    if [ "$o" = "-" ]; then unset PT_JIT_OPTIONS; else export PT_JIT_OPTIONS="$o"; fi
    out=$(timeout -k 10 300 python tools/probe_cfg.py C2 640 360 16 2>/dev/null) || exit $?
    python -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('C2 640x360x16 %-34s %8.3f Msamples/s  kernel %8.1f ms' % (sys.argv[2], d['Msamples_per_s'], d['kernel_ms']))" "$out" "$o"
    out=$(timeout -k 10 300 python bench.py --config C5 --no-cpu 2>/dev/null) || exit $?
    python -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('C5 bench       %-34s %8.2f Msamples/s  ms %8.1f' % (sys.argv[2], d['value'], d['ms_per_step']))" "$out" "$o"
  done
done
