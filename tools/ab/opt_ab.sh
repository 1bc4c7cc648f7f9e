#!/bin/bash
# Interleaved A/B of compiler-option variants (PT_JIT_OPTIONS) on the C3 probe.
# usage: tools/ab/opt_ab.sh SPP REPS "opts1" "opts2" ...   ("-" = none)
SPP=$1; REPS=$2; shift 2
for r in $(seq "$REPS"); do
  for d in "$@"; do
    if [ "$d" = "-" ]; then unset PT_JIT_OPTIONS; else export PT_JIT_OPTIONS="$d"; fi
    out=$(timeout -k 10 300 python tools/perf_probe.py "$SPP" 2>/dev/null) || exit $?
    python -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('%-52s %7.2f Msamples/s  kernel %8.1f ms' % (sys.argv[2], d['Msamples_per_s'], d['kernel_ms']))" "$out" "$d"
  done
done
