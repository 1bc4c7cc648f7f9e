#!/bin/bash
# Interleaved A/B over device-library texts x compiler-option variants on one box.
# usage: tools/ab/matrix.sh SPP REPS "hdr1 hdr2 ..." "opts1" "opts2" ...   ("-" = built-in / none)
SPP=$1; REPS=$2; HDRS=$3; shift 3
for r in $(seq "$REPS"); do
  for h in $HDRS; do
    for o in "$@"; do
      if [ "$h" = "-" ]; then unset PT_DEVICE_HEADER; else export PT_DEVICE_HEADER="$h"; fi
      if [ "$o" = "-" ]; then unset PT_JIT_OPTIONS; else export PT_JIT_OPTIONS="$o"; fi
      out=$(timeout -k 10 300 python tools/perf_probe.py "$SPP" 2>/dev/null) || exit $?
      python -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('%-18s %-34s %7.2f Msamples/s  kernel %8.1f ms' % (sys.argv[2], sys.argv[3], d['Msamples_per_s'], d['kernel_ms']))" "$out" "$h" "$o"
    done
  done
done
