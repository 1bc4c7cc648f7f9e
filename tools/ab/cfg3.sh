#!/bin/bash
# GPU parity suite, then same-box A/B of device headers on C3 (64 spp frame),
# C5 (65536 hashed px x 8192 spp) and C2 (65536 hashed px x 16 spp).
# usage: tools/ab/cfg3.sh OUT REPS header...   ("-" = built-in)
OUT=$1; REPS=$2; shift 2; mkdir -p "$OUT"
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq "$REPS"); do
  for h in "$@"; do
    if [ "$h" = "-" ]; then unset PT_DEVICE_HEADER; else export PT_DEVICE_HEADER=$h; fi
    out=$(timeout -k 10 300 python3 tools/perf_probe.py 64 2>/dev/null) || exit $?
    python3 -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('C3 %-18s %9.2f Msamples/s  slow %.2f/sample' % (sys.argv[2], d['Msamples_per_s'], d['slow_queries']/d['samples']))" "$out" "$h"
    for p in "C5 65536 8192" "C2 65536 16"; do
      timeout -k 10 300 python3 tools/cfg_probe.py $p > "$OUT/p.json" 2>/dev/null || exit $?
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('%s %-18s %9.3f Msamples/s  kernel %8.1f ms' % (d['config'], sys.argv[2], d['Msamples_per_s'], d['kernel_ms']))" "$OUT/p.json" "$h"
    done
  done
done
