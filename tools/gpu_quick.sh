#!/bin/bash
# GPU parity suite + C3 probe at SPP (+ phase split).  usage: tools/gpu_quick.sh OUTDIR [SPP] [phase]
OUT=${1:-gpurun_out/q}; SPP=${2:-64}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -5 "$OUT/gpu_tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/perf_probe.py "$SPP" > "$OUT/probe.json" 2> "$OUT/probe.err" || exit $?
cat "$OUT/probe.json"
if [ "$3" = phase ]; then
    timeout -k 10 300 python tools/phase_probe.py "$SPP" > "$OUT/phase.txt" 2>&1 || exit $?
    cat "$OUT/phase.txt"
fi
