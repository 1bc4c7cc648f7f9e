#!/bin/bash
# GPU parity suite + quick C3 probe (+ optional phase split).  usage: tools/gpu_check.sh OUTDIR [phase]
OUT=${1:-gpurun_out/check}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/perf_probe.py 16 > "$OUT/probe.json" 2> "$OUT/probe.err" || exit $?
python -c "import json,sys; d=json.load(open('$OUT/probe.json')); print('C3 16spp: %.2f Msamples/s, kernel %.1f ms' % (d['Msamples_per_s'], d['kernel_ms']))"
if [ "$2" = phase ]; then
    timeout -k 10 300 python tools/phase_probe.py 16 > "$OUT/phase.txt" 2>&1 || exit $?
    cat "$OUT/phase.txt"
fi
