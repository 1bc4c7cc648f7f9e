#!/bin/bash
# Perf screening: C3 probe only (no parity suite).  usage: tools/quick_probe.sh OUTDIR [spp]
OUT=${1:-gpurun_out/quick}
mkdir -p "$OUT"
timeout -k 10 200 python tools/perf_probe.py ${2:-16} > "$OUT/probe.json" 2> "$OUT/probe.err" || exit $?
python -c "import json; d=json.load(open('$OUT/probe.json')); print('C3 %dspp: %.2f Msamples/s, kernel %.1f ms' % (d['spp'], d['Msamples_per_s'], d['kernel_ms']))"
