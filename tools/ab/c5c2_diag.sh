#!/bin/bash
# Phase split (PT_PHASE_TIMING builds) of the C5 and C2 bench commands, then
# the PMC passes of the C5 bench.  usage: tools/ab/c5c2_diag.sh OUTDIR
OUT=$1; mkdir -p "$OUT"
for c in C5 C2; do
    timeout -k 10 400 python tools/phase_probe.py bench $c > "$OUT/phase_$c.txt" 2>&1 || exit $?
    echo "== $c"; cat "$OUT/phase_$c.txt" | cut -c1-400
done
bash tools/pmc_bench.sh "$OUT/pmc_C5" --config C5 > "$OUT/pmc_C5.txt" 2>&1 || exit $?
tail -40 "$OUT/pmc_C5.txt"
