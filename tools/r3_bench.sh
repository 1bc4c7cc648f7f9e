#!/bin/bash
# Bench lines of the round: C3 (with its CPU leg), C5 and C2 (no CPU leg), each
# step under its own limit, stopping at the first failure.
OUT=${1:-gpurun_out/bench}; mkdir -p "$OUT"
for c in C3 C5 C2; do
  extra=""; [ $c = C3 ] || extra="--no-cpu"
  timeout -k 10 400 python3 bench.py --config $c $extra > "$OUT/$c.json" 2> "$OUT/$c.err"
  rc=$?; echo "bench $c rc=$rc"; tail -1 "$OUT/$c.json"; [ $rc -eq 0 ] || exit $rc
done
