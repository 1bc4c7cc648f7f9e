#!/bin/bash
# GPU tests, then an interleaved same-box A/B of device-library texts.
# usage: tools/gpu_ab.sh OUTDIR SPP REPS header...
OUT=$1; SPP=$2; REPS=$3; shift 3
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 "$OUT/gpu_tests.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab/ab.sh "$SPP" "$REPS" "$@" > "$OUT/ab.txt" 2>&1
rc=$?; cat "$OUT/ab.txt"; exit $rc
