#!/bin/bash
# The round-end GPU checks: pytest -m gpu, then smoke() (each step under its own limit).
OUT=${1:-gpurun_out/suite}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 "$OUT/gpu_tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; cat "$OUT/smoke.log" | tail -2; exit $rc
