#!/bin/bash
# GPU suite + smoke + default bench after PT_KATT 10 for trees with a Difference (no lane walks)
OUT=gpurun_out/r4k10; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py > $OUT/bench_C3.json 2> $OUT/bench_C3.err || exit $?
tail -1 $OUT/bench_C3.json | cut -c1-150
