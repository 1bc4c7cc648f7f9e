#!/bin/bash
# round-end check of the committed tree: GPU suite, smoke(), default bench line
OUT=gpurun_out/r4end; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -1 $OUT/bench.json | cut -c1-200
