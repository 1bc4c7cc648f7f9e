#!/bin/bash
# GPU suite, then the C3 evidence (PMC passes + rocprof kernel stats) and the plain bench line
OUT=gpurun_out/r4f; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/r4_final.sh $OUT C3 || exit $?
timeout -k 10 300 python3 bench.py > $OUT/bench_C3.json 2> $OUT/bench_C3.err || exit $?
tail -1 $OUT/bench_C3.json | cut -c1-400
