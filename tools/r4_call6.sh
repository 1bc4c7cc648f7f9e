#!/bin/bash
# round-end check after the scheduler option: GPU suite, smoke(), C3 / C2 / C5 bench lines
OUT=gpurun_out/r4end2; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
for c in C3 C5 C2; do
  timeout -k 10 400 python3 bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit $?
  tail -1 $OUT/bench_$c.json | cut -c1-120
done
