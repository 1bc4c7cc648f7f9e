#!/bin/bash
# final: GPU suite, smoke(), the C5 evidence again (dequeue prefetch now on for lane-walk scenes), the default bench line
OUT=gpurun_out/r4z; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
bash tools/r4_final.sh $OUT C5 || exit $?
timeout -k 10 300 python3 bench.py --config C5 > $OUT/bench_C5.json 2> $OUT/bench_C5.err || exit $?
tail -1 $OUT/bench_C5.json | cut -c1-200
timeout -k 10 300 python3 bench.py > $OUT/bench_C3.json 2> $OUT/bench_C3.err || exit $?
tail -1 $OUT/bench_C3.json | cut -c1-200
