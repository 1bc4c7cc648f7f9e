#!/bin/bash
# GPU suite, then the C5 evidence (PMC passes + rocprof kernel stats), the
# plain C5 bench line and one whole 3840x2160x8192 frame on one GPU
OUT=gpurun_out/r4g; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/r4_final.sh $OUT C5 || exit $?
timeout -k 10 300 python3 bench.py --config C5 > $OUT/bench_C5.json 2> $OUT/bench_C5.err || exit $?
tail -1 $OUT/bench_C5.json | cut -c1-300
timeout -k 10 300 python3 bench.py --config C5 --subset 0 --no-cpu > $OUT/bench_C5_whole_frame.json 2> $OUT/bench_C5_whole.err || exit $?
tail -1 $OUT/bench_C5_whole_frame.json | cut -c1-400
