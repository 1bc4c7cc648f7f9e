#!/bin/bash
# C2 evidence (PMC passes + rocprof kernel stats) and the plain C2 bench line
OUT=gpurun_out/r4h; mkdir -p $OUT
bash tools/r4_final.sh $OUT C2 || exit $?
timeout -k 10 400 python3 bench.py --config C2 > $OUT/bench_C2.json 2> $OUT/bench_C2.err || exit $?
tail -1 $OUT/bench_C2.json | cut -c1-300
