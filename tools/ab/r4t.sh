#!/bin/bash
# lane index recomputed per use / lane sums in LDS: A/B on C3 / C5 / C2, same box
OUT=gpurun_out/r4t; mkdir -p $OUT
SKIP_TESTS=1 bash tools/ab/cfg3.sh $OUT 2 tools/ab/prev4.h - tools/ab/lr.h tools/ab/ll.h tools/ab/lrll.h || exit $?
