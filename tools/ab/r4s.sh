#!/bin/bash
# sphere skip (PT_SPHERE_SKIP) A/B on C3 / C5 / C2, same box
OUT=gpurun_out/r4s; mkdir -p $OUT
SKIP_TESTS=1 bash tools/ab/cfg3.sh $OUT 2 - tools/ab/skip.h || exit $?
