#!/bin/bash
# pass queries' contexts as vector values (cv.h = PT_CTX_VGPR 1) on C3 / C5 / C2, same box
OUT=gpurun_out/r4w; mkdir -p $OUT
SKIP_TESTS=1 bash tools/ab/cfg3.sh $OUT 2 - tools/ab/cv.h || exit $?
