#!/bin/bash
# C2 with the reference's full material mix: the lane-scatter parity tests,
# then the bright disk, hashed subsets and the whole frame at 1 spp (each step
# under its own limit).
OUT=${1:-gpurun_out/c2mix}; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "lane_scatter or c2_full_mix" > $OUT/tests.log 2>&1; rc=$?; tail -15 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python3 tools/cfg_probe.py C2 256 1 disk:429:397:30 > $OUT/disk256.json 2>&1 && tail -1 $OUT/disk256.json && \
timeout -k 10 100 python3 tools/cfg_probe.py C2 8192 1 > $OUT/mix8k.json 2>&1 && tail -1 $OUT/mix8k.json && \
timeout -k 10 150 python3 tools/cfg_probe.py C2 0 1 > $OUT/full1.json 2>&1 && tail -1 $OUT/full1.json
