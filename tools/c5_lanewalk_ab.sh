#!/bin/bash
# C5 A/B of the per-lane tree walk depth (pt_scene_set_lane_walk): bench-like subset and the glass disk.
OUT=${1:-gpurun_out/lw}; mkdir -p "$OUT"
for k in "$@"; do :; done
for k in 0 2 3 4; do
  for what in mixed disk; do
    if [ $what = disk ]; then A="4096 256 disk:2460:1080:400"; else A="65536 256"; fi
    PROBE_LANE_WALK=$k timeout -k 10 200 python3 tools/cfg_probe.py C5 $A > "$OUT/${what}_$k.json" 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('lane_walk', sys.argv[2], sys.argv[3], '%.1f Msamples/s  kernel %.1f ms  q/s %.3f' % (d['Msamples_per_s'], d['kernel_ms'], d['queries_per_sample']))" "$OUT/${what}_$k.json" $k $what
  done
done
