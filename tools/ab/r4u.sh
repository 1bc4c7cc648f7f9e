#!/bin/bash
# C5 lane-walk depth 2/3/1, dequeue prefetch on C3/C5, C2 at 3 workgroups per CU (same box)
OUT=gpurun_out/r4u; mkdir -p $OUT
p() { timeout -k 10 300 python3 tools/cfg_probe.py "$@" > $OUT/p.json 2>/dev/null || exit $?; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('%-40s %9.3f Msamples/s' % (sys.argv[2], d['Msamples_per_s']))" $OUT/p.json "$TAG"; }
for r in 1 2; do
  TAG="C5 lane_walk=2"; p C5 65536 8192
  TAG="C5 lane_walk=3"; PROBE_LANE_WALK=3 p C5 65536 8192
  TAG="C5 lane_walk=1"; PROBE_LANE_WALK=1 p C5 65536 8192
  TAG="C5 prefetch"; PT_DEVICE_HEADER=tools/ab/pf.h p C5 65536 8192
  TAG="C2 wg=4"; p C2 65536 16
  TAG="C2 wg=3"; PROBE_WG=3 p C2 65536 16
done
SKIP_TESTS=1 bash tools/ab/cfg3.sh $OUT 2 - tools/ab/pf.h 2>&1 | grep "^C3" || exit $?
