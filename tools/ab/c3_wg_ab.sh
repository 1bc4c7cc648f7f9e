#!/bin/bash
# C3 occupancy A/B (workgroups per CU via PROBE_WG; default = the LDS limit, 5), same box.
OUT=${1:-gpurun_out/ab4}; mkdir -p $OUT
for r in 1 2 3; do
for wg in 5 4 3; do
  spec=""; [ $wg = 5 ] || spec="PROBE_WG=$wg"
  env $spec timeout -k 10 120 python3 tools/cfg_probe.py C3 0 128 > $OUT/p.json 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('wg %s  %7.2f Msamples/s  kernel %8.1f ms' % (sys.argv[2], d['Msamples_per_s'], d['kernel_ms']))" $OUT/p.json $wg
done
done
