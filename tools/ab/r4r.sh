#!/bin/bash
# C3-regression bisect (wave index scalar / ring split) + C2 fast-spine A/B
OUT=gpurun_out/r4r; mkdir -p $OUT
SKIP_TESTS=1 bash tools/ab/cfg3.sh $OUT 2 tools/ab/head.h - tools/ab/sw0.h tools/ab/rs0.h tools/ab/swrs0.h || exit $?
for r in 1 2; do for fs in 0 1; do
  PROBE_FAST_SPINE=$fs timeout -k 10 300 python3 tools/cfg_probe.py C2 65536 16 > $OUT/c2fs.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('C2 fast_spine=%s %9.3f Msamples/s' % (sys.argv[2], d['Msamples_per_s']))" $OUT/c2fs.json $fs
done; done
for r in 1 2; do for wg in 2 3; do
  PROBE_WG=$wg timeout -k 10 300 python3 tools/cfg_probe.py C5 65536 8192 > $OUT/c5wg.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('C5 wg=%s %9.3f Msamples/s' % (sys.argv[2], d['Msamples_per_s']))" $OUT/c5wg.json $wg
done; done
bash tools/r4_extra.sh gpurun_out/r4x
