#!/bin/bash
# C2 / C5 phase splits on the final kernel, then the clear pass for union-only scenes (cu.h) on C2 (same box)
OUT=gpurun_out/r4v; mkdir -p $OUT
timeout -k 10 400 python3 tools/phase_probe.py bench C2 > $OUT/phase_C2.txt 2>&1 || exit $?
timeout -k 10 300 python3 tools/phase_probe.py bench C5 > $OUT/phase_C5.txt 2>&1 || exit $?
cat $OUT/phase_C2.txt $OUT/phase_C5.txt | grep -v "^{"
for r in 1 2; do for h in - tools/ab/cu.h; do
  if [ "$h" = "-" ]; then unset PT_DEVICE_HEADER; else export PT_DEVICE_HEADER=$h; fi
  timeout -k 10 300 python3 tools/cfg_probe.py C2 65536 16 > $OUT/p.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('C2 %-14s %9.3f Msamples/s' % (sys.argv[2], d['Msamples_per_s']))" $OUT/p.json $h
done; done
