#!/bin/bash
# attempts per lane per generation round (PT_KATT 8 default / 6 / 4) on C2, same box
OUT=gpurun_out/r4k; mkdir -p $OUT
for r in 1 2 3 4; do
  for k in "" 6 4; do
    if [ -z "$k" ]; then unset PT_DEVICE_DEFINES; else export PT_DEVICE_DEFINES="PT_KATT=$k"; fi
    timeout -k 10 300 python3 tools/cfg_probe.py C2 65536 16 > $OUT/p.json 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('C2 KATT %-4s %9.3f Msamples/s' % (sys.argv[2] or '8', d['Msamples_per_s']))" $OUT/p.json "$k"
  done
done
