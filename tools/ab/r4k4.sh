#!/bin/bash
# PT_KATT on C3: 10 (the default for trees with a Difference) / 12, perf_probe 64 spp, same box
OUT=gpurun_out/r4k4; mkdir -p $OUT
for r in 1 2 3; do
  for k in "" 12; do
    if [ -z "$k" ]; then unset PT_DEVICE_DEFINES; else export PT_DEVICE_DEFINES="PT_KATT=$k"; fi
    out=$(timeout -k 10 300 python3 tools/perf_probe.py 64 2>/dev/null) || exit $?
    python3 -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('C3 KATT %-4s %9.2f Msamples/s' % (sys.argv[2] or '10', d['Msamples_per_s']))" "$out" "$k"
  done
done
