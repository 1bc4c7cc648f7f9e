#!/bin/bash
# GPU suite (lane-major jump stride now PT_KATT l), then PT_KATT on C2: 6 (new default for Difference-free scenes) / 8 / 4, same box
OUT=gpurun_out/r4k2; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3 4; do
  for k in "" 8 4; do
    if [ -z "$k" ]; then unset PT_DEVICE_DEFINES; else export PT_DEVICE_DEFINES="PT_KATT=$k"; fi
    timeout -k 10 300 python3 tools/cfg_probe.py C2 65536 16 > $OUT/p.json 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('C2 KATT %-4s %9.3f Msamples/s' % (sys.argv[2] or '6', d['Msamples_per_s']))" $OUT/p.json "$k"
  done
done
