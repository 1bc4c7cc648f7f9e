#!/bin/bash
# GPU parity suite on the built-in library, then interleaved C3 A/B probes and
# a small C2 probe per header.  usage: tools/ab/run_ab.sh OUT headerA headerB
# (a baseline header: git show REV:path-trace_amd/csrc/device/pt_device.h > /tmp/prev.h)
OUT=$1; shift
bash tools/gpu_check.sh "$OUT" || exit $?
bash tools/ab_probe.sh 16 2 "$@" || exit $?
for h in "$@"; do
  PT_DEVICE_HEADER=$h timeout -k 10 300 python tools/probe_cfg.py C2 320 180 1 > "$OUT/c2_$(basename $h).json" 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$OUT/c2_$(basename $h).json').read().splitlines()[-1]); print('$h C2 320x180x1: %.3f Msamples/s slow_frac %.3f' % (d['Msamples_per_s'], d['slow_frac']))"
done
