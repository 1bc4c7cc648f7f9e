#!/bin/bash
# C2 with the full material mix (matBrightDiffuseWhite): single samples on the
# bright sphere, then a small hashed subset; fast spine on and off.
OUT=${1:-gpurun_out/c2}; mkdir -p "$OUT"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], '%.6f Msamples/s kernel %.1f ms q/s %.1f px %d' % (d['Msamples_per_s'], d['kernel_ms'], d['queries_per_sample'], d['pixels']))" "$1" "$2"; }
for fs in 0 1; do
  PROBE_FAST_SPINE=$fs timeout -k 10 150 python3 tools/cfg_probe.py C2 4 1 disk:429:397:30 > "$OUT/disk4_fs$fs.json" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }; show "$OUT/disk4_fs$fs.json" "bright4 fs$fs"
done
for fs in 0 1; do
  PROBE_C2_PLAIN=1 PROBE_FAST_SPINE=$fs timeout -k 10 150 python3 tools/cfg_probe.py C2 16384 16 > "$OUT/plain_fs$fs.json" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }; show "$OUT/plain_fs$fs.json" "plain16k fs$fs"
done
