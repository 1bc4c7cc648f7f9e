#!/bin/bash
# LLVM scheduler options (PT_JIT_OPTIONS) on C3, perf_probe 64 spp, same box
OUT=gpurun_out/r4o; mkdir -p $OUT
for r in 1 2; do
  for o in "" "-mllvm -amdgpu-sched-strategy=max-ilp" "-mllvm -amdgpu-use-amdgpu-trackers" "-mllvm -amdgpu-disable-unclustered-high-rp-reschedule"; do
    out=$(PT_JIT_OPTIONS="$o" timeout -k 10 300 python3 tools/perf_probe.py 64 2>/dev/null) || exit $?
    python3 -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('C3 %-55s %9.2f Msamples/s' % (sys.argv[2] or 'default', d['Msamples_per_s']))" "$out" "$o"
  done
done
