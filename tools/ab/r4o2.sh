#!/bin/bash
# LLVM scheduler options (PT_JIT_OPTIONS) on C2 / C5 (cfg_probe), same box
OUT=gpurun_out/r4o2; mkdir -p $OUT
for r in 1 2; do
  for o in "" "-mllvm -amdgpu-use-amdgpu-trackers" "-mllvm -amdgpu-disable-unclustered-high-rp-reschedule"; do
    for p in "C2 65536 16" "C5 65536 8192"; do
      PT_JIT_OPTIONS="$o" timeout -k 10 300 python3 tools/cfg_probe.py $p > $OUT/p.json 2>/dev/null || exit $?
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('%s %-55s %9.3f Msamples/s' % (d['config'], sys.argv[2] or 'default', d['Msamples_per_s']))" $OUT/p.json "$o"
    done
  done
done
