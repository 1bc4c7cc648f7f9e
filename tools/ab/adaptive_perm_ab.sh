#!/bin/bash
# Adaptive caller at C3 16 spp: sample-major slot permutation on/off x chunk cap (same box).
OUT=${1:-gpurun_out/ab3}; mkdir -p $OUT
for r in 1 2; do
for spec in "PT_SAMPLE_PERM=1 PT_CHUNK_MAX=64" "PT_SAMPLE_PERM=0 PT_CHUNK_MAX=64" "PT_SAMPLE_PERM=1 PT_CHUNK_MAX=16" "PT_SAMPLE_PERM=0 PT_CHUNK_MAX=8"; do
  env $spec timeout -k 10 120 python3 tools/probe_adaptive.py C3 16 > $OUT/a.json 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('%-36s adaptive %7.1f ms (exact %7.1f)  full %7.1f ms' % (sys.argv[2], d['adaptive_kernel_ms'], d['exact_batches']['kernel_ms'], d['full_kernel_ms']))" $OUT/a.json "$spec"
done
done
