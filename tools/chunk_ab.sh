#!/bin/bash
# A/B of chunk size (PT_CHUNK_MAX), dequeue prefetch and C5 occupancy, interleaved on one box.
OUT=${1:-gpurun_out/chunk}; mkdir -p "$OUT"
run() { # label env... -- probe args
  local label=$1; shift
  out=$(env "$@" 2>/dev/null) || exit $?
  python3 -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('%-40s %8.2f Msamples/s  kernel %8.1f ms' % (sys.argv[2], d['Msamples_per_s'], d['kernel_ms']))" "$out" "$label"
}
for r in 1 2; do
  for cm in 32 64; do
    run "C3 chunk$cm prefetch" PT_CHUNK_MAX=$cm timeout -k 10 200 python3 tools/perf_probe.py 64
    run "C3 chunk$cm noprefetch" PT_CHUNK_MAX=$cm PT_DEVICE_DEFINES=PT_DEQUEUE_PREFETCH=0 timeout -k 10 200 python3 tools/perf_probe.py 64
    run "C5 chunk$cm prefetch wg2" PT_CHUNK_MAX=$cm timeout -k 10 200 python3 tools/cfg_probe.py C5 65536 2048
    run "C5 chunk$cm noprefetch wg2" PT_CHUNK_MAX=$cm PT_DEVICE_DEFINES=PT_DEQUEUE_PREFETCH=0 timeout -k 10 200 python3 tools/cfg_probe.py C5 65536 2048
    run "C5 chunk$cm prefetch wg3" PT_CHUNK_MAX=$cm PROBE_WG=3 timeout -k 10 200 python3 tools/cfg_probe.py C5 65536 2048
    run "C5 chunk$cm prefetch wg4" PT_CHUNK_MAX=$cm PROBE_WG=4 timeout -k 10 200 python3 tools/cfg_probe.py C5 65536 2048
  done
done
