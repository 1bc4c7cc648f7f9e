mkdir -p gpurun_out/ab2
for cm in 64 16 8 4; do
  PT_CHUNK_MAX=$cm timeout -k 10 120 python3 tools/probe_adaptive.py C3 16 > gpurun_out/ab2/adaptive_chunk$cm.json 2>&1 || exit $?
  echo "chunk $cm"; tail -1 gpurun_out/ab2/adaptive_chunk$cm.json
done
for wg in 4 2 3; do
  PROBE_WG=$wg timeout -k 10 150 python3 tools/cfg_probe.py C2 16384 64 > gpurun_out/ab2/c2_wg$wg.json 2>&1 || exit $?
  echo "C2 wg $wg"; tail -1 gpurun_out/ab2/c2_wg$wg.json | cut -c1-250
done
