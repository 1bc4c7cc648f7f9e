#!/bin/bash
# Round-4 records: adaptive caller vs full frame (C3 16 spp) and the C4 shard
# balance of both N>1 partitions at 8 ranks (each rank's share on one GPU).
OUT=${1:-gpurun_out/r4x}; mkdir -p "$OUT"
timeout -k 10 300 python3 tools/probe_adaptive.py C3 16 > "$OUT/adaptive_c3_16.json" 2> "$OUT/adaptive.err" || exit $?
cat "$OUT/adaptive_c3_16.json"
for s in samples tiles; do
  timeout -k 10 400 python3 tools/shard_times.py C4 8 0 $s > "$OUT/shards_c4_$s.jsonl" 2> "$OUT/shards_$s.err" || exit $?
  tail -1 "$OUT/shards_c4_$s.jsonl"
done
