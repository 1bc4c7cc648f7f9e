#!/bin/bash
# Full benchmark + its rocprofv3 kernel-trace summary + HBM traffic passes.
# usage: tools/round_profile.sh OUTDIR
OUT=${1:-gpurun_out/round}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
timeout -k 10 400 python3 "$ROOT/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; exit 1; }
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- python3 "$ROOT/bench.py" > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { echo "prof rc=$?"; exit 1; }
echo "kernel trace done"
bash "$ROOT/tools/pmc_traffic.sh" "$OUT/traffic"
