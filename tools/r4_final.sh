#!/bin/bash
# Round-4 final evidence per config: the PMC passes first (copied into profiles/round4 so
# the bench line that follows carries them), then the bench under rocprofv3
# kernel-trace stats.  usage: tools/r3_final.sh OUTDIR configs...
OUT=${1:-gpurun_out/final}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
for c in "$@"; do
  bash "$ROOT/tools/pmc_bench.sh" "$OUT/pmc_$c" --config $c
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cp "$OUT/pmc_$c/pmc.json" "$ROOT/profiles/round4/pmc_bench_$c.json"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o bench --output-format csv -- python3 "$ROOT/bench.py" --config $c --no-cpu > "$OUT/prof_$c.json" 2> "$OUT/prof_$c.err")
  rc=$?; echo "prof $c rc=$rc"; tail -1 "$OUT/prof_$c.json" | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
