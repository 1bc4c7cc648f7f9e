#!/bin/bash
# Round-3 evidence: per config, the bench's rocprofv3 kernel-trace summary and
# its PMC passes (tools/pmc_bench.sh), each step under its own limit.
# usage: tools/r3_evidence.sh OUTDIR [configs...]
OUT=${1:-gpurun_out/r3ev}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
CFGS=("$@"); [ ${#CFGS[@]} -gt 0 ] || CFGS=(C3 C5)
for c in "${CFGS[@]}"; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o bench --output-format csv -- python3 "$ROOT/bench.py" --config $c --no-cpu > "$OUT/prof_$c.json" 2> "$OUT/prof_$c.err")
  rc=$?; echo "prof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  bash "$ROOT/tools/pmc_bench.sh" "$OUT/pmc_$c" --config $c
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
