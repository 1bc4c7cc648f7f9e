#!/bin/bash
# HBM traffic of the benchmark's render kernel: separate rocprofv3 --pmc passes
# for FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md, HBM section) over the
# bench command itself.  usage: tools/pmc_traffic.sh OUTDIR [bench args...]
OUT=${1:-gpurun_out/traffic}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $c -d "$OUT/$c" -o $c --output-format csv -- python3 "$ROOT/bench.py" --no-cpu "$@" > "$OUT/$c.log" 2>&1
    rc=$?; echo "$c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done
python3 "$ROOT/tools/traffic_summary.py" "$OUT" > "$OUT/traffic.json" && cat "$OUT/traffic.json"
