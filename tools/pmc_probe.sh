#!/bin/bash
# HBM write / fetch traffic of tools/cfg_probe.py under env specs (one rocprofv3
# --pmc pass per counter and spec).  usage: tools/pmc_probe.sh OUT "CONFIG NPIX SPP" spec...
OUT=$1; PROBE=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
i=0
for spec in "$@"; do
  envs=(); [ "$spec" != "-" ] && IFS=, read -ra envs <<< "$spec"
  for ctr in WRITE_SIZE FETCH_SIZE; do
    i=$((i+1))
    env "${envs[@]}" timeout -k 10 300 rocprofv3 --pmc $ctr -d "$OUT/p$i" -o p --output-format csv -- python3 "$ROOT/tools/cfg_probe.py" $PROBE > "$OUT/p$i.log" 2>&1 || exit $?
    python3 - "$OUT/p$i" "$ctr" "$spec" "$OUT/p$i.log" <<'PY'
import csv, glob, json, sys
d, ctr, spec, log = sys.argv[1:5]
v = sum(float(r["Counter_Value"]) for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True)
        for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("pt_render_fast"))
b = [json.loads(l) for l in open(log) if l.startswith("{")][-1]
kb = v * (2 if ctr == "FETCH_SIZE" else 1)
print("%-32s %-10s %12.1f B/sample  %8.3f Msamples/s" % (spec, ctr, kb * 1024 / b["samples"], b["Msamples_per_s"]))
PY
  done
done
