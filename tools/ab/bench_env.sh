#!/bin/bash
# Interleaved same-box A/B of whole bench.py runs under environment specs
# (each "-" or VAR=value[,VAR=value]).  usage: tools/ab/bench_env.sh CONFIG REPS spec...
CFG=$1; REPS=$2; shift 2
for r in $(seq "$REPS"); do
  for spec in "$@"; do
    envs=(); [ "$spec" != "-" ] && IFS=, read -ra envs <<< "$spec"
    out=$(env "${envs[@]}" timeout -k 10 600 python3 bench.py --config "$CFG" --no-cpu 2>/dev/null | grep '^{') || exit $?
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('%-4s %-36s %9.3f Msamples/s  %9.1f ms/frame' % (sys.argv[2], sys.argv[3], d['value'], d['ms_per_step']))" "$out" "$CFG" "$spec"
  done
done
