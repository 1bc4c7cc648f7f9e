#!/bin/bash
# Same-box A/B of device-library variants on config probes.
# usage: tools/ab/cfg_hdr_ab.sh OUT REPS "CONFIG NPIX SPP" spec...   (spec: "-" or VAR=value[,VAR=value])
OUT=$1; REPS=$2; PROBE=$3; shift 3; mkdir -p $OUT
for r in $(seq $REPS); do
  for spec in "$@"; do
    envs=(); [ "$spec" != "-" ] && IFS=, read -ra envs <<< "$spec"
    env "${envs[@]}" timeout -k 10 200 python3 tools/cfg_probe.py $PROBE > $OUT/p.json 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('%-14s %-40s %9.3f Msamples/s  kernel %9.1f ms' % (d['config'], sys.argv[2], d['Msamples_per_s'], d['kernel_ms']))" $OUT/p.json "$spec"
  done
done
