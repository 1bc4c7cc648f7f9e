#!/bin/bash
# Interleaved C3 A/B probes between environment settings in one GPU session.
# usage: tools/ab_env.sh SPP REPS spec1 [spec2 ...]
#   spec = "-" (built-in) or VAR=value[,VAR=value] (e.g. PT_JIT_OPTIONS=-fno-slp-vectorize)
SPP=$1; REPS=$2; shift 2
for r in $(seq "$REPS"); do
    for s in "$@"; do
        envs=()
        [ "$s" != "-" ] && IFS=, read -ra envs <<< "$s"
        out=$(env "${envs[@]}" timeout -k 10 300 python tools/perf_probe.py "$SPP" 2>/dev/null) || exit $?
        python -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('%-44s %7.2f Msamples/s  kernel %8.1f ms' % (sys.argv[2], d['Msamples_per_s'], d['kernel_ms']))" "$out" "$s"
    done
done
