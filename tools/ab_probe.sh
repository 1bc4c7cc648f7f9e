#!/bin/bash
# A/B the C3 probe between device-library texts in one GPU session, interleaved.
# usage: tools/ab_probe.sh SPP REPS header1 [header2 ...]   ("-" = built-in library)
SPP=$1; REPS=$2; shift 2
for r in $(seq "$REPS"); do
    for h in "$@"; do
        if [ "$h" = "-" ]; then
            out=$(timeout -k 10 300 python tools/perf_probe.py "$SPP" 2>/dev/null) || exit $?
        else
            out=$(PT_DEVICE_HEADER="$h" timeout -k 10 300 python tools/perf_probe.py "$SPP" 2>/dev/null) || exit $?
        fi
        python -c "import json,sys; d=json.loads(sys.argv[1].splitlines()[-1]); print('%-28s %7.2f Msamples/s  kernel %8.1f ms' % (sys.argv[2], d['Msamples_per_s'], d['kernel_ms']))" "$out" "$h"
    done
done
