#!/bin/bash
# Per device-header variant: the C3 phase split (PT_PHASE_TIMING build) and two
# PMC passes (issue mix, wave-cycle split) of the 64-spp probe.
# usage: tools/ab/diag.sh OUTDIR header...   ("-" = the built-in library)
OUT=$1; shift
mkdir -p "$OUT"
for h in "$@"; do
    if [ "$h" = "-" ]; then unset PT_DEVICE_HEADER; name=cur; else export PT_DEVICE_HEADER=$(readlink -f "$h"); name=$(basename "$h" .h); fi
    timeout -k 10 300 python tools/phase_probe.py 64 > "$OUT/phase_$name.txt" 2>&1 || exit $?
    echo "== $name"; cat "$OUT/phase_$name.txt" | tail -20
    bash tools/pmc_quick.sh "$OUT/pmc_$name" 64 > "$OUT/pmc_$name.txt" 2>&1 || exit $?
    tail -30 "$OUT/pmc_$name.txt"
done
