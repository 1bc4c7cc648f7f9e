#!/bin/bash
# Phase split of one C2 bright-sphere launch (4 samples), fast spine.
OUT=${1:-gpurun_out/c2ph}; mkdir -p "$OUT"
PT_DEVICE_DEFINES=PT_PHASE_TIMING PT_PHASE_DUMP=1 PROBE_FAST_SPINE=1 timeout -k 10 150 python3 tools/cfg_probe.py C2 4 1 disk:429:397:30 > "$OUT/ph.txt" 2>&1
rc=$?; cat "$OUT/ph.txt"; exit $rc
