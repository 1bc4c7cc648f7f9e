#!/bin/bash
# Instruction-cache counters for the render kernel: C3 (perf_probe) and a small C2 frame.
OUT=${1:-gpurun_out/icache}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
C="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQC_TC_INST_REQ SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 --pmc $C -d "$OUT/c3" -o c3 --output-format csv -- python3 "$ROOT/tools/perf_probe.py" 8 > "$OUT/c3.log" 2>&1
rc=$?; echo "c3 rc=$rc"; case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 300 rocprofv3 --pmc $C -d "$OUT/c2" -o c2 --output-format csv -- python3 "$ROOT/tools/probe_cfg.py" C2 160 90 1 > "$OUT/c2.log" 2>&1
rc=$?; echo "c2 rc=$rc"; exit $rc
