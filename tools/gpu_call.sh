#!/bin/bash
# The one parametrised GPU-box driver: each STEP runs under its own time limit
# and the first failing step ends the call (no retries, nothing after a fault).
#   usage: tools/gpu_call.sh OUTDIR STEP [STEP ...]
# STEPs
#   tests                 pytest -m gpu (whole suite)            tests:EXPR  only -k EXPR
#   smoke                 __graft_entry__.smoke()
#   bench:CFG[:ARGS]      bench.py --config CFG, ARGS comma-separated (e.g. bench:C3:--steps,2)
#   dist:CFG              bench.py --force-dist: the N > 1 step (RCCL group, per-pixel sums,
#                         device reduce) at world size 1, frame dumped beside the plain one
#   ab:SPP:REPS:H1,H2     interleaved same-box A/B of device-library headers on the C3
#                         frame at SPP (tools/ab/ab.sh; "-" = the built-in library)
#   defs:SPP:REPS:D1|D2   the same for PT_DEVICE_DEFINES variants (tools/ab/defs.sh)
#   cfg:CFG,NPIX,SPP:REPS:S1|S2   A/B on tools/cfg_probe.py (hashed pixels of a config); a spec
#                         is "-" or VAR=value[,VAR=value] (PT_DEVICE_HEADER=..., PT_DEVICE_DEFINES=...)
#   benchab:CFG:REPS:S1|S2   whole bench.py runs (--no-cpu) under env specs, interleaved
#                         (tools/ab/bench_env.sh; spec "-" or VAR=value[,VAR=value])
#   phase:SPP             PT_PHASE_TIMING phase split of the C3 frame (tools/phase_probe.py)
#   shards:CFG:WORLD:SPP:SPLIT:TILE:DEAL   tools/shard_times.py (each rank's share on this GPU)
#   evidence:CFG          the bench line's evidence, bound to the timed code object:
#                         PMC passes (tools/pmc_bench.sh) -> profiles/round6/pmc_bench_CFG.json,
#                         then bench.py under rocprofv3 --kernel-trace --stats ->
#                         profiles/round6/bench_CFG_{rocprof.json,kernel_stats.csv}
#                         (also kept under OUTDIR/round6/: only gpurun_out/ comes back from the box)
OUT=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; OUT=$(cd "$OUT" && pwd)
PROF="$ROOT/profiles/round6"; mkdir -p "$PROF"
cd "$ROOT"
run() {  # run LIMIT LOG cmd...
    lim=$1; log=$2; shift 2
    timeout -k 10 "$lim" "$@" > "$log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; tail -20 "$log"; exit $rc; fi
}
for step in "$@"; do
  IFS=: read -r kind a b c <<< "$step"
  case $kind in
  tests)
    if [ -n "$a" ]; then K=(-k "$a"); else K=(); fi
    run 900 "$OUT/gpu_tests.log" python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ "${K[@]}"
    tail -1 "$OUT/gpu_tests.log" ;;
  smoke)
    run 300 "$OUT/smoke.log" python3 -c "import __graft_entry__ as g; g.smoke()"
    tail -1 "$OUT/smoke.log" ;;
  bench)
    IFS=, read -r -a EXTRA <<< "$b"
    tag=$a; [ -n "$b" ] && tag="${a}_$(echo "$b" | tr -c 'A-Za-z0-9' '_')"
    run 900 "$OUT/bench_$tag.log" python3 bench.py --config "$a" "${EXTRA[@]}"
    grep '^{' "$OUT/bench_$tag.log" > "$OUT/bench_$tag.json"; cut -c1-400 "$OUT/bench_$tag.json" ;;
  dist)
    run 900 "$OUT/plain_$a.log" python3 bench.py --config "$a" --no-cpu --dump-frame "$OUT/plain_$a.npy"
    run 900 "$OUT/dist_$a.log" python3 bench.py --config "$a" --no-cpu --force-dist --dump-frame "$OUT/dist_$a.npy"
    grep '^{' "$OUT/dist_$a.log" | cut -c1-400
    python3 -c "import numpy as np,sys; a=np.load(sys.argv[1]); b=np.load(sys.argv[2]); print('force-dist frame: %d of %d values differ from the plain frame' % ((a.view(np.uint32)!=b.view(np.uint32)).sum(), a.size))" "$OUT/plain_$a.npy" "$OUT/dist_$a.npy"
    rm -f "$OUT/plain_$a.npy" "$OUT/dist_$a.npy" ;;
  ab)
    IFS=, read -r -a HS <<< "$c"
    run 1200 "$OUT/ab_$a.txt" bash tools/ab/ab.sh "$a" "$b" "${HS[@]}"; cat "$OUT/ab_$a.txt" ;;
  defs)
    IFS='|' read -r -a DS <<< "$c"
    run 1200 "$OUT/defs_$a.txt" bash tools/ab/defs.sh "$a" "$b" "${DS[@]}"; cat "$OUT/defs_$a.txt" ;;
  cfg)
    IFS='|' read -r -a SP <<< "$c"
    run 1200 "$OUT/cfg_${a//,/_}.txt" bash tools/ab/cfg_hdr_ab.sh "$OUT/cfgp" "$b" "${a//,/ }" "${SP[@]}"
    cat "$OUT/cfg_${a//,/_}.txt" ;;
  benchab)
    IFS='|' read -r -a SP <<< "$c"
    run 1500 "$OUT/benchab_$a.txt" bash tools/ab/bench_env.sh "$a" "$b" "${SP[@]}"; cat "$OUT/benchab_$a.txt" ;;
  shards)
    IFS=: read -r _ a b c d e f <<< "$step"
    tag="${a}_${b}_${c}_${d}_${e}_${f}"
    run 900 "$OUT/shards_$tag.jsonl" python3 tools/shard_times.py "$a" "$b" "$c" "$d" "$e" "$f"
    tail -1 "$OUT/shards_$tag.jsonl" ;;
  phase)
    run 600 "$OUT/phase_$a.txt" python3 tools/phase_probe.py "$a"; cat "$OUT/phase_$a.txt" ;;
  evidence)
    run 1500 "$OUT/pmc_$a.log" bash tools/pmc_bench.sh "$OUT/pmc_$a" --config "$a"
    cp "$OUT/pmc_$a/pmc.json" "$PROF/pmc_bench_$a.json"  # the line under rocprof below attaches it
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$a" -o bench \
        --output-format csv -- python3 "$ROOT/bench.py" --config "$a" --no-cpu > "$OUT/prof_$a.log" 2>&1)
    rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: rocprofv3 bench $a"; tail -20 "$OUT/prof_$a.log"; exit $rc; }
    grep '^{' "$OUT/prof_$a.log" > "$PROF/bench_${a}_rocprof.json"
    cp "$(find "$OUT/prof_$a" -name '*kernel_stats.csv' | head -1)" "$PROF/bench_${a}_kernel_stats.csv"
    mkdir -p "$OUT/round6"; cp "$PROF/pmc_bench_$a.json" "$PROF/bench_${a}_rocprof.json" "$PROF/bench_${a}_kernel_stats.csv" "$OUT/round6/"
    cut -c1-300 "$PROF/bench_${a}_rocprof.json"; head -3 "$PROF/bench_${a}_kernel_stats.csv" ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
