set -o pipefail
OUT=gpurun_out/r2a; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/perf_probe.py 64 > $OUT/probe64.json 2> $OUT/probe.err || exit $?
cat $OUT/probe64.json
timeout -k 10 300 python tools/phase_probe.py 64 > $OUT/phase64.txt 2>&1 || exit $?
cat $OUT/phase64.txt
bash tools/pmc.sh $OUT/pmc 64
