set -o pipefail
OUT=gpurun_out/r2f; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "config_scale or sample_split or c4_eight" > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 bench.py --no-cpu > $OUT/prof_bench.json 2> $OUT/prof.err || exit $?
echo "kernel trace ok"
bash tools/pmc_bench.sh $OUT/pmc
