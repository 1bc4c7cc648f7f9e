set -o pipefail
OUT=gpurun_out/r2e; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "c4_eight or benchmark_configs" > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
cat $OUT/bench_c2.json
timeout -k 10 300 python bench.py --config C5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit $?
cat $OUT/bench_c5.json
timeout -k 10 400 python tools/shard_times.py C4 8 4096 > $OUT/shards_c4.jsonl 2> $OUT/shards.err || exit $?
tail -1 $OUT/shards_c4.jsonl
