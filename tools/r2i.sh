#!/bin/bash
# Round-2 evidence run: C2/config-scale GPU tests, C3 bench under rocprofv3
# kernel trace, PMC passes of the C3 bench, C2 and C5 bench lines.
set -o pipefail
O=gpurun_out/r2i; mkdir -p $O; R=$(pwd)
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "C2 or config_scale or c2" > $O/gpu.log 2>&1 || exit 1
echo "tests ok"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_c3 -o c3 --output-format csv -- python3 $R/bench.py > $R/$O/bench_c3.json 2> $R/$O/bench_c3.err) || exit 2
echo "c3 ok"
timeout -k 10 900 tools/pmc_bench.sh $O/pmc_c3 > $O/pmc_c3.log 2>&1 || exit 3
echo "pmc ok"
timeout -k 10 400 python -u bench.py --config C2 > $O/bench_c2.json 2> $O/bench_c2.err || exit 4
echo "c2 ok"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_c5 -o c5 --output-format csv -- python3 $R/bench.py --config C5 > $R/$O/bench_c5.json 2> $R/$O/bench_c5.err) || exit 5
echo "c5 ok"
