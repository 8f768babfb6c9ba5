#!/bin/bash
# round 3: full GPU suite (incl. tgemm + TP-on-one-GPU), WS bench, kernel-stats profile
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-700
[ $rc -eq 0 ] || { tail -30 $O/bench.log; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 420 --timeout-method thread > $O/gpu_tests.log 2>&1
trc=$?; echo "gpu tests rc=$trc"; grep -E "passed|failed|error" $O/gpu_tests.log | tail -3
grep -E "^TP=|FAILED" $O/gpu_tests.log | head
[ $trc -eq 0 ] || grep -B5 -A30 "Error" $O/gpu_tests.log | head -60
[ $trc -eq 0 ] || [ $trc -eq 1 ] || exit $trc  # a crash / timeout: nothing more on the GPU
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r3prof -o run -- python3 bench.py --steps 2 --warmup 1 > $O/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 $O/prof_bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
cp $(find /tmp/r3prof -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv
python3 scripts/gap_analysis.py $(find /tmp/r3prof -name '*kernel_trace.csv' | head -1) $O/gaps.md > /dev/null
head -25 $O/kernel_stats.csv | cut -c1-200
echo done
exit $trc
