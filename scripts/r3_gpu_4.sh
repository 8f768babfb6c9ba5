#!/bin/bash
# round 3, call 4: compute-queue staging upload + LM-head tile-kernel sweep, bench + gaps.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_staging_gpu.py tests/test_tgemm_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/kern_tests.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -3 $O/kern_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tgemm_sweep.py --shapes lm_head --m 256,128,64 --bn 128,256 --out $O/lm_head_sweep.json --table omnia_amd/ops/tuned/wgemm_mi355x.json --min-gain 1.02 2>&1 | tee $O/lm_head_sweep.log
rc=$?; echo "lm sweep rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp omnia_amd/ops/tuned/wgemm_mi355x.json $O/wgemm_mi355x.json
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_model_correctness.py -m gpu -q --timeout 300 --timeout-method thread > $O/engine_tests.log 2>&1
rc=$?; echo "engine tests rc=$rc"; tail -3 $O/engine_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r3cprof -o run -- python3 bench.py --steps 2 --warmup 1 > $O/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 $O/prof_bench.log | cut -c1-300
TR=$(find /tmp/r3cprof -name '*kernel_trace.csv' | head -1)
python3 scripts/gap_analysis.py $TR $O/gaps.md > /dev/null
gzip -c $TR > $O/kernel_trace.csv.gz
cp $(find /tmp/r3cprof -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv
sed -n 1,30p $O/gaps.md
exit $rc
