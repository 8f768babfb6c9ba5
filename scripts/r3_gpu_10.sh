#!/bin/bash
# round 3, call 10: engine-core inbox thread -- serve test, bench, traced bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
summ() { python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('value','ms_per_step','p50_ttft_ms','p95_ttft_ms','p50_tpot_ms','p95_frame_gap_ms','p50_turn_latency_ms')})"; }
timeout -k 10 300 python -u -m pytest tests/test_serve_gpu.py tests/test_engine_gpu.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | summ
[ $rc -eq 0 ] || exit $rc
rm -rf $O/arr && OMNIA_TRACE_ARRIVALS=$PWD/$O/arr timeout -k 10 400 python -u bench.py > $O/bench_traced.log 2>&1
rc=$?; echo "traced bench rc=$rc"; tail -1 $O/bench_traced.log | summ
python3 scripts/arrival_spread.py $O/arr | tee $O/arrival_spread.txt
exit $rc
