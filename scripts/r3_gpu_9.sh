#!/bin/bash
# round 3, call 9: host-path diagnosis of the WS bench -- raw per-request stage
# timestamps, then Python profiles of client / facade / runtime / engine-core.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
summ() { python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('value','ms_per_step','p50_ttft_ms','p95_ttft_ms','p50_tpot_ms','p95_frame_gap_ms','p50_turn_latency_ms')})"; }
rm -rf $O/arr && OMNIA_TRACE_ARRIVALS=$PWD/$O/arr timeout -k 10 400 python -u bench.py > $O/bench_traced.log 2>&1
rc=$?; echo "traced bench rc=$rc"; tail -1 $O/bench_traced.log | summ
[ $rc -eq 0 ] || exit $rc
python3 scripts/arrival_spread.py $O/arr | tee $O/arrival_spread.txt
rm -rf $O/pyprof && OMNIA_PYPROFILE=$PWD/$O/pyprof timeout -k 10 400 python -u bench.py > $O/bench_prof.log 2>&1
rc=$?; echo "profiled bench rc=$rc"; tail -1 $O/bench_prof.log | summ
ls -la $O/pyprof
exit $rc
