#!/bin/bash
# round 3, call 8: register-pipelined tgemm (tests + M=256 sweep -> table), then the
# closed-loop bench separate vs mixed steps.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
summ() { python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('value','ms_per_step','p50_ttft_ms','p95_ttft_ms','p50_tpot_ms','p95_tpot_ms','p95_frame_gap_ms','p50_turn_latency_ms')})"; }
timeout -k 10 300 python -u -m pytest tests/test_tgemm_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/tgemm_tests.log 2>&1
rc=$?; echo "tgemm tests rc=$rc"; tail -3 $O/tgemm_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/tgemm_sweep.py --m 256 --shapes qkv,o,gate_up,down --bn 64,128,256 --out $O/tgemm_sweep.json --table omnia_amd/ops/tuned/wgemm_mi355x.json --min-gain 1.0 2>&1 | tee $O/tgemm_sweep.log
rc=$?; echo "sweep rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp omnia_amd/ops/tuned/wgemm_mi355x.json $O/wgemm_mi355x.json
for mb in 0 16384; do
  timeout -k 10 400 python -u bench.py --mixed-budget $mb > $O/closed_mb$mb.log 2>&1
  rc=$?; echo "closed mixed_budget=$mb rc=$rc"; tail -1 $O/closed_mb$mb.log | summ
  [ $rc -eq 0 ] || exit $rc
done
rm -rf /tmp/arr && OMNIA_TRACE_ARRIVALS=/tmp/arr timeout -k 10 400 python -u bench.py > $O/bench_traced.log 2>&1
rc=$?; echo "traced bench rc=$rc"; tail -1 $O/bench_traced.log | summ
python3 scripts/arrival_spread.py /tmp/arr | tee $O/arrival_spread.txt
exit $rc
