#!/bin/bash
# round 3, call 5: device token hand-off + pipelined mixed steps: GPU engine tests,
# closed-loop bench separate vs mixed, open-loop separate vs mixed.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_model_correctness.py tests/test_serve_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $O/engine_tests.log 2>&1
rc=$?; echo "engine tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/engine_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
for mb in 0 16384 4096; do
  timeout -k 10 600 python -u bench.py --mixed-budget $mb > $O/closed_mb$mb.log 2>&1
  rc=$?; echo "closed mixed_budget=$mb rc=$rc"; tail -1 $O/closed_mb$mb.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('value','ms_per_step','p50_ttft_ms','p50_tpot_ms','p95_frame_gap_ms','p50_turn_latency_ms')})"
  [ $rc -eq 0 ] || exit $rc
done
for mb in 0 2048; do
  timeout -k 10 400 python -u bench.py --arrival poisson --rate 75 --steps 2 --warmup 1 --mixed-budget $mb > $O/ol_mb$mb.log 2>&1
  rc=$?; echo "open-loop mixed_budget=$mb rc=$rc"; tail -1 $O/ol_mb$mb.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('value','p50_ttft_ms','p95_ttft_ms','p50_tpot_ms','p95_tpot_ms','p95_frame_gap_ms','p50_turn_latency_ms')})"
  [ $rc -eq 0 ] || exit $rc
done
