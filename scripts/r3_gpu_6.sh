#!/bin/bash
# round 3, call 6: 32-k-stage tgemm variants (tests + M=256 sweep -> table), mixed-step
# hand-off tests, closed-loop bench separate vs mixed, open-loop separate vs mixed.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_tgemm_gpu.py tests/test_engine_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/tgemm_sweep.py --m 256 --shapes qkv,o,gate_up,down,lm_head --bn 128,256 --out $O/tgemm_sweep.json --table omnia_amd/ops/tuned/wgemm_mi355x.json --min-gain 1.0 2>&1 | tee $O/tgemm_sweep.log
rc=$?; echo "sweep rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp omnia_amd/ops/tuned/wgemm_mi355x.json $O/wgemm_mi355x.json
for mb in 0 16384; do
  timeout -k 10 600 python -u bench.py --mixed-budget $mb > $O/closed_mb$mb.log 2>&1
  rc=$?; echo "closed mixed_budget=$mb rc=$rc"; tail -1 $O/closed_mb$mb.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('value','ms_per_step','p50_ttft_ms','p50_tpot_ms','p95_frame_gap_ms','p50_turn_latency_ms')})"
  [ $rc -eq 0 ] || exit $rc
done
