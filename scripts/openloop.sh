#!/bin/bash
# Open-loop (poisson arrivals) WS bench at a fixed rate, separate vs mixed steps.
mkdir -p gpurun_out
RATE=${RATE:-75}
for mb in ${BUDGETS:-0 512}; do
  timeout -k 10 400 python -u bench.py --arrival poisson --rate $RATE --steps ${STEPS:-2} --warmup 1 --mixed-budget $mb > gpurun_out/ol_mb$mb.log 2>&1
  rc=$?; echo "mixed_budget=$mb rc=$rc"; tail -1 gpurun_out/ol_mb$mb.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('value','p50_ttft_ms','p95_ttft_ms','p50_tpot_ms','p95_tpot_ms','p95_frame_gap_ms','p50_turn_latency_ms')})"
  [ $rc -eq 0 ] || exit $rc
done
