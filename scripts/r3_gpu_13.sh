#!/bin/bash
# round 3, call 13: mixed vs separate steps (closed + open loop) on the current
# host path, decode attention page-size / schedule sweep.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3l
mkdir -p $O
summ() { python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('value','ms_per_step','p50_ttft_ms','p95_ttft_ms','p50_tpot_ms','p95_tpot_ms','p95_frame_gap_ms','p50_turn_latency_ms')})"; }
for mb in 16384 0; do
  timeout -k 10 400 python -u bench.py --mixed-budget $mb > $O/closed_mb$mb.log 2>&1
  rc=$?; echo "closed mixed_budget=$mb rc=$rc"; tail -1 $O/closed_mb$mb.log | summ
  [ $rc -eq 0 ] || exit $rc
done
for mb in 2048 0; do
  timeout -k 10 400 python -u bench.py --arrival poisson --rate 75 --steps 2 --warmup 1 --mixed-budget $mb > $O/ol_mb$mb.log 2>&1
  rc=$?; echo "open-loop mixed_budget=$mb rc=$rc"; tail -1 $O/ol_mb$mb.log | summ
  [ $rc -eq 0 ] || exit $rc
done
for bs in 32 64; do
  timeout -k 10 200 python -u scripts/attn_bench.py --ctx 576,2048 --parts 512,1024 --bs $bs > $O/attn_bs$bs.log 2>&1
  rc=$?; echo "attn bs=$bs rc=$rc"; tail -6 $O/attn_bs$bs.log
  [ $rc -eq 0 ] || exit $rc
done
