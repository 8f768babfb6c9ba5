#!/bin/bash
# round 3, call 11: same-box A/B of the host-path changes (engine-core inbox
# thread, serving-process GC tuning), default measured first and last.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3j
mkdir -p $O
summ() { python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('value','ms_per_step','p50_ttft_ms','p50_tpot_ms','p95_frame_gap_ms','p50_turn_latency_ms')})"; }
run() {
  tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py > $O/bench_$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; tail -1 $O/bench_$tag.log | summ
  return $rc
}
run default OMNIA_X=1 && run noinbox OMNIA_CORE_INBOX_THREAD=0 && run nogc OMNIA_GC_THRESHOLD=off && run both_off OMNIA_CORE_INBOX_THREAD=0 OMNIA_GC_THRESHOLD=off && run default2 OMNIA_X=1
