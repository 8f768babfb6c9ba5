#!/bin/bash
# round 3: driver bench command after the idle-session-page fix (per-wave times)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1
rc=$?; echo "bench20 rc=$rc"; tail -1 $O/bench20.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('value','ms_per_step','p50_turn_latency_ms','p50_tpot_ms','wave_ms')})"
[ $rc -eq 0 ] || { tail -30 $O/bench20.log; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_projection.py -m gpu -v -s --timeout 120 --timeout-method thread > $O/proj_gpu.log 2>&1
rc=$?; echo "proj gpu rc=$rc"; grep -E "t-SNE|passed|failed" $O/proj_gpu.log
exit $rc
