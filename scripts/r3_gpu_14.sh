#!/bin/bash
# round 3, re-entry check at HEAD: the driver's bench command, smoke, full GPU suite
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-900
[ $rc -eq 0 ] || { tail -30 $O/bench.log; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 420 --timeout-method thread > $O/gpu_tests.log 2>&1
trc=$?; echo "gpu tests rc=$trc"; grep -E "passed|failed|error" $O/gpu_tests.log | tail -3
grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
exit $trc
