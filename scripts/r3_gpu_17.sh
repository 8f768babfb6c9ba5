#!/bin/bash
# round 3 final: full GPU suite + smoke at HEAD
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3p
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 420 --timeout-method thread > $O/gpu_tests.log 2>&1
trc=$?; echo "gpu tests rc=$trc"; grep -E "passed|failed|error" $O/gpu_tests.log | tail -2
grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
exit $trc
