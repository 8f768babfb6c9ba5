#!/bin/bash
# round 4 call 20: the TP=2 batch-8 engine test after the fix (fp32 top-k in the TP
# sampler, as at the round-3 commit where it passed); only if it passes, the rest
# of the TP engine tests.  Per-rank logs + command trace for the first.
set -o pipefail
mkdir -p gpurun_out/r4_20/diag
timeout -k 10 300 python -u scripts/tp_diag.py gpurun_out/r4_20/diag 2 0 8 > gpurun_out/r4_20/diag.log 2>&1
rc=$?
cut -c1-600 gpurun_out/r4_20/diag.log | tail -6
[ $rc -ne 0 ] && { for f in gpurun_out/r4_20/diag/rank*.log; do echo "== $f"; grep -v "Gloo\|amdgpu" $f | tail -6 | cut -c1-300; done; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 420 --timeout-method thread tests/test_tp_gpu.py > gpurun_out/r4_20/tp_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r4_20/tp_tests.log | tail -10
exit $rc
