#!/bin/bash
# round 4 call 14: the full GPU suite as the driver runs it at round end, plus smoke()
set -o pipefail
mkdir -p gpurun_out/r4_14
timeout -k 10 1050 python -u -m pytest tests -x -v -m gpu --timeout 450 --timeout-method thread > gpurun_out/r4_14/gpu_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r4_14/gpu_suite.log
grep -E "FAILED|Error" gpurun_out/r4_14/gpu_suite.log | head -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_14/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/r4_14/smoke.log
exit $rc
