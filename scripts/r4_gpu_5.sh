#!/bin/bash
# round 4 call 5: multi-rank serving modes on one MI355X (EP a2a 2/4/8, CP 2/4, TP pipelined b64)
set -o pipefail
mkdir -p gpurun_out/r4_5
timeout -k 10 900 python -u -m pytest -v -s --timeout 450 --timeout-method thread tests/test_ep_cp_gpu.py > gpurun_out/r4_5/ep_cp.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|EP=|CP=" gpurun_out/r4_5/ep_cp.log | cut -c1-600 | tail -20
[ $rc -ne 0 ] && { tail -60 gpurun_out/r4_5/ep_cp.log; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 450 --timeout-method thread "tests/test_tp_gpu.py" -k "True" > gpurun_out/r4_5/tp.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|TP=" gpurun_out/r4_5/tp.log | cut -c1-600 | tail -20
[ $rc -ne 0 ] && tail -60 gpurun_out/r4_5/tp.log
exit $rc
