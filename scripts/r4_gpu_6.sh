#!/bin/bash
# round 4 call 6: fused TP Gumbel kernel + multi-rank serving modes on one MI355X
set -o pipefail
mkdir -p gpurun_out/r4_6
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tp_gumbel_gpu.py > gpurun_out/r4_6/gumbel.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error" gpurun_out/r4_6/gumbel.log | tail -5
[ $rc -ne 0 ] && { tail -40 gpurun_out/r4_6/gumbel.log; exit $rc; }
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_tp_overlap_gpu.py > gpurun_out/r4_6/overlap.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|overlap world" gpurun_out/r4_6/overlap.log | cut -c1-800 | tail -8
[ $rc -ne 0 ] && { tail -40 gpurun_out/r4_6/overlap.log; exit $rc; }
timeout -k 10 900 python -u -m pytest -v -s --timeout 450 --timeout-method thread tests/test_ep_cp_gpu.py > gpurun_out/r4_6/ep_cp.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|EP=|CP=" gpurun_out/r4_6/ep_cp.log | cut -c1-600 | tail -20
[ $rc -ne 0 ] && { tail -60 gpurun_out/r4_6/ep_cp.log; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 450 --timeout-method thread "tests/test_tp_gpu.py" -k "True" > gpurun_out/r4_6/tp.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|TP=" gpurun_out/r4_6/tp.log | cut -c1-600 | tail -20
[ $rc -ne 0 ] && tail -60 gpurun_out/r4_6/tp.log
exit $rc
