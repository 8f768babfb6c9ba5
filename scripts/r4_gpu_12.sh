#!/bin/bash
# round 4 call 12: 4-wave pgemm v2 (interleaved memory ops) sweep; EP8 Mixtral; mixed A/B
set -o pipefail
mkdir -p gpurun_out/r4_12
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pgemm_gpu.py -k "bit_identical or swiglu or qkv" > gpurun_out/r4_12/pgemm_test.log 2>&1
rc=$?; tail -3 gpurun_out/r4_12/pgemm_test.log
[ $rc -ne 0 ] && { tail -40 gpurun_out/r4_12/pgemm_test.log; exit $rc; }
timeout -k 10 300 python -u scripts/pgemm_sweep.py --schedule 1 --out gpurun_out/r4_12/sweep1.json > gpurun_out/r4_12/sweep1.log 2>&1 || { tail -20 gpurun_out/r4_12/sweep1.log; exit 1; }
grep -E "M=" gpurun_out/r4_12/sweep1.log | cut -c1-200
bash scripts/r4_gpu_9.sh || exit $?
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 450 --timeout-method thread "tests/test_tp_gpu.py" -k "256" > gpurun_out/r4_12/tp_mixed.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|TP=" gpurun_out/r4_12/tp_mixed.log | cut -c1-400 | tail -6
[ $rc -ne 0 ] && tail -40 gpurun_out/r4_12/tp_mixed.log
exit $rc
