#!/bin/bash
# round 4 call 10: 4-wave pgemm schedule -- correctness on both schedules, sweep vs 8-wave
# and hipBLASLt, then the bench with the 4-wave schedule
set -o pipefail
mkdir -p gpurun_out/r4_10
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pgemm_gpu.py > gpurun_out/r4_10/pgemm_test.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/r4_10/pgemm_test.log | tail -8
[ $rc -ne 0 ] && { tail -40 gpurun_out/r4_10/pgemm_test.log; exit $rc; }
timeout -k 10 300 python -u scripts/pgemm_sweep.py --schedule 0 --out gpurun_out/r4_10/sweep0.json > gpurun_out/r4_10/sweep0.log 2>&1 || { tail -20 gpurun_out/r4_10/sweep0.log; exit 1; }
timeout -k 10 300 python -u scripts/pgemm_sweep.py --schedule 1 --out gpurun_out/r4_10/sweep1.json > gpurun_out/r4_10/sweep1.log 2>&1 || { tail -20 gpurun_out/r4_10/sweep1.log; exit 1; }
grep -E "M=" gpurun_out/r4_10/sweep0.log | cut -c1-200
echo ---- 4wave
grep -E "M=" gpurun_out/r4_10/sweep1.log | cut -c1-200
