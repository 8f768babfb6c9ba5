#!/bin/bash
# round 4 call 1: pgemm numerics + prefill sweep vs hipBLASLt
set -o pipefail
mkdir -p gpurun_out/r4_1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pgemm_gpu.py > gpurun_out/r4_1/test.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r4_1/test.log; exit 1; }
tail -3 gpurun_out/r4_1/test.log
timeout -k 10 400 python -u scripts/pgemm_sweep.py --out gpurun_out/r4_1/sweep.json > gpurun_out/r4_1/sweep.log 2>&1
rc=$?
cat gpurun_out/r4_1/sweep.log
exit $rc
