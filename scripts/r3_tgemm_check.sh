#!/bin/bash
# round 3: tgemm.hip numerics on the GPU, then the end-to-end decode GEMM sweep
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tgemm_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r3_tgemm_test.log 2>&1 || { echo "tgemm tests failed"; tail -30 gpurun_out/r3_tgemm_test.log; exit 1; }
tail -3 gpurun_out/r3_tgemm_test.log
timeout -k 10 500 python -u scripts/tgemm_sweep.py --table gpurun_out/r3_tgemm_winners.json \
  > gpurun_out/r3_tgemm_sweep.log 2>&1
rc=$?
cat gpurun_out/r3_tgemm_sweep.log | cut -c1-400
exit $rc
