#!/bin/bash
# dgemm numerics then the decode-GEMM sweep
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dgemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dgemm_tests.log 2>&1
rc=$?; echo "dgemm tests rc=$rc"; tail -15 gpurun_out/dgemm_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/dgemm_sweep.py ${SWEEP_ARGS} > gpurun_out/dgemm_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/dgemm_sweep.log | tail -60
exit $rc
