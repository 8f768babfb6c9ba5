#!/bin/bash
# CP kernel path + prefill/model correctness GPU tests
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cp_serving.py tests/test_kernels_gpu.py tests/test_model_correctness.py tests/test_context_parallel.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/cp_gpu.log 2>&1
rc=$?; echo "rc=$rc"; tail -5 gpurun_out/cp_gpu.log
exit $rc
