#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cp_serving.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/cp_gpu2.log 2>&1
rc=$?; echo "rc=$rc"; tail -4 gpurun_out/cp_gpu2.log
exit $rc
