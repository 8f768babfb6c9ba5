#!/bin/bash
# serve e2e GPU test + kernel-stat profile of the engine-path bench
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_serve_gpu.py -x -v -s --timeout 360 --timeout-method thread > gpurun_out/serve_gpu.log 2>&1
rc=$?; echo "serve test rc=$rc"; tail -5 gpurun_out/serve_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
BENCH_ARGS="--path engine --steps 2 --warmup 1" bash scripts/profile.sh
