#!/bin/bash
# round 4 call 7: TP pipelined engine at batch 64 (tap snapshot fix), 1-GPU bench, and the
# open-loop (poisson, ~80 % load) A/B of mixed steps
set -o pipefail
mkdir -p gpurun_out/r4_7
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 450 --timeout-method thread "tests/test_tp_gpu.py" -k "True" > gpurun_out/r4_7/tp.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|TP=" gpurun_out/r4_7/tp.log | cut -c1-600 | tail -20
[ $rc -ne 0 ] && { tail -60 gpurun_out/r4_7/tp.log; exit $rc; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r4_7/bench.log 2>&1 || { tail -30 gpurun_out/r4_7/bench.log; exit 1; }
tail -1 gpurun_out/r4_7/bench.log | cut -c1-900
for mb in 0 16384; do
  timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --arrival poisson --rate 76 --mixed-budget $mb > gpurun_out/r4_7/poisson_mb$mb.log 2>&1 || { tail -30 gpurun_out/r4_7/poisson_mb$mb.log; exit 1; }
  tail -1 gpurun_out/r4_7/poisson_mb$mb.log | cut -c1-700
done
