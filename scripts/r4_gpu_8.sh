#!/bin/bash
# round 4 call 8: pipelined EP decode on one GPU (EP 2/4/8 + CP), 1-GPU bench (incremental
# UTF-8 detokenizer), open-loop poisson A/B of mixed steps
set -o pipefail
mkdir -p gpurun_out/r4_8
timeout -k 10 900 python -u -m pytest -v -s --timeout 450 --timeout-method thread tests/test_ep_cp_gpu.py > gpurun_out/r4_8/ep_cp.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|EP=|CP=" gpurun_out/r4_8/ep_cp.log | cut -c1-400 | tail -20
[ $rc -ne 0 ] && { tail -60 gpurun_out/r4_8/ep_cp.log; exit $rc; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r4_8/bench.log 2>&1 || { tail -30 gpurun_out/r4_8/bench.log; exit 1; }
tail -1 gpurun_out/r4_8/bench.log | cut -c1-1200
for mb in 0 16384; do
  timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --arrival poisson --rate 76 --mixed-budget $mb > gpurun_out/r4_8/poisson_mb$mb.log 2>&1 || { tail -30 gpurun_out/r4_8/poisson_mb$mb.log; exit 1; }
  tail -1 gpurun_out/r4_8/poisson_mb$mb.log | cut -c1-900
done
