#!/bin/bash
# round 4 call 9: EP=8 at Mixtral-8x7B layer shapes; closed-loop A/B of backlog-gated mixed
# steps against separate steps; open-loop poisson with the gate
set -o pipefail
mkdir -p gpurun_out/r4_12
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 650 --timeout-method thread tests/test_ep_cp_gpu.py -k mixtral > gpurun_out/r4_12/ep8_mixtral.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|EP=8" gpurun_out/r4_12/ep8_mixtral.log | cut -c1-300 | tail -12
[ $rc -ne 0 ] && { tail -40 gpurun_out/r4_12/ep8_mixtral.log; exit $rc; }
for mb in 0 16384 0 16384; do
  timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --mixed-budget $mb > gpurun_out/r4_12/closed_mb$mb.log 2>&1 || { tail -30 gpurun_out/r4_12/closed_mb$mb.log; exit 1; }
  tail -1 gpurun_out/r4_12/closed_mb$mb.log | cut -c1-420
  cat gpurun_out/r4_12/closed_mb$mb.log >> gpurun_out/r4_12/closed_all.log
done
timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --arrival poisson --rate 76 --mixed-budget 16384 > gpurun_out/r4_12/poisson_mb16384_gated.log 2>&1 || { tail -30 gpurun_out/r4_12/poisson_mb16384_gated.log; exit 1; }
tail -1 gpurun_out/r4_12/poisson_mb16384_gated.log | cut -c1-700
