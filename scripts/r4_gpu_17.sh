#!/bin/bash
# round 4 call 17: decode attention partition sweep, then the full GPU suite + smoke
set -o pipefail
mkdir -p gpurun_out/r4_17
timeout -k 10 180 python -u scripts/decode_attn_sweep.py > gpurun_out/r4_17/attn_sweep.log 2>&1 || exit $?
cat gpurun_out/r4_17/attn_sweep.log | grep -v amdgpu.ids
OMNIA_DECODE_UG=1 timeout -k 10 180 python -u scripts/decode_attn_sweep.py > gpurun_out/r4_17/attn_sweep_ug1.log 2>&1 || exit $?
cat gpurun_out/r4_17/attn_sweep_ug1.log | grep -v amdgpu.ids
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 450 --timeout-method thread > gpurun_out/r4_17/gpu_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r4_17/gpu_suite.log
grep -E "FAILED|Error" gpurun_out/r4_17/gpu_suite.log | head -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_17/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/r4_17/smoke.log
exit $rc
