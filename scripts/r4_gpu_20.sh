#!/bin/bash
# round 4 call 20: TP fault diagnosis -- bf16 top-k of the TP sampler in isolation
# (eager + graph), then the TP=2 batch-8 engine with per-rank logs, the command
# trace and every rank's exit code (the fault is expected in the second step)
set -o pipefail
mkdir -p gpurun_out/r4_20/diag
timeout -k 10 120 python -u scripts/topk_check.py > gpurun_out/r4_20/topk.log 2>&1
rc=$?
grep -v amdgpu gpurun_out/r4_20/topk.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/tp_diag.py gpurun_out/r4_20/diag 2 0 8 > gpurun_out/r4_20/diag.log 2>&1
rc=$?
cat gpurun_out/r4_20/diag.log | cut -c1-1500 | tail -12
for f in gpurun_out/r4_20/diag/rank*.log; do echo "== $f"; grep -v "Gloo\|amdgpu" $f | tail -8 | cut -c1-400; done
exit $rc
