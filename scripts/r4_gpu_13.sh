#!/bin/bash
# round 4 call 13: default engine (backlog-gated mixed steps on) closed + open loop, then
# locate the TP mixed-step fault of call 12 (serialized kernels: the failing launch raises at
# its own call site) -- last, so nothing runs on the GPU after a fault
set -o pipefail
mkdir -p gpurun_out/r4_13
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r4_13/closed_default.log 2>&1 || { tail -30 gpurun_out/r4_13/closed_default.log; exit 1; }
tail -1 gpurun_out/r4_13/closed_default.log | cut -c1-600
timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --arrival poisson --rate 76 > gpurun_out/r4_13/poisson_default.log 2>&1 || { tail -30 gpurun_out/r4_13/poisson_default.log; exit 1; }
tail -1 gpurun_out/r4_13/poisson_default.log | cut -c1-600
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread "tests/test_tp_gpu.py" -k "256" > gpurun_out/r4_13/tp_mixed_serial.log 2>&1
rc=$?
grep -E "PASSED|FAILED|TP=" gpurun_out/r4_13/tp_mixed_serial.log | cut -c1-300 | tail -4
grep -n -A40 "Traceback" gpurun_out/r4_13/tp_mixed_serial.log | grep -E "File|Error" | head -40
exit $rc
