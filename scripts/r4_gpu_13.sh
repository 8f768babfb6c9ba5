#!/bin/bash
# round 4 call 13: locate the TP mixed-step fault of call 12 (serialized kernels: the
# failing launch raises at its own call site)
set -o pipefail
mkdir -p gpurun_out/r4_13
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread "tests/test_tp_gpu.py" -k "256" > gpurun_out/r4_13/tp_mixed_serial.log 2>&1
rc=$?
grep -E "PASSED|FAILED|TP=" gpurun_out/r4_13/tp_mixed_serial.log | cut -c1-300 | tail -4
grep -n -B2 -A30 "Traceback" gpurun_out/r4_13/tp_mixed_serial.log | grep -E "File|Error" | head -40
exit $rc
