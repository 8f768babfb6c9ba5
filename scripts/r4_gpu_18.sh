#!/bin/bash
# round 4 call 18: GPU suite without the TP engine tests, smoke, the bench; then
# (last) the TP=2 batch-8 engine test alone under a kernel trace (fault bisect)
set -o pipefail
mkdir -p gpurun_out/r4_18
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --ignore=tests/test_tp_gpu.py --timeout 450 --timeout-method thread > gpurun_out/r4_18/gpu_suite.log 2>&1
rc=$?
tail -4 gpurun_out/r4_18/gpu_suite.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r4_18/gpu_suite.log | head -10; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_18/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/r4_18/smoke.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r4_18/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r4_18/bench.log | cut -c1-600
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4_18/tp_trace -- python3 -u -m pytest -x -v -s --timeout 250 --timeout-method thread "tests/test_tp_gpu.py::test_tp_engine_on_one_gpu_matches_dense_oracle[2-False-8-0]" > gpurun_out/r4_18/tp.log 2>&1
rc=$?
grep -E "PASSED|FAILED|illegal" gpurun_out/r4_18/tp.log | head -5
exit $rc
