#!/bin/bash
# round 4 call 21: the round-end GPU tiers at HEAD -- full GPU suite (TP engine
# cases skipped by default), smoke, the driver's bench command, then a kernel
# trace of a short bench for the per-kernel breakdown
set -o pipefail
mkdir -p gpurun_out/r4_21
timeout -k 10 800 python -u -m pytest tests -x -v -m gpu --timeout 450 --timeout-method thread > gpurun_out/r4_21/gpu_suite.log 2>&1
rc=$?
tail -3 gpurun_out/r4_21/gpu_suite.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r4_21/gpu_suite.log | head -10; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_21/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r4_21/smoke.log | cut -c1-200
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_21/bench_driver_cmd.log 2>&1 || exit $?
tail -1 gpurun_out/r4_21/bench_driver_cmd.log | cut -c1-400
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_21/prof -- python3 -u bench.py --steps 3 --warmup 1 > gpurun_out/r4_21/bench_prof.log 2>&1
rc=$?
ls gpurun_out/r4_21/prof | head
exit $rc
