#!/bin/bash
# round 4 call 2: fused prefill path through the engine (oracle gate) + WS bench A/B
set -o pipefail
mkdir -p gpurun_out/r4_2
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_model_correctness.py -k "gpu_llama3_8b" > gpurun_out/r4_2/test.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4_2/test.log; exit 1; }
grep -E "passed|failed|worst" gpurun_out/r4_2/test.log | tail -5
timeout -k 10 420 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r4_2/bench_pgemm.log 2>&1 || { echo "bench pgemm failed"; tail -30 gpurun_out/r4_2/bench_pgemm.log; exit 1; }
tail -1 gpurun_out/r4_2/bench_pgemm.log
OMNIA_PGEMM=0 timeout -k 10 420 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r4_2/bench_lib.log 2>&1 || { echo "bench lib failed"; tail -30 gpurun_out/r4_2/bench_lib.log; exit 1; }
tail -1 gpurun_out/r4_2/bench_lib.log
