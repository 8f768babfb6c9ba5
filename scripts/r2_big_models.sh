#!/bin/bash
# single-GPU 70B and Mixtral re-measure on the round-2 kernels + the headline at 5 steps
mkdir -p gpurun_out/big
timeout -k 10 900 python -u bench.py --model llama-3-70b --path engine --concurrency 128 --steps 2 --warmup 1 > gpurun_out/big/llama70b.log 2>&1
rc=$?; echo "70b rc=$rc"; tail -1 gpurun_out/big/llama70b.log | cut -c1-360
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --path engine --concurrency 128 --steps 2 --warmup 1 > gpurun_out/big/mixtral.log 2>&1
rc=$?; echo "mixtral rc=$rc"; tail -1 gpurun_out/big/mixtral.log | cut -c1-360
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 > gpurun_out/big/headline5.log 2>&1
rc=$?; echo "headline rc=$rc"; tail -1 gpurun_out/big/headline5.log | cut -c1-360
exit $rc
