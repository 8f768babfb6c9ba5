#!/bin/bash
mkdir -p gpurun_out/chunk
for c in 32768 16384 24576; do
  timeout -k 10 600 python -u bench.py --max-prefill-tokens $c > gpurun_out/chunk/c$c.log 2>&1
  rc=$?; echo "chunk $c rc=$rc $(tail -1 gpurun_out/chunk/c$c.log | grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*')"
  [ $rc -eq 0 ] || exit $rc
done
