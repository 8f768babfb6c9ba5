#!/bin/bash
# Tune prefill GEMM shapes at a larger prefill chunk, then sweep bench configs.
# Each GPU step has its own time limit; the script stops at the first failure.
mkdir -p gpurun_out
if [ -n "$TUNE_PREFILL" ]; then
  MODELS=llama-3-8b BATCHES=256 PREFILL=$TUNE_PREFILL timeout -k 10 900 \
    python scripts/tune_gemms.py > gpurun_out/tune.log 2>&1 || exit $?
  cp omnia_amd/ops/tuned/tunableop_gfx950_0.csv gpurun_out/tuned.csv
fi
IFS=';' read -ra CONFIGS <<< "${SWEEP:---max-prefill-tokens 16384}"
for args in "${CONFIGS[@]}"; do
  echo "== $args" >> gpurun_out/sweep.log
  timeout -k 10 420 python bench.py --steps 3 --warmup 1 $args >> gpurun_out/sweep.log 2>&1 || exit $?
  tail -1 gpurun_out/sweep.log
done
