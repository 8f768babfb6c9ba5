#!/bin/bash
# closed-loop headline with co-scheduled prefill + decode (mixed steps), two budgets
mkdir -p gpurun_out
for mb in 16384 8192; do
  timeout -k 10 600 python -u bench.py --mixed-budget $mb > gpurun_out/bench_mixed_$mb.log 2>&1
  rc=$?; echo "mixed $mb rc=$rc"; tail -1 gpurun_out/bench_mixed_$mb.log | cut -c1-420
  [ $rc -eq 0 ] || exit $rc
done
