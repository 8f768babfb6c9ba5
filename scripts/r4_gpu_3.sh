#!/bin/bash
# round 4 call 3: pgemm variant A/B + rocprofv3 kernel stats of the WS bench (fused prefill)
set -o pipefail
mkdir -p gpurun_out/r4_3
timeout -k 10 400 python -u scripts/pgemm_variants.py > gpurun_out/r4_3/variants.log 2>&1 || { echo "variants failed"; tail -30 gpurun_out/r4_3/variants.log; exit 1; }
cat gpurun_out/r4_3/variants.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_3/prof -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/r4_3/bench_prof.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/r4_3/bench_prof.log; exit 1; }
tail -1 gpurun_out/r4_3/bench_prof.log
find gpurun_out/r4_3/prof -name "*kernel_stats.csv" | head -3
