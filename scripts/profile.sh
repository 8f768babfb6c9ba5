#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py ${BENCH_ARGS:---steps 1 --warmup 1} > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof_bench.log
find gpurun_out/prof -name '*stats*' | head
exit $rc
