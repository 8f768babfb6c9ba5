#!/bin/bash
# full GPU suite + smoke + kernel-stats profile of the default (WS) bench
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/final/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/final/smoke.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/finalprof -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/final/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/final/prof_bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
cp $(find /tmp/finalprof -name '*kernel_stats.csv' | head -1) gpurun_out/final/kernel_stats.csv
python3 scripts/gap_analysis.py $(find /tmp/finalprof -name '*kernel_trace.csv' | head -1) gpurun_out/final/gaps.md > /dev/null
echo done
