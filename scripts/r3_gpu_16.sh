#!/bin/bash
# round 3: rocprofv3 kernel stats + idle-gap summary of the WS bench at HEAD
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r3prof -o run -- python3 bench.py --steps 3 --warmup 1 > $O/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 $O/prof_bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
cp $(find /tmp/r3prof -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv
python3 scripts/gap_analysis.py $(find /tmp/r3prof -name '*kernel_trace.csv' | head -1) $O/gaps.md > /dev/null
head -22 $O/kernel_stats.csv | cut -c1-160
echo done
