#!/bin/bash
# kernel trace of the WS-path bench -> GPU idle-gap summary (trace deleted after)
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/gaps
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/wsprof -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/gaps/bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/gaps/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
for f in $(find /tmp/wsprof -name '*kernel_trace.csv'); do
  echo "== $f"; python3 scripts/gap_analysis.py "$f" "gpurun_out/gaps/$(basename $(dirname $f))_gaps.md"
done
