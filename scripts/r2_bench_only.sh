#!/bin/bash
# default headline bench (WS path) only
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-700
exit $rc
