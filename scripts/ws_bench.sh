#!/bin/bash
# WebSocket-path headline bench at several stream-coalescing windows + the
# in-process runtime path for comparison.  Stops at the first failure.
mkdir -p gpurun_out
for iv in ${INTERVALS:-0 20}; do
  timeout -k 10 400 python -u bench.py --steps ${STEPS:-3} --warmup 1 --stream-interval-ms $iv > gpurun_out/ws_iv$iv.log 2>&1
  rc=$?; echo "ws interval=$iv rc=$rc"; tail -1 gpurun_out/ws_iv$iv.log
  [ $rc -eq 0 ] || exit $rc
done
if [ -n "$COMPARE" ]; then
  timeout -k 10 400 python -u bench.py --steps ${STEPS:-3} --warmup 1 --path runtime > gpurun_out/rt.log 2>&1
  rc=$?; echo "runtime rc=$rc"; tail -1 gpurun_out/rt.log
fi
exit $rc
