#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) over the attention
# and decode-GEMM micro-benchmarks, plus a kernel-stats pass over the bench.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
  -d gpurun_out/pmc/attn_fetch -o run -- python3 scripts/attn_bench.py --ctx 576,2048 --parts 1024 --iters 3 \
  > gpurun_out/pmc/attn_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d gpurun_out/pmc/prefill_sq -o run -- python3 scripts/prefill_attn_bench.py \
  > gpurun_out/pmc/prefill_sq.log 2>&1 || exit $?
echo pmc-ok
