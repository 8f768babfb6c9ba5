#!/bin/bash
# round 4 call 4: PMC passes over the prefill GEMM (pgemm vs hipBLASLt)
set -o pipefail
mkdir -p gpurun_out/r4_4
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d gpurun_out/r4_4/p1 -o p1 -- python3 scripts/pgemm_pmc.py > gpurun_out/r4_4/p1.log 2>&1 || { echo "p1 failed"; tail -20 gpurun_out/r4_4/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/r4_4/p2 -o p2 -- python3 scripts/pgemm_pmc.py > gpurun_out/r4_4/p2.log 2>&1 || { echo "p2 failed"; tail -20 gpurun_out/r4_4/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_4/p3 -o p3 -- python3 scripts/pgemm_pmc.py > gpurun_out/r4_4/p3.log 2>&1 || { echo "p3 failed"; tail -20 gpurun_out/r4_4/p3.log; exit 1; }
ls gpurun_out/r4_4/*
