#!/bin/bash
# round 3, call 2: TP-on-one-GPU test (TP=8 memory fix), tgemm PMC passes, WS bench
# trace with mid-size gap attribution.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tp_gpu.py -v -s --timeout 420 --timeout-method thread > $O/tp_gpu.log 2>&1
trc=$?; echo "tp gpu rc=$trc"; grep -E "^TP=|passed|failed" $O/tp_gpu.log | tail -5
[ $trc -eq 0 ] || grep -A12 "Error" $O/tp_gpu.log | head -40
[ $trc -eq 0 ] || [ $trc -eq 1 ] || exit $trc
timeout -k 10 400 python -u -m pytest tests/test_config5.py -m gpu -v -s --timeout 360 --timeout-method thread > $O/cfg5_gpu.log 2>&1
crc=$?; echo "cfg5 gpu rc=$crc"; tail -3 $O/cfg5_gpu.log
[ $crc -eq 0 ] || [ $crc -eq 1 ] || exit $crc
for cfg in "gate_up 256 128 1 0" "qkv 256 128 4 0" "down 256 128 8 0"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d /tmp/pmc_$tag -o a -- python3 scripts/tgemm_pmc.py $cfg > $O/pmc_a_$tag.log 2>&1
  echo "pmc A $tag rc=$?"
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d /tmp/pmc_$tag -o b -- python3 scripts/tgemm_pmc.py $cfg > $O/pmc_b_$tag.log 2>&1
  echo "pmc B $tag rc=$?"
  for f in $(find /tmp/pmc_$tag -name '*counter_collection.csv'); do cp $f $O/$(basename $(dirname $f))_${tag}_$(basename $f); done
done
ls $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r3bprof -o run -- python3 bench.py --steps 2 --warmup 1 > $O/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 $O/prof_bench.log | cut -c1-300
TR=$(find /tmp/r3bprof -name '*kernel_trace.csv' | head -1)
python3 scripts/gap_analysis.py $TR $O/gaps.md > /dev/null
gzip -c $TR > $O/kernel_trace.csv.gz
sed -n 1,40p $O/gaps.md
exit $trc
