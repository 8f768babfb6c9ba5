#!/bin/bash
# round 3, call 3: config-5 GPU test, tgemm PMC passes, WS bench trace with gap attribution.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_config5.py tests/test_keda.py -m gpu -v -s --timeout 360 --timeout-method thread 2>&1 | tee $O/cfg45_gpu.log
crc=$?; echo "cfg4/5 gpu rc=$crc"
[ $crc -eq 0 ] || [ $crc -eq 1 ] || exit $crc
timeout -k 10 300 python -u -m pytest tests/test_tgemm_gpu.py -q --timeout 120 --timeout-method thread > $O/tgemm_test.log 2>&1
echo "tgemm test rc=$?"; tail -2 $O/tgemm_test.log
timeout -k 10 400 python -u scripts/prefill_sweep.py --out $O/prefill_sweep.json 2>&1 | tee $O/prefill_sweep.log
echo "prefill sweep rc=$?"
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
cp $(find /tmp/r3bprof -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv
sed -n 1,40p $O/gaps.md
exit $crc
