#!/bin/bash
# PMC counters over the GPT-2-small bench step (kernel trace only; one pass per counter set)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_step -o run \
  --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  -- python3 bench.py --steps 2 --warmup 1 --no-ckpt > gpurun_out/pmc_step.log 2>&1
rc=$?; echo "PMC1 EXIT $rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_step2 -o run \
  --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
  -- python3 bench.py --steps 2 --warmup 1 --no-ckpt > gpurun_out/pmc_step2.log 2>&1
rc=$?; echo "PMC2 EXIT $rc"; [ $rc -eq 0 ] || exit $rc
f1=$(find gpurun_out/pmc_step -name '*counter_collection.csv' | head -1)
f2=$(find gpurun_out/pmc_step2 -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_util.py "$f1" "$f2" > gpurun_out/pmc_step_summary.txt
head -60 gpurun_out/pmc_step_summary.txt
