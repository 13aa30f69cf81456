#!/bin/bash
# Round-3 pass U: greedy round packing of the grouped weight gradients (252-tile groups + split-K
# remainder) - group tests, GPT-2 bench x2, RCCL 1-rank rehearsal of the GPT-2 bench path with
# grouping + side stream, GPT-2 kernel trace.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_wgrad_group_gpu.py tests/test_optim_overlap_gpu.py tests/test_gpt2_parity_gpu.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/wgrad_pack_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 4 gpurun_out/wgrad_pack_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-ckpt > gpurun_out/gpt2_pack_r$r.log 2>&1
  rc=$?; echo "GPT2 PACK r$r EXIT $rc $(tail -n 1 gpurun_out/gpt2_pack_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
  [ $rc -eq 0 ] || exit $rc
  RTDC_WGRAD_GROUP=0 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-ckpt > gpurun_out/gpt2_nogroup_r$r.log 2>&1
  rc=$?; echo "GPT2 NOGROUP r$r EXIT $rc $(tail -n 1 gpurun_out/gpt2_nogroup_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29581 bench.py --gpus 1 --steps 10 --warmup 3 --force-dist > gpurun_out/rccl_bench_gpt2_group.log 2>&1
rc=$?; echo "RCCL BENCH EXIT $rc"; tail -n 1 gpurun_out/rccl_bench_gpt2_group.log | grep -o '"ms_per_step": [0-9.]*\|"ranks_in_sync": [a-z]*\|"ms_per_step_during_async_save": [0-9.]*' | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_prof_gpt2.sh > /dev/null 2>&1; echo "PROF EXIT $?"; head -12 gpurun_out/prof_gpt2_summary.txt
