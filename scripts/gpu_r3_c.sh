#!/bin/bash
# Round 3 GPU pass C: full GPU suite, product path (GPT-2 through train_flow + exact resume),
# Llama-3-8B full train-state 1/8 shard (simulated rank 0 of 8) save + cold restore, and
# Llama-3-8B under the trainer with one async checkpoint (the same simulated shard).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/r3c_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 3 gpurun_out/r3c_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_product_r3.sh || exit $?
timeout -k 10 400 python -u bench.py --model llama3-8b --steps 5 --warmup 2 --overlap-steps 3 \
  --simulate-world 8 --simulate-rank 0 > gpurun_out/r3c_llama_shard.log 2>&1
rc=$?; echo "LLAMA SHARD EXIT $rc"; tail -n 1 gpurun_out/r3c_llama_shard.log
[ $rc -eq 0 ] || exit $rc
RTDC_HOME=/tmp/rtdc_home_llama RTDC_DCP_SIMULATE=8:0 timeout -k 10 400 python -u train_flow.py run \
  --model llama3-8b --steps 12 --ckpt_every_n_steps 10 --num_workers 1 > gpurun_out/r3c_llama_trainer.log 2>&1
rc=$?; echo "LLAMA TRAINER EXIT $rc"; grep -E "report|committed" gpurun_out/r3c_llama_trainer.log | tail -n 4
for f in $(find /tmp/rtdc_home_llama -name result.json); do cp $f gpurun_out/r3c_llama_trainer_result.json; done
exit $rc
