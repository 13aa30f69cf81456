#!/bin/bash
# hipBLASLt auto-routing of few-row plain products: model tests + Llama / GPT-2 steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py tests/test_gpt2_parity_gpu.py tests/test_optim_overlap_gpu.py tests/test_wgrad_group_gpu.py > gpurun_out/z_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/z_tests.log; exit 1; }
tail -n 1 gpurun_out/z_tests.log
for v in "X=0" "RTDC_FWD_BLASLT=0 RTDC_DGRAD_BLASLT=0"; do
  env $v timeout -k 10 400 python bench.py --model llama3-8b --steps 5 --warmup 2 --no-ckpt > gpurun_out/z_llama.log 2>&1 || { echo "llama bench failed"; tail -5 gpurun_out/z_llama.log; exit 1; }
  echo "llama [$v] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/z_llama.log)"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/z_gpt2.log 2>&1 || { echo "gpt2 bench failed"; exit 1; }
echo "gpt2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/z_gpt2.log)"
