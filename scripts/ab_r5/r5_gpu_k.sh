#!/bin/bash
# flash forward: software-pipelined variant (RTDC_FA_FWD=3) vs the shipped one, then the rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pipelined or lazy_rescale or deterministic" > gpurun_out/k_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/k_tests.log; exit 1; }
tail -n 1 gpurun_out/k_tests.log
for r in 1 2 3; do for v in 1 3; do
  RTDC_FA_FWD=$v timeout -k 10 120 python benchmarks/attn_bench.py --only gpt2 --reps 30 > gpurun_out/attn_v.log 2>&1 || { echo "attn $v failed"; exit 1; }
  echo "FWD=$v $(grep kernel_fwd gpurun_out/attn_v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel_fwd_us"], d["kernel_fwd_TF"])')"
done; done
bash scripts/gpu.sh multirank
