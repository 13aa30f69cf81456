#!/bin/bash
# 2 gloo ranks sharing one GPU: step time through the checkpoint phase, then the full multirank rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29591 \
  scripts/diag_postckpt.py > gpurun_out/diag_full.log 2>&1 || { echo "diag failed rc=$?"; exit 1; }
grep "ms/step" gpurun_out/diag_full.log
RTDC_BENCH_VERBOSE=0 bash scripts/gpu.sh multirank
