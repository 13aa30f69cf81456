#!/bin/bash
# ResNet-18 stem pool+BN backward statistics blocks (RTDC_POOL_BN_BLOCKS), alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for nb in 1024 2048 4096 512; do
  RTDC_POOL_BN_BLOCKS=$nb timeout -k 10 240 python bench.py --model resnet18 --steps 20 --warmup 5 --no-ckpt > gpurun_out/t_bench_${nb}_$r.log 2>&1 || { echo "bench failed"; exit 1; }
  echo "blocks=$nb $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/t_bench_${nb}_$r.log)"
done; done
