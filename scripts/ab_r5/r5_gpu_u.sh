#!/bin/bash
# norm backward: waves (RTDC_NORM_BWD_WAVES) at the GPT-2 LayerNorm and Llama RMSNorm shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for nw in 4096 2048 1024 512 256; do
  RTDC_NORM_BWD_WAVES=$nw timeout -k 10 120 python benchmarks/norm_bench.py > gpurun_out/u_norm_${nw}_$r.log 2>&1 || { echo "norm_bench failed"; tail -5 gpurun_out/u_norm_${nw}_$r.log; exit 1; }
  echo "waves=$nw $r $(grep '"bwd"' gpurun_out/u_norm_${nw}_$r.log | tr '\n' ' ')"
done; done
