#!/bin/bash
# is the post-engine slowdown gloo's, or any two processes sharing the GPU?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
port=29610
one() { local tag=$1 np=$2; shift 2; port=$((port + 1))
  env "$@" timeout -k 10 200 python -m torch.distributed.run --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port $port scripts/diag_postckpt.py > gpurun_out/diag_$tag.log 2>&1 || { echo "$tag failed rc=$?"; exit 1; }
  echo "== $tag"; grep -E "ms/step" gpurun_out/diag_$tag.log | grep -v warm; }
one nodist1_engine 1 DIAG_NODIST=1 DIAG_N=20 DIAG_MODE=engine
one nodist2_engine 2 DIAG_NODIST=1 DIAG_N=20 DIAG_MODE=engine
one nodist2_plan 2 DIAG_NODIST=1 DIAG_N=20 DIAG_MODE=plan
one nodist2_rawstream 2 DIAG_NODIST=1 DIAG_N=20 DIAG_MODE=rawstream
