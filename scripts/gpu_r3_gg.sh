#!/bin/bash
# Round-3 pass GG: the N-rank bench paths with this build (deferred column sums, flash partials,
# stem gather backward): the 2-rank gloo-on-one-GPU rehearsal (plain, ResNet, ZeRO-1 + bf16, P2P)
# and the RCCL path as a 1-rank nccl group with forced collectives.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_multirank.sh || exit $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29581 bench.py --gpus 1 --steps 10 --warmup 3 --force-dist > gpurun_out/gg_rccl_gpt2.log 2>&1
rc=$?; echo "RCCL GPT2 EXIT $rc"; tail -n 1 gpurun_out/gg_rccl_gpt2.log | grep -o '"ms_per_step": [0-9.]*\|"ranks_in_sync": [a-z]*\|"ms_per_step_during_async_save": [0-9.]*' | tr '\n' ' '; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29582 bench.py --gpus 1 --steps 10 --warmup 3 --force-dist --model resnet18 > gpurun_out/gg_rccl_resnet.log 2>&1
rc=$?; echo "RCCL RESNET EXIT $rc"; tail -n 1 gpurun_out/gg_rccl_resnet.log | grep -o '"ms_per_step": [0-9.]*\|"ranks_in_sync": [a-z]*' | tr '\n' ' '; echo
exit $rc
