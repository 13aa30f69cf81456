#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench path on one GPU: both ranks share cuda:0 and talk
# gloo (RCCL refuses two ranks on one device); exercises DDP (native bucket engine), buffer
# broadcast (ResNet BatchNorm), sharded DCP save dedup + restore.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 4 --backend gloo > gpurun_out/mr_gpt2.log 2>&1
rc=$?; echo "MR GPT2 EXIT $rc"; tail -n 2 gpurun_out/mr_gpt2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29534 bench.py --gpus 2 --steps 3 --warmup 1 --model resnet18 --batch 32 --backend gloo \
  > gpurun_out/mr_resnet.log 2>&1
rc=$?; echo "MR RESNET EXIT $rc"; tail -n 2 gpurun_out/mr_resnet.log
[ $rc -eq 0 ] || exit $rc
# the opt-in communication modes on the same 2-rank path: bf16 gradients, ZeRO-1, P2P buckets
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29535 bench.py --gpus 2 --steps 3 --warmup 1 --batch 4 --backend gloo --zero 1 \
  --grad-comm-dtype bf16 > gpurun_out/mr_gpt2_zero.log 2>&1
rc=$?; echo "MR GPT2 ZERO EXIT $rc"; tail -n 2 gpurun_out/mr_gpt2_zero.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29536 bench.py --gpus 2 --steps 3 --warmup 1 --batch 4 --backend gloo --p2p-kb 4096 --no-ckpt \
  > gpurun_out/mr_gpt2_p2p.log 2>&1
rc=$?; echo "MR GPT2 P2P EXIT $rc"; tail -n 2 gpurun_out/mr_gpt2_p2p.log
exit $rc
