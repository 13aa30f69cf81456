#!/bin/bash
# Round-3 pass L: RCCL rehearsal on one GPU - the forced-collectives DDP test (1-rank nccl group),
# then bench.py's whole multi-GPU path (--force-dist: RCCL preflight, DDP native engine with an
# RCCL all-reduce per bucket, in-sync check, bucket sweep, sharded checkpoint) under torchrun.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -x -v -m gpu -k "forced or gloo_two" --timeout 240 --timeout-method thread > gpurun_out/rccl_test.log 2>&1
rc=$?; echo "TEST EXIT $rc"; tail -n 8 gpurun_out/rccl_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29571 bench.py --gpus 1 --steps 10 --warmup 3 --force-dist > gpurun_out/rccl_bench_gpt2.log 2>&1
rc=$?; echo "BENCH GPT2 EXIT $rc"; tail -n 1 gpurun_out/rccl_bench_gpt2.log | cut -c1-3000
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29572 bench.py --gpus 1 --steps 10 --warmup 3 --force-dist --grad-comm-dtype bf16 --model resnet18 > gpurun_out/rccl_bench_resnet.log 2>&1
rc=$?; echo "BENCH RESNET EXIT $rc"; tail -n 1 gpurun_out/rccl_bench_resnet.log | cut -c1-3000
exit $rc
