#!/bin/bash
# New GPU tests (DDP engine on GPU, workload trainer restart), headline bench, and the
# 2-rank gloo-on-one-GPU rehearsal of the multi-rank bench path with bf16 gradient comm.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py tests/test_optim.py -x -v -m gpu --timeout 200 --timeout-method thread \
  > gpurun_out/tests_new.log 2>&1
rc=$?; echo "NEW TESTS EXIT $rc"; tail -n 12 gpurun_out/tests_new.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "BENCH EXIT $rc"; tail -n 1 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --batch 4 --backend gloo --grad-comm-dtype bf16 --no-ckpt > gpurun_out/bench_gloo2_bf16.log 2>&1
rc=$?; echo "GLOO2 EXIT $rc"; tail -n 1 gpurun_out/bench_gloo2_bf16.log
exit $rc
