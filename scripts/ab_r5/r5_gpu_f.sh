# Round-5 GPU session F: 8 ranks writing / restoring their Llama-3-8B ZeRO-1 shards at once (one GPU, gloo).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/f
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29641 benchmarks/ckpt_multiwriter.py > gpurun_out/f/multiwriter.log 2>&1
grep '^{' gpurun_out/f/multiwriter.log
