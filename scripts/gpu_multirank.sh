cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 4 --backend gloo > gpurun_out/mr1.log 2>&1
echo "MR EXIT $?" >> gpurun_out/mr1.log
