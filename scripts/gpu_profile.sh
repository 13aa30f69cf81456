# Stock-torch baseline + rocprofv3 kernel stats of bench.py (GPU box)
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python benchmarks/torch_reference_gpt2.py --steps 10 --warmup 3 > gpurun_out/torchref.log 2>&1
echo "TORCHREF EXIT $?" >> gpurun_out/torchref.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python3 bench.py --steps 5 --warmup 2 --no-ckpt > gpurun_out/prof1.log 2>&1
echo "PROF EXIT $?" >> gpurun_out/prof1.log
