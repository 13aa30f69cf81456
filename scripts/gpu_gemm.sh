cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/t3.log 2>&1
echo "TEST EXIT $?" >> gpurun_out/t3.log
timeout -k 10 300 python benchmarks/gemm_bench.py --reps 10 --sweep > gpurun_out/gemm2.log 2>&1
echo "GEMM EXIT $?" >> gpurun_out/gemm2.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-ckpt > gpurun_out/bench3.log 2>&1
echo "BENCH EXIT $?" >> gpurun_out/bench3.log
