cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -m gpu > gpurun_out/t2.log 2>&1
echo "TEST EXIT $?" >> gpurun_out/t2.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.log 2>&1
echo "BENCH EXIT $?" >> gpurun_out/bench1.log
