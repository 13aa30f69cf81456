cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -m gpu > gpurun_out/t4.log 2>&1
echo "TEST EXIT $?" >> gpurun_out/t4.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench4.log 2>&1
echo "BENCH EXIT $?" >> gpurun_out/bench4.log
