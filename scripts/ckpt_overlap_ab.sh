# Round-5 GPU session A: grouped persistent GEMM tests, async-save overlap A/B, Llama wgrad A/B.
set -e
export TMPDIR=/tmp
O=gpurun_out/ov; mkdir -p $O
(nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python -c "from ray_torch_distributed_checkpoint_amd.utils.hostinfo import available_cpus as a; print('avail',a())"; df -h /tmp) > $O/host.txt 2>&1 || true
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_group_gpu.py > $O/wgrad_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/sdma.json 2> $O/sdma.err
RTDC_CKPT_D2H=hip timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/hip.json 2> $O/hip.err
RTDC_CKPT_D2H=hip RTDC_CKPT_ARENA=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/hip_noarena.json 2> $O/hip_noarena.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --overlap-steps 15 > $O/sdma15.json 2> $O/sdma15.err
RTDC_G8G_PERSIST=0 timeout -k 10 400 python bench.py --model llama3-8b --steps 6 --warmup 2 --no-ckpt > $O/llama_g8g.json 2> $O/llama_g8g.err
timeout -k 10 400 python bench.py --model llama3-8b --steps 6 --warmup 2 --no-ckpt > $O/llama_g8gp.json 2> $O/llama_g8gp.err
