set -e
export TMPDIR=/tmp
O=gpurun_out/ov; mkdir -p $O
(nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python -c "from ray_torch_distributed_checkpoint_amd.utils.hostinfo import available_cpus as a; print('avail',a())"; df -h /tmp) > $O/host.txt 2>&1 || true
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/sdma.json 2> $O/sdma.err
RTDC_CKPT_D2H=hip timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/hip.json 2> $O/hip.err
RTDC_CKPT_D2H=hip RTDC_CKPT_ARENA=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/hip_noarena.json 2> $O/hip_noarena.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --overlap-steps 15 > $O/sdma15.json 2> $O/sdma15.err
