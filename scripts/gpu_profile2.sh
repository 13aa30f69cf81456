cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-ckpt > gpurun_out/prof2.log 2>&1
echo "PROF EXIT $?" >> gpurun_out/prof2.log
