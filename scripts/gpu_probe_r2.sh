#!/bin/bash
# Probe: scratch-disk bandwidth (direct + buffered), host RAM, ResNet-18 and Llama-3-8B benches
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
{
  echo "== df"; df -h /tmp | cat
  echo "== mem"; free -g | cat
  echo "== nproc $(nproc)"
  echo "== dd direct write 4 GiB"; timeout 120 dd if=/dev/zero of=/tmp/ddtest bs=64M count=64 oflag=direct 2>&1 | tail -1
  echo "== dd buffered write+fsync 4 GiB"; timeout 120 dd if=/dev/zero of=/tmp/ddtest2 bs=64M count=64 conv=fsync 2>&1 | tail -1
  echo "== dd direct read"; timeout 120 dd if=/tmp/ddtest of=/dev/null bs=64M iflag=direct 2>&1 | tail -1
  rm -f /tmp/ddtest /tmp/ddtest2
} > gpurun_out/probe.log 2>&1
cat gpurun_out/probe.log
timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/bench_resnet.log 2>&1
rc=$?; echo "RESNET EXIT $rc"; tail -n 1 gpurun_out/bench_resnet.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --model llama3-8b --steps 6 --warmup 2 > gpurun_out/bench_llama.log 2>&1
rc=$?; echo "LLAMA EXIT $rc"; tail -n 1 gpurun_out/bench_llama.log
exit $rc
