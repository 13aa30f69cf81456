#!/bin/bash
# Timing-only diagnostic builds of the 8-wave GEMM (RTDC_G8_DIAG bits: 1 = no main-loop vmcnt
# waits, 2 = LDS fragments read only in the first K-tile, 4 = no loop barriers; results WRONG,
# never shipped): ab/_C_diag<N>.so for RTDC_EXT_SO A/B runs.
set -e
cd /root/repo/ray_torch_distributed_checkpoint_amd
B=build
OBJS=$(ls $B/*.o | grep -v gemm_8ph)
TDIR=$(python -c "import torch,os; print(os.path.dirname(torch.__file__))")
for N in "$@"; do
  (/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DRTDC_G8_DIAG=$N -I csrc -c csrc/kernels/gemm_8ph.hip -o /tmp/g8_diag$N.o && \
   /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS /tmp/g8_diag$N.o -o ../ab/_C_diag$N.so -L $TDIR/lib -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -lz -Wl,-rpath,$TDIR/lib && echo built $N) &
done
wait
