#!/bin/bash
# A/B builds of the extension with extra -D flags on the kernel files that include gemm_8ph.h:
#   bash scripts/build_variant.sh <name> "-DFOO=1 -DBAR=2"   ->  abv/_C_<name>.so  (RTDC_EXT_SO=...)
# The other objects come from the in-tree build (run _build first).
set -e
cd /root/repo/ray_torch_distributed_checkpoint_amd
NAME=$1; DEFS=$2
mkdir -p ../abv /tmp/variant_$NAME
TDIR=$(python -c "import torch,os; print(os.path.dirname(torch.__file__))")
VAR=${VAR:-"gemm_8ph gemm_bf16 gemm4b gemm8b"}  # VAR="attn_flash" etc. to vary other kernel files
OBJS=""
for o in build/*.o; do
  b=$(basename $o .hip.o); skip=0
  for v in $VAR; do [ "$b" = "$v" ] && skip=1; done
  [ $skip = 0 ] && OBJS="$OBJS $o"
done
for v in $VAR; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $DEFS -I csrc -c csrc/kernels/$v.hip -o /tmp/variant_$NAME/$v.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS /tmp/variant_$NAME/*.o -o ../abv/_C_$NAME.so \
  -L $TDIR/lib -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -lhsa-runtime64 -lz -Wl,-rpath,$TDIR/lib
echo built abv/_C_$NAME.so
