#!/bin/bash
# Variant builds of xgemm5 (CPU side): build_abl/<name>/librocket_kernels.so with extra -D flags,
# every other kernel object as in the main build.  VARIANTS="name:-DX=1,-DY=2 name2:..."
# Probe one with ROCKET_LIBDIR=build_abl/<name> (scripts/r6/gpu_abl.sh).
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
OBJ=$(python3 -c "import rocket_amd.native.build as b; print(b.OBJDIR)")
for v in $VARIANTS; do
  n=${v%%:*}; f=${v#*:}; f=${f//,/ }
  D=$R/build_abl/$n; mkdir -p $D
  (cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I$R/rocket_amd/native/kernels \
     --offload-arch=gfx950 -munsafe-fp-atomics $f -c $R/rocket_amd/native/kernels/xgemm5.hip -o $D/xgemm5.o)
  objs=$(ls $OBJ/*.hip.o | grep -v xgemm5.hip.o)
  (cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/librocket_kernels.so $objs $D/xgemm5.o)
  cp $R/rocket_amd/_lib/librocket_runtime.so $D/ 2>/dev/null || true
  rm -f $D/xgemm5.o
done
