#!/bin/bash
# tools/build_ab.sh NAME "-DMACRO=V ..." — an A/B variant of librtgpu.so built from this tree with extra
# kernel defines, as raytracing-practice_amd/lib/ab/librtgpu_NAME.so (git-ignored, travels with gpurun),
# for tools/ab_schedule.py --libs NAME=... same-box comparisons.
set -eu
cd "$(dirname "$0")/.."
name=$1
defs=${2:-}
obj=raytracing-practice_amd/build/ab_$name
mkdir -p "$obj" raytracing-practice_amd/lib/ab
HIPFLAGS="-std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wextra -Wno-unused-parameter -Iinclude -Iraytracing-practice_amd/csrc $defs"
/opt/rocm/bin/hipcc $HIPFLAGS -fno-slp-vectorize -c raytracing-practice_amd/csrc/rtg_kernels.hip -o "$obj/rtg_kernels.o"
for f in rtg_api rtg_bvh rtg_comm; do
  /opt/rocm/bin/hipcc $HIPFLAGS -x hip -c raytracing-practice_amd/csrc/$f.cpp -o "$obj/$f.o"
done
/opt/rocm/bin/hipcc $HIPFLAGS -c raytracing-practice_amd/csrc/rtg_gpubvh.hip -o "$obj/rtg_gpubvh.o"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC "$obj"/*.o -o raytracing-practice_amd/lib/ab/librtgpu_$name.so \
  -Wl,-soname,librtgpu_$name.so -lrccl
echo "built raytracing-practice_amd/lib/ab/librtgpu_$name.so"
