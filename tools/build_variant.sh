#!/bin/bash
# Development A/B builds: the product library with one engine compiled with extra defines.
#   bash tools/build_variant.sh <name> -DFOO=1 ...            ->  mujocoposelearning_amd/libhsim_<name>.so (fp64 engine varied)
#   PREC=f32 bash tools/build_variant.sh <name> -DFOO=1 ...   ->  the same with the fp32 engine varied
# (the other engine, PPO/GAE kernels and host code are the product objects; run `make` first)
set -e
cd "$(dirname "$0")/../mujocoposelearning_amd/csrc"
NAME=$1; shift
OBJ=../../build/obj
COMMON="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-hip-fp32-correctly-rounded-divide-sqrt"
if [ "${PREC:-f64}" == "f32" ]; then
  /opt/rocm/bin/hipcc $COMMON -DHS_ONLY_F32 "$@" -c hs_kernels.hip -o $OBJ/hs_kernels_f32_$NAME.o
  K32=$OBJ/hs_kernels_f32_$NAME.o; K64=$OBJ/hs_kernels_f64.o
else
  /opt/rocm/bin/hipcc $COMMON -mllvm -disable-machine-licm -mllvm --amdgpu-sched-strategy=iterative-ilp \
    -DHS_ONLY_F64 "$@" -c hs_kernels.hip -o $OBJ/hs_kernels_f64_$NAME.o
  K32=$OBJ/hs_kernels_f32.o; K64=$OBJ/hs_kernels_f64_$NAME.o
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $K32 $K64 $OBJ/gae.o $OBJ/ppo.o $OBJ/hs_api.o $OBJ/mjcf.o \
  -o ../libhsim_$NAME.so
echo built mujocoposelearning_amd/libhsim_$NAME.so
