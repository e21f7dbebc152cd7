#!/bin/bash
# Build a copy of libfa_hip.so with extra -D flags on the forward objects (A/B builds):
#   tools/exp/build_fwd_variant.sh OUT.so "-DFOO=1 ..."
set -e
C=/root/repo/flashattention.jl_amd/csrc
B=/tmp/fwdvar_$$
mkdir -p $B
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-gpu-rdc -munsafe-fp-atomics -fno-slp-vectorize -mllvm -amdgpu-sched-strategy=max-ilp -mllvm -amdgpu-use-amdgpu-trackers $2"
/opt/rocm/bin/hipcc $F -x hip -c $C/fa_fwd.hip -o $B/fa_fwd.o &
/opt/rocm/bin/hipcc $F -x hip -c $C/fa_fwd_pers.hip -o $B/fa_fwd_pers.o &
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $1 $C/build/api.cpp.o $B/fa_fwd.o $B/fa_fwd_pers.o $C/build/fa_fwd_p4.hip.o \
    $C/build/fa_bwd.hip.o $C/build/fa_windowed_fwd.o $C/build/fa_windowed_bwd.o $C/build/fa_circulant.hip.o $C/build/fa_softmax.hip.o $C/build/fa_f64.hip.o
rm -rf $B
