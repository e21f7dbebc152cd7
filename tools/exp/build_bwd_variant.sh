#!/bin/bash
# Build a copy of libfa_hip.so with extra flags on fa_bwd.hip (A/B builds):
#   tools/exp/build_bwd_variant.sh OUT.so "-mllvm ... -DFOO=1"
set -e
[ -n "$1" ] || { echo "usage: $0 OUT.so \"flags\"" >&2; exit 2; }
C=/root/repo/flashattention.jl_amd/csrc
B=/tmp/bwdvar_$$
mkdir -p $B
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-gpu-rdc -munsafe-fp-atomics $2 -x hip -c $C/fa_bwd.hip -o $B/fa_bwd.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $1 $C/build/api.cpp.o $C/build/fa_fwd.hip.o $C/build/fa_fwd_p4.hip.o \
    $B/fa_bwd.o $C/build/fa_windowed_fwd.o $C/build/fa_windowed_bwd.o $C/build/fa_circulant.hip.o $C/build/fa_softmax.hip.o $C/build/fa_f64.hip.o
rm -rf $B
