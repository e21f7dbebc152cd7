#!/bin/bash
# Build a copy of libfa_hip.so whose fa_bwd.hip is edited by python scripts (A/B ablations):
#   tools/exp/build_bwd_edit.sh OUT.so "flags" edit1.py [edit2.py ...]
set -e
C=/root/repo/flashattention.jl_amd/csrc
B=/tmp/bwded_$$
mkdir -p $B
out=$1; flags=$2; shift 2
cp $C/fa_bwd.hip $B/fa_bwd.hip
sed -i "s#\"fa_common.h\"#\"$C/fa_common.h\"#; s#\"fa_internal.h\"#\"$C/fa_internal.h\"#; s#\"../../include/fa_hip.h\"#\"/root/repo/include/fa_hip.h\"#" $B/fa_bwd.hip
for e in "$@"; do python3 $e $B/fa_bwd.hip; done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-gpu-rdc -munsafe-fp-atomics $flags -x hip -c $B/fa_bwd.hip -o $B/fa_bwd.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out $C/build/api.cpp.o $C/build/fa_fwd.hip.o $C/build/fa_fwd_p4.hip.o \
    $B/fa_bwd.o $C/build/fa_windowed_fwd.o $C/build/fa_windowed_bwd.o $C/build/fa_circulant.hip.o $C/build/fa_softmax.hip.o $C/build/fa_f64.hip.o
rm -rf $B
