set -o pipefail
mkdir -p gpurun_out/ep
AB_ROUNDS=10 timeout -k 10 300 python tools/ab_bwd_libs.py tools/exp/abr6/libfa_e0.so flashattention.jl_amd/libfa_hip.so --shapes 8192,128,64 4096,64,64 4096,128,64 > gpurun_out/ep/ab.log 2>&1 || exit 1
for a in se0 se1; do echo "== $a"; FA_HIP_LIB=tools/exp/abr6/libfa_$a.so timeout -k 10 120 python tools/exp/bwd4_stamp.py 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/ep/stamps.log
