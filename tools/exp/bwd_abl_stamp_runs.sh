set -o pipefail
mkdir -p gpurun_out/abl
for m in 0 4 5 7 8 10; do
  echo "== mode $m"
  FA_BWD_MODE=$m FA_HIP_LIB=tools/exp/abr6/libfa_sabl.so timeout -k 10 120 python tools/exp/bwd4_stamp.py 2>&1 | grep -v amdgpu.ids || exit 1
done
