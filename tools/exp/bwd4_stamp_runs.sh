set -o pipefail
mkdir -p gpurun_out/w4
for a in stamp st1 st2 st4 st7; do
  echo "== $a"
  FA_HIP_LIB=tools/exp/abr6/libfa_$a.so timeout -k 10 120 python tools/exp/bwd4_stamp.py 2>&1 | grep -v amdgpu.ids | sed -n '/waves=4/,$p' || exit 1
done
set -o pipefail
for a in g1q3 g2q3 g4q3 g2q1; do
  echo "== $a"
  FA_HIP_LIB=tools/exp/abr6/libfa_$a.so timeout -k 10 120 python tools/exp/bwd4_stamp.py 2>&1 | grep -v amdgpu.ids | sed -n '/waves=4/,$p' || exit 1
done
