# variants a..f: copies of csrc/fa_windowed.hip (HEAD / edited) generated per experiment, not tracked
# variants a (HEAD), b (decode once, no loop), c (persistent, launch bounds 6) x ablations 0, 3
set -e
cd "$(dirname "$0")"
B=../../../flashattention.jl_amd/csrc/build
for vv in ${VARS:-a b c}; do for abl in 0 3; do
  v=${vv%%:*}; mode=${vv#*:}; [ "$mode" = "$vv" ] && mode=0; tag=$v; [ "$mode" != 0 ] && tag=$v$mode
  sed "s#../../flashattention.jl_amd/csrc/fa_windowed.hip#wv/$v.hip#" ../win_ablate.hip > /tmp/wab_$v.hip
  cp /tmp/wab_$v.hip ../wab_$v.hip
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -fno-gpu-rdc -Wl,--version-script=$(pwd)/exports.map -DFA_WIN_ABL=$abl -DWV_MODE=$mode -o lib_${tag}_$abl.so -x hip ../wab_$v.hip -x none $B/fa_fwd.hip.o $B/fa_bwd.hip.o &
done; done; wait
rm -f ../wab_?.hip
