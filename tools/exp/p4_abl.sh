#!/bin/bash
# Build the timing-only ablation variants of the p4 forward (tools/exp/p4_lab.hip with
# FA_P4_ABL) as libp4_lab_a<N>.so.  Usage: bash tools/exp/p4_abl.sh 0 1 2 4 8
cd "$(dirname "$0")"
for a in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -fno-gpu-rdc -fno-slp-vectorize \
    -DFA_P4_ABL=$a -DP4_NO_STAMP -o libp4_lab_a$a.so p4_lab.hip &
done
wait
