#!/bin/bash
# Build diagnostic variants of the p4 forward (tools/exp/p4_lab.hip) as libp4_lab_<tag>.so.
# Each argument is TAG=FLAGS, e.g.  a0="-DFA_P4_ABL=0"  pf2="-DFA_P4_PF=2"
# (FA_P4_ABL timing-only ablation bits: see fa_fwd_p4.hip).
cd "$(dirname "$0")"
for arg in "$@"; do
  tag="${arg%%=*}"; flags="${arg#*=}"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -fno-gpu-rdc -fno-slp-vectorize \
    -DP4_NO_STAMP $flags -o libp4_lab_$tag.so p4_lab.hip &
done
wait
