// fa_fwd_params.h — launch parameters of the dense forward kernels
// (fa_fwd.hip: generic / tiled / split-KV kernels).
#pragma once

#include <hip/hip_runtime.h>

namespace fa {

struct FwdParams {
    const void* Q;
    const void* K;
    const void* V;
    void* O;
    float* l;
    float* m;
    int N, Nk, d, dv;
    int ldk;   // K / V row stride in elements (= Nk, or Nk rounded up to 8 in padded workspace copies)
    int nqb, total_wg;
    // split-KV (small grids): nsplit key ranges of tps tiles each; partial results
    // (fp32, unnormalised, relative to the split's max) go to opart / lpart / mpart,
    // indexed by (split * batch + b)
    int nsplit, tps, batch;
    float *opart, *lpart, *mpart;
    float scale, scale_log2;
    float rescale_log2;   // lazy-rescale threshold (log2 units): kRescaleLog2, or the debug knob
    int fast;  // K/V rows 16-B aligned and Nk a multiple of the chunk width
    int wide = 0;     // N % 8 == 0, Q and O 16-B aligned: Q / O staged through LDS (16-B accesses)
};

}  // namespace fa
