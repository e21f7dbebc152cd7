// In-kernel cycle and clock stamps of the dense forward (dense_fwd_tiled): the
// product source included with FA_FWD_STAMP defined (and FA_FWD_ABL from the
// command line for the timing-only ablations).  Diagnostic only, never shipped.
// Build / run: tools/exp/fwd_stamp.py.
//
// Per workgroup, waves 0 and 4 (lane 0) each record s_memtime at phase k
// (0 entry, 1 main loop start, 2 main loop end, 3 after the O stores) and
// s_memrealtime (100 MHz) at phases 0 and 3: slots [16 * wg + 8 * half + k],
// realtime at +6 / +7.  The stamps go to a buffer of their own.
#include <hip/hip_runtime.h>
__device__ unsigned long long g_fstamp[16 * 8192];
#define FA_FWD_STAMP(k)                                                                               \
    do {                                                                                              \
        if ((threadIdx.x & 255) == 0) {                                                               \
            const int slot_ = blockIdx.x * 16 + (threadIdx.x >> 8) * 8;                               \
            ::g_fstamp[slot_ + (k)] = __builtin_amdgcn_s_memtime();                                   \
            if ((k) == 0) ::g_fstamp[slot_ + 6] = __builtin_amdgcn_s_memrealtime();                   \
            if ((k) == 3) ::g_fstamp[slot_ + 7] = __builtin_amdgcn_s_memrealtime();                   \
        }                                                                                             \
    } while (0)
#include "../../flashattention.jl_amd/csrc/fa_fwd.hip"

extern "C" int fwd_stamp_launch(int variant, const void* Q, const void* K, const void* V, void* O, float* l,
                                float* m, int N, int d, int batch, void* stream) {
    fa::DenseArgs a{FA_DTYPE_BF16, Q, K, V, O, l, m, N, N, d, d, batch, 1.0f / sqrtf((float)d)};
    const char* why = "";
    fa::g_fwd_variant = variant;
    const int rc = fa::launch_dense_fwd(a, (hipStream_t)stream, &why);
    fa::g_fwd_variant = 0;
    return rc;
}

extern "C" int fwd_stamp_read(unsigned long long* host_out, int nwg) {
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (nwg > 8192) return 4;
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_fstamp), sizeof(unsigned long long) * 16 * nwg) == hipSuccess ? 0 : 3;
}
