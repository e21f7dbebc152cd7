// Launch timeline of the dense forward (dense_fwd_tiled): the product source included
// with FA_FWD_STAMP defined.  Per workgroup, wave 0 lane 0 records s_memrealtime
// (100 MHz) at phase k (0 entry, 1 main loop start, 2 main loop end, 3 after the O
// stores) and the CU it runs on (HW_REG_HW_ID, HW_REG_XCC_ID).  Diagnostic only,
// never shipped; the stamps go to a buffer of their own.  Run: tools/exp/fwd_timeline.py.
#include <hip/hip_runtime.h>
__device__ unsigned long long g_tl[8 * 8192];
#define FA_FWD_STAMP(k)                                                                               \
    do {                                                                                              \
        if (threadIdx.x == 0) {                                                                       \
            ::g_tl[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                          \
            if ((k) == 0)                                                                             \
                ::g_tl[blockIdx.x * 8 + 4] =                                                          \
                    ((unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) << 32) | \
                    __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));                      \
        }                                                                                             \
    } while (0)
#include "../../flashattention.jl_amd/csrc/fa_fwd.hip"

extern "C" int fwd_tl_launch(const void* Q, const void* K, const void* V, void* O, float* l, float* m, int N,
                             int d, int batch, void* stream) {
    fa::DenseArgs a{FA_DTYPE_BF16, Q, K, V, O, l, m, N, N, d, d, batch, 1.0f / sqrtf((float)d)};
    const char* why = "";
    return fa::launch_dense_fwd(a, (hipStream_t)stream, &why);
}

extern "C" int fwd_tl_read(unsigned long long* host_out, int nwg) {
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (nwg > 8192) return 4;
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_tl), sizeof(unsigned long long) * 8 * nwg) == hipSuccess ? 0 : 3;
}
