// Phase timestamps of the one-window-per-workgroup windowed kernel (win_rows1)
// at configs[2] geometry: includes the product source with FA_STAMP defined.
// Build: see tools/exp/win_stamp.py.  Diagnostic only (never shipped).
#include <hip/hip_runtime.h>
__device__ unsigned long long g_stamp_buf[8 * 16384];
#define FA_STAMP(k)                                                                        \
    do {                                                                                   \
        if (threadIdx.x == 0) {                                                            \
            ::g_stamp_buf[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memtime();            \
            if ((k) == 0) ::g_stamp_buf[blockIdx.x * 8 + 6] = __builtin_amdgcn_s_memrealtime(); \
            if ((k) == 5) ::g_stamp_buf[blockIdx.x * 8 + 7] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                                  \
    } while (0)
#include "../../flashattention.jl_amd/csrc/fa_windowed.hip"

extern "C" int stamp_run(const void* q, const void* k, const void* v, void* y, float* l, float* m, int B,
                         unsigned long long* host_out) {
    fa::WindowedArgs a{};
    a.dtype = FA_DTYPE_BF16; a.q = q; a.k = k; a.v = v; a.y = y; a.l = l; a.m = m;
    a.g.nsp = 2; a.g.S[0] = 128; a.g.S[1] = 128; a.g.S[2] = 1;
    a.g.ws = 7; a.g.stride = 7; a.g.pad = 3;
    a.g.O[0] = 19; a.g.O[1] = 19; a.g.O[2] = 1; a.g.T = 49; a.g.L = 361; a.g.P = 128 * 128;
    a.d = 64; a.dv = 64; a.batch = B; a.scale = 0.125f;
    const fa::WinDev g = fa::to_dev(a.g);
    hipError_t e = fa::launch_rows1_dd<fa::bf16, 64, 64>(a, g, nullptr);
    if (e != hipSuccess) return 1;
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamp_buf), sizeof(unsigned long long) * 8 * 361 * B) != hipSuccess) return 3;
    return 0;
}

// the fused windowed backward (win_bwd_rows) at the same geometry; phases:
// 0 start, 1 q/k staged, 2 v/dy staged + D sums, 3 phase 1 (P, dS) done, 4 stores issued
extern "C" int stamp_run_bwd(const void* q, const void* k, const void* v, const void* y, const void* dy,
                             const float* l, const float* m, void* dq, void* dk, void* dv, int B,
                             unsigned long long* host_out) {
    fa::WindowedBwdArgs a{};
    a.dtype = FA_DTYPE_BF16; a.q = q; a.k = k; a.v = v; a.y = y; a.dy = dy; a.l = l; a.m = m;
    a.dq = dq; a.dk = dk; a.dv_ = dv;
    a.g.nsp = 2; a.g.S[0] = 128; a.g.S[1] = 128; a.g.S[2] = 1;
    a.g.ws = 7; a.g.stride = 7; a.g.pad = 3;
    a.g.O[0] = 19; a.g.O[1] = 19; a.g.O[2] = 1; a.g.T = 49; a.g.L = 361; a.g.P = 128 * 128;
    a.d = 64; a.dv = 64; a.batch = B; a.scale = 0.125f;
    const char* why = nullptr;
    if (fa::windowed_bwd_rows<fa::bf16>(a, nullptr, &why) != 0) return 1;
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamp_buf), sizeof(unsigned long long) * 8 * 361 * B) != hipSuccess) return 3;
    return 0;
}
