// Phase timestamps of the strip windowed forward (win_strip) at configs[2]
// geometry: the product source included with FA_STAMP defined.  Phases:
// 0 entry, 1 first Q/K chunk landed, 2 QKᵀ done, 3 softmax done + V landed,
// 4 first V chunk's y stored, 5 end.  Diagnostic only (never shipped);
// build / run: tools/exp/strip_stamp.py.
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

extern "C" int strip_stamp_run(const void* q, const void* k, const void* v, void* y, float* l, float* m, int B,
                               int mode, unsigned long long* host_out, int nwg_max, void* ws, size_t ws_bytes) {
    fa::WindowedArgs a{};
    a.dtype = FA_DTYPE_BF16; a.q = q; a.k = k; a.v = v; a.y = y; a.l = l; a.m = m;
    a.g.nsp = 2; a.g.S[0] = 128; a.g.S[1] = 128; a.g.S[2] = 1;
    a.g.ws = 7; a.g.stride = 7; a.g.pad = 3;
    a.g.O[0] = 19; a.g.O[1] = 19; a.g.O[2] = 1; a.g.T = 49; a.g.L = 361; a.g.P = 128 * 128;
    a.d = 64; a.dv = 64; a.batch = B; a.scale = 0.125f;
    a.workspace = ws; a.workspace_bytes = ws_bytes;
    const fa::WinDev g = fa::to_dev(a.g);
    fa::g_win_force_composed = mode;
    hipError_t e = fa::launch_rows1_dd<fa::bf16, 64, 64>(a, g, nullptr);
    fa::g_win_force_composed = 0;
    if (e != hipSuccess) return 1;
    if (!host_out) return 0;
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamp_buf), sizeof(unsigned long long) * 8 * nwg_max) != hipSuccess) return 3;
    return 0;
}
