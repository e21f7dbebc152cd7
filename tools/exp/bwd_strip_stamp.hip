// Phase timestamps of the strip windowed backward (win_bwd_strip) at configs[2]
// geometry: the product source included with FA_STAMP defined.  Phases:
// 0 strip start, 1 + j load j landed (after its wait and barrier), 9..14 the six
// gradient chunks (dV 0/1, dK 0/1, dQ 0/1) stored, 15 end,
// per strip (the kernel is persistent: fa_sid
// is the strip).  Diagnostic only (never shipped);
// build / run: tools/exp/bwd_strip_stamp.py.
#include <hip/hip_runtime.h>
__device__ unsigned long long g_stamp_buf[24 * 16384];
__device__ unsigned long long g_stamp_ws[256];   // the strip counters' workspace (2 KiB)
#define FA_BSTAMP(k)                                                                        \
    do {                                                                                   \
        if (threadIdx.x == 0) {                                                            \
            ::g_stamp_buf[fa_sid * 24 + (k)] = __builtin_amdgcn_s_memtime();            \
            if ((k) == 0) ::g_stamp_buf[fa_sid * 24 + 16] = __builtin_amdgcn_s_memrealtime(); \
            if ((k) == 15) ::g_stamp_buf[fa_sid * 24 + 17] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                                  \
    } while (0)
#include "../../flashattention.jl_amd/csrc/fa_windowed.hip"

extern "C" int bwd_stamp_run(const void* q, const void* k, const void* v, const void* y, const void* dy, float* l,
                             float* m, void* dq, void* dk, void* dv, int B, int mode, unsigned long long* host_out,
                             int nwg_max) {
    fa::WindowedBwdArgs a{};
    a.dtype = FA_DTYPE_BF16; a.q = q; a.k = k; a.v = v; a.y = y; a.dy = dy; a.l = l; a.m = m;
    a.dq = dq; a.dk = dk; a.dv_ = dv;
    a.g.nsp = 2; a.g.S[0] = 128; a.g.S[1] = 128; a.g.S[2] = 1;
    a.g.ws = 7; a.g.stride = 7; a.g.pad = 3;
    a.g.O[0] = 19; a.g.O[1] = 19; a.g.O[2] = 1; a.g.T = 49; a.g.L = 361; a.g.P = 128 * 128;
    a.d = 64; a.dv = 64; a.batch = B; a.scale = 0.125f;
    void* ws = nullptr;
    if (hipGetSymbolAddress(&ws, HIP_SYMBOL(g_stamp_ws)) != hipSuccess) return 4;
    a.workspace = ws; a.workspace_bytes = sizeof(unsigned long long) * 256;
    fa::g_win_force_composed = mode;
    const char* why = nullptr;
    int rc = fa::windowed_bwd_rows<fa::bf16>(a, nullptr, &why);
    fa::g_win_force_composed = 0;
    if (rc != 0) return 1;
    if (!host_out) return 0;
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamp_buf), sizeof(unsigned long long) * 24 * nwg_max) != hipSuccess) return 3;
    return 0;
}
