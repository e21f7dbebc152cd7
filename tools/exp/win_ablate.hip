// Timing-only ablations of the two-window row-shift forward (win_rows1s) at
// configs[2] geometry: includes the product source with FA_WIN_ABL set (see
// fa_windowed.hip).  Build/run: tools/exp/win_ablate.py.  Never shipped.
#include <hip/hip_runtime.h>
#include "../../flashattention.jl_amd/csrc/fa_windowed.hip"

extern "C" __attribute__((visibility("default"))) int abl_run(const void* q, const void* k, const void* v, void* y, float* l, float* m, int B) {
    fa::WindowedArgs a{};
    a.dtype = FA_DTYPE_BF16; a.q = q; a.k = k; a.v = v; a.y = y; a.l = l; a.m = m;
    a.g.nsp = 2; a.g.S[0] = 128; a.g.S[1] = 128; a.g.S[2] = 1;
    a.g.ws = 7; a.g.stride = 7; a.g.pad = 3;
    a.g.O[0] = 19; a.g.O[1] = 19; a.g.O[2] = 1; a.g.T = 49; a.g.L = 361; a.g.P = 128 * 128;
    a.d = 64; a.dv = 64; a.batch = B; a.scale = 0.125f;
    const fa::WinDev g = fa::to_dev(a.g);
#ifdef WV_MODE
    fa::g_win_force_composed = WV_MODE;   // forced kernel variant (fa_debug_set_win_composed)
#endif
    return fa::launch_rows1_dd<fa::bf16, 64, 64>(a, g, nullptr) == hipSuccess ? 0 : 1;
}
