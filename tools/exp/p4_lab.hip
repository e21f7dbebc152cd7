// Diagnostic build of the one-wave-per-SIMD forward (fa_fwd_p4.hip): phase stamps.
// Never shipped.  Build / run: tools/exp/p4_lab.py.
//
// FA_P4_STAMP(pt, j): lane 0 of every wave records s_memtime at phase boundaries of
// tiles 16..19 of the workgroup's first block (pt 2..6) and at block points (pt 0, 1,
// 7, 8) of its first two blocks; s_memrealtime at kernel start and end for the clock.
#include <hip/hip_runtime.h>
__device__ unsigned long long g_p4st[256 * 4 * 64];
#ifndef P4_NO_STAMP
#define FA_P4_STAMP(pt, j)                                                                            \
    do {                                                                                              \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        unsigned long long t_;                                                                        \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                     \
        __builtin_amdgcn_sched_barrier(0);                                                            \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 256) {                                            \
            const int base_ = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;                             \
            if ((j) < 0 && p4_blk < 2) ::g_p4st[base_ + 40 + p4_blk * 8 + (pt)] = t_;                 \
            if ((j) >= 16 && (j) < 20 && p4_blk == 0) ::g_p4st[base_ + ((j) - 16) * 8 + (pt)] = t_;  \
            if ((pt) == 0) ::g_p4st[base_ + 60] = __builtin_amdgcn_s_memrealtime();                   \
            if ((pt) == 8) ::g_p4st[base_ + 61] = __builtin_amdgcn_s_memrealtime();                   \
            if ((pt) == 8) ::g_p4st[base_ + 62] = t_;                                                 \
        }                                                                                             \
    } while (0)
#endif
#ifdef P4_SLOTS
// s_memtime every 4th MFMA slot of the X/Y stream (8 samples per tile at d = 64, 16 at
// 128), recorded for tile 16 of each workgroup's first block; the wait for the samples
// is deferred to the end of the stream (no lgkmcnt wait inside it)
__device__ unsigned long long g_p4slot[256 * 4 * 16];
#define FA_P4_SLOT_DECL unsigned long long p4ts[16] = {};
#define FA_P4_SLOT(i)                                                                          \
    if constexpr ((i) % 4 == 0 && (i) / 4 < 16) asm volatile("s_memtime %0" : "=s"(p4ts[(i) / 4])::"memory");
#define FA_P4_SLOT_FLUSH(j)                                                                    \
    do {                                                                                       \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                     \
        if ((j) == 16 && p4_blk == 0 && (threadIdx.x & 63) == 0 && blockIdx.x < 256)          \
            for (int q_ = 0; q_ < 16; ++q_)                                                    \
                ::g_p4slot[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 + q_] = p4ts[q_];         \
    } while (0)
#endif
#include "../../flashattention.jl_amd/csrc/fa_fwd_p4.hip"

extern "C" int p4_launch(int dtype, const void* Q, const void* K, const void* V, void* O, float* l, float* m, int N,
                         int d, int batch, void* stream) {
    fa::FwdParams p{};
    p.Q = Q; p.K = K; p.V = V; p.O = O; p.l = l; p.m = m;
    p.N = N; p.Nk = N; p.d = d; p.dv = d; p.ldk = N;
    p.batch = batch;
    p.scale = 1.0f / sqrtf((float)d);
    p.scale_log2 = p.scale * fa::kLog2e;
    p.rescale_log2 = fa::kRescaleLog2;
    p.fast = 1; p.wide = 1; p.nsplit = 1;
    p.nqb = (N + 255) / 256;
    p.total_wg = p.nqb * batch;
    hipError_t e = hipSuccess;
    if (!fa::launch_dense_fwd_p4(p, d, d, dtype, (hipStream_t)stream, &e)) return 5;
    return e == hipSuccess ? 0 : 6;
}
#ifdef P4_SLOTS
extern "C" int p4_read_slots(unsigned long long* host_out) {
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_p4slot), sizeof(g_p4slot)) == hipSuccess ? 0 : 3;
}
#endif
extern "C" int p4_read(unsigned long long* host_out) {
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_p4st), sizeof(g_p4st)) == hipSuccess ? 0 : 3;
}
