// Ablation build of the v2 forward (tools/exp only; not part of the product).
#include <type_traits>
#include "../../flashattention.jl_amd/csrc/fa_common.h"
namespace fa {

int g_fwd_variant = 2;  // 1: v2 fast, 2: pipelined, 3: pipelined + prescale (debug knob)

struct FwdParams {
    const void* Q;
    const void* K;
    const void* V;
    void* O;
    float* l;
    float* m;
    int N, Nk, d, dv;
    int nqb, total_wg;
    float scale, scale_log2;
    int fast;  // K/V rows 16-B aligned and Nk a multiple of the chunk width
};

constexpr int kBM = 128;  // query rows per workgroup (4 waves x 32)
constexpr int kBN = 64;   // keys per tile
constexpr int kThreads = 256;

// One 16-byte chunk (16/sizeof(T) elements) of row `row`, columns
// [col0, col0+EPC) of a row-major [nrows][ncols] slab; zero out of range.
template <class T>
__device__ __forceinline__ u32x4 load_chunk(const T* base, int row, int col0, int nrows,
                                            int ncols, bool fast) {
    constexpr int EPC = 16 / sizeof(T);
    u32x4 z = {0u, 0u, 0u, 0u};
    if (row >= nrows) return z;
    const T* src = base + (int64_t)row * ncols;
    if (fast) {
        if (col0 >= ncols) return z;
        return *(const u32x4*)(src + col0);
    }
    union {
        T e[EPC];
        u32x4 v;
    } u;
#pragma unroll
    for (int e = 0; e < EPC; ++e) u.e[e] = (col0 + e < ncols) ? src[col0 + e] : (T)0.0f;
    return u.v;
}

constexpr float kRescaleLog2 = 8.0f;
#ifndef FA_SCHED_GROUPS
#define FA_SCHED_GROUPS 1
#endif
#ifndef FA_VALU_PER_QK
#define FA_VALU_PER_QK 12
#endif

template <class T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab_rsrc(const T* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

template <class T, int D, int DV, int ABL>
__global__ __launch_bounds__(kThreads, 2) void abl_fwd(FwdParams p) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int KROW = kBN * 2;
    constexpr int VROW = kBN * 2 + 16;
    constexpr int KBYTES = D * KROW, VBYTES = DV * VROW, STAGE = KBYTES + VBYTES;
    constexpr int KCH = D * 8 / kThreads;
    constexpr int VCH = DV * 8 / kThreads;
    static_assert(KCH >= 1 && VCH >= 1, "head dim class too small");
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

    const int lid = xcd_remap(blockIdx.x, p.total_wg);
    const int b = lid / p.nqb;
    const int qb = lid - b * p.nqb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int N = p.N, Nk = p.Nk, d = p.d, dv = p.dv;
    const auto qrs = slab_rsrc((const T*)p.Q + (int64_t)b * N * d, (uint32_t)(N * d * (int)sizeof(T)));
    const auto krs = slab_rsrc((const T*)p.K + (int64_t)b * Nk * d, (uint32_t)(Nk * d * (int)sizeof(T)));
    const auto vrs = slab_rsrc((const T*)p.V + (int64_t)b * Nk * dv, (uint32_t)(Nk * dv * (int)sizeof(T)));

    const int qi = qb * kBM + wave * 32 + r;
    F8 qf[D / 16];
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int f = 16 * s + 8 * h + e;
            const unsigned short u = __builtin_amdgcn_raw_buffer_load_b16(qrs, (f * N + qi) * 2, 0, 0);
            qf[s][e] = __builtin_bit_cast(T, u);
        }

    const int g = lane >> 4, kh = g & 1, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
    int koff[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
        koff[kb] = (8 * h + qq) * KROW + (((kb * 2 + kh) ^ (((qq >> 1) & 1) << 1)) * 32) + 8 * sig;
    const int voff = r * VROW + 16 * h;

    // per-thread global offsets (bytes) and LDS store offsets of its chunks
    int kgo[KCH], kso[KCH], vgo[VCH], vso[VCH];
#pragma unroll
    for (int it = 0; it < KCH; ++it) {
        const int ch = tid + kThreads * it, f = ch >> 3, pc = ch & 7;
        kgo[it] = (f * Nk + pc * 8) * 2;
        kso[it] = f * KROW + (((pc >> 1) ^ (((f >> 1) & 1) << 1)) * 32) + (pc & 1) * 16;
    }
#pragma unroll
    for (int it = 0; it < VCH; ++it) {
        const int ch = tid + kThreads * it, f = ch >> 3, pc = ch & 7;
        vgo[it] = (f * Nk + pc * 8) * 2;
        vso[it] = f * VROW + pc * 16;
    }
    const int my_key8 = (tid & 7) * 8;  // first key of this thread's chunks within a tile

    f32x16 oacc[DV / 32];
#pragma unroll
    for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
        for (int x = 0; x < 16; ++x) oacc[cb][x] = 0.0f;
    float m_used = kNegInf, m_true = kNegInf, l_run = 0.0f;
    const float c = p.scale_log2;
    const float thr_raw = kRescaleLog2 / c;

    u32x4 kreg[KCH], vreg[VCH];
    auto gload = [&](int j) {
        const int kb0 = j * kBN * 2;
#pragma unroll
        for (int it = 0; it < KCH; ++it) kreg[it] = __builtin_amdgcn_raw_buffer_load_b128(krs, kgo[it] + kb0, 0, 0);
#pragma unroll
        for (int it = 0; it < VCH; ++it) vreg[it] = __builtin_amdgcn_raw_buffer_load_b128(vrs, vgo[it] + kb0, 0, 0);
        // keys >= Nk (partial last tile) read the next feature row: zero V there so
        // that P = 0 meets a finite value (K is masked to -inf on the scores).
        const bool dead = j * kBN + my_key8 >= Nk;
#pragma unroll
        for (int it = 0; it < VCH; ++it)
            if (dead) vreg[it] = u32x4{0u, 0u, 0u, 0u};
    };
    auto lstore = [&](char* buf) {
#pragma unroll
        for (int it = 0; it < KCH; ++it) *(u32x4*)(buf + kso[it]) = kreg[it];
#pragma unroll
        for (int it = 0; it < VCH; ++it) *(u32x4*)(buf + KBYTES + vso[it]) = vreg[it];
    };

    auto compute = [&](const char* klds, const char* vlds, int j) {
        f32x16 sacc[2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
            for (int x = 0; x < 16; ++x) sacc[kb][x] = 0.0f;
#pragma unroll
            for (int s = 0; s < D / 16; ++s) {
                const char* a = klds + koff[kb] + 16 * s * KROW;
                F4 lo, hi;
                if constexpr (ABL & 64) { lo = __builtin_shufflevector(qf[s], qf[s], 0, 1, 2, 3); hi = __builtin_shufflevector(qf[s], qf[s], 4, 5, 6, 7); asm volatile("" :: "v"(a)); }
                else { lo = __builtin_bit_cast(F4, ds_read_tr16(a)); hi = __builtin_bit_cast(F4, ds_read_tr16(a + 4 * KROW)); }
                const F8 af = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                if constexpr (ABL & 8) { asm volatile("" :: "v"(af)); sacc[kb][s] += (float)qf[s][kb]; }
                else sacc[kb] = mfma32x32x16(af, qf[s], sacc[kb]);
            }
        }
        const int key0 = j * kBN;
        if (key0 + kBN > Nk) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int x = 0; x < 16; ++x) {
                    const int kt = kb * 32 + (x & 3) + 4 * ((x >> 2) & 1) + 8 * h + 16 * (x >> 3);
                    if (key0 + kt >= Nk) sacc[kb][x] = kNegInf;
                }
        }
        float mt = kNegInf;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x) mt = fmaxf(mt, sacc[kb][x]);
        mt = swap_halves_max(mt);
        m_true = fmaxf(m_true, mt);
        if (__builtin_amdgcn_ballot_w64(mt > m_used + thr_raw) != 0) {   // wave-uniform, rare
            const float m_new = fmaxf(m_used, mt);
            const float alpha = exp2_fast((m_used - m_new) * c);
            l_run *= alpha;
#pragma unroll
            for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                for (int x = 0; x < 16; ++x) oacc[cb][x] *= alpha;
            m_used = m_new;
        }
        const float mc = m_used * c;
        float ls = 0.0f;
        F8 pf[2][2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                float pv;
                if constexpr (ABL & 1) pv = fmaf(sacc[kb][x], c, -mc);
                else if constexpr (ABL & 16) pv = sacc[kb][x];
                else pv = exp2_fast(fmaf(sacc[kb][x], c, -mc));
                ls += pv;
                pf[kb][x >> 3][x & 7] = (T)pv;
            }
        l_run += ls;
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    F8 va;
                    if constexpr (ABL & 128) va = pf[kb][s ^ 1];
                    else va = *(const F8*)(vlds + voff + cb * 32 * VROW + (kb * 32 + 16 * s) * 2);
                    if constexpr (ABL & 4) { asm volatile("" :: "v"(va), "v"(pf[kb][s])); }
                    else oacc[cb] = mfma32x32x16(va, pf[kb][s], oacc[cb]);
                }
    };

    const int ntiles = (Nk + kBN - 1) / kBN;
    char* const buf0 = smem;
    char* const buf1 = smem + STAGE;
    gload(0);
    lstore(buf0);
    __syncthreads();
    for (int j = 0; j < ntiles; j += 2) {
        if constexpr (!(ABL & 2)) gload(min(j + 1, ntiles - 1));
        compute(buf0, buf0 + KBYTES, j);
        if constexpr (!(ABL & 2)) lstore(buf1);
        if constexpr (!(ABL & 32)) __syncthreads();
        if (j + 1 < ntiles) {
            if constexpr (!(ABL & 2)) gload(min(j + 2, ntiles - 1));
            compute(buf1, buf1 + KBYTES, j + 1);
            if constexpr (!(ABL & 2)) lstore(buf0);
            __syncthreads();
        }
    }

    const float lt = swap_halves_sum(l_run);
    const float inv = 1.0f / lt;
    if (qi < N) {
        T* Ob = (T*)p.O + (int64_t)b * N * dv;
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int cc = cb * 32 + acc_row(x, h);
                if (cc < dv) Ob[(int64_t)cc * N + qi] = (T)(oacc[cb][x] * inv);
            }
        if (h == 0) {
            p.m[(int64_t)b * N + qi] = m_true * p.scale;
            p.l[(int64_t)b * N + qi] = lt * exp2_fast((m_used - m_true) * c);
        }
    }
}

}  // namespace fa
extern "C" int abl_fwd_launch(int abl, const void* Q, const void* K, const void* V, void* O, float* l, float* m,
                              int N, int Nk, int batch, void* stream) {
    fa::FwdParams p;
    p.Q = Q; p.K = K; p.V = V; p.O = O; p.l = l; p.m = m;
    p.N = N; p.Nk = Nk; p.d = 64; p.dv = 64;
    p.nqb = (N + 127) / 128; p.total_wg = p.nqb * batch;
    p.scale = 0.125f; p.scale_log2 = 0.125f * fa::kLog2e; p.fast = 1;
    dim3 g(p.total_wg), blk(256);
    hipStream_t s = (hipStream_t)stream;
    switch (abl) {
#define C(A) case A: hipLaunchKernelGGL((fa::abl_fwd<fa::bf16, 64, 64, A>), g, blk, 0, s, p); break;
        C(0) C(12) C(14) C(28) C(30) C(76) C(140) C(204) C(206) C(222) C(64) C(128) C(192) C(194)
#undef C
        default: return -1;
    }
    return (int)hipGetLastError();
}
