// fa_fwd.hip — dense flash-attention forward for gfx950 (MI355X, CDNA4).
//
// Replaces the blockwise forward dense_fa!(O, l, m, Q, K, V)
// (reference src/dense.jl:21-102).  Same result — O = softmax(τ Q Kᵀ) V with
// l = Σ exp(s − m), m = max s per query row (src/dense.jl:78-91) — computed
// MI355X-first rather than translated:
//
//  * one workgroup = 4 waves = 128 query rows of one batch slab; each wave owns
//    32 query rows for the whole key sweep (FA-2 order: O accumulates
//    unnormalised in fp32 registers and is divided by l once at the end; the
//    reference renormalises O every tile, src/dense.jl:89 — mathematically
//    equal, documented in DESIGN.md);
//  * key/value tiles of 64 tokens are staged HBM → registers → LDS (issue the
//    next tile's global loads before computing the current one, write them
//    after the tile's barrier: async-STAGE split);
//  * both tile products run on MFMA.  Scores are computed TRANSPOSED,
//    Sᵀ = K·Qᵀ (keys on accumulator rows / registers, queries on lanes), so the
//    fp32 score tile converted to bf16 is already the B operand of Oᵀ = Vᵀ·Pᵀ:
//    no LDS round trip for P, and row max / row sum are register reductions
//    plus one v_permlane32_swap;
//  * the reference layout keeps tokens contiguous, so the QKᵀ contraction
//    (over features) is strided: K tiles are read with the gfx950 transpose
//    read ds_read_b64_tr_b16 from an XOR-swizzled image (conflict-free), while
//    Vᵀ fragments (contraction over tokens, contiguous) are plain ds_read_b128
//    from a padded image (conflict-free);
//  * the key order inside each 16-key group of a K fragment is permuted
//    (bits 2 and 3 swapped) so that each lane's 8 bf16 P values cover 8
//    CONSECUTIVE keys, which makes the Vᵀ fragment one 16-byte read;
//  * exp2 with τ·log2(e) folded into one FMA; the running max is kept in raw
//    dot-product units and converted to natural-log units (m = τ·max) on store;
//  * ragged N / Nk: keys past Nk get score −inf (the reference CUDA kernel
//    zero-fills them, src/cuda/flash.jl:45 — Appendix A.4, not inherited),
//    queries past N are computed on zeros and not stored;
//  * head dims are padded (zero features) to the compiled class 32/64/128,
//    so the reference's own test shape (dqk = 12, dv = 6, test/test.jl:6-10)
//    runs on the same kernels;
//  * blockIdx is remapped so that all workgroups of one batch slab share an
//    XCD (its 4 MiB L2 then serves the slab's K/V re-reads).
//
// fp32 inputs use the exact-f32 MFMA v_mfma_f32_32x32x2_f32 (no TF32 on
// gfx950) with the same structure; that path exists for fp32 parity, the
// performance path is bf16 / fp16.
#include <type_traits>

#include "fa_common.h"
#include "fa_internal.h"
#include "fa_fwd_params.h"
#include "../../include/fa_hip.h"

// Diagnostic hooks (tools/exp/fwd_stamp.hip; empty / 0 in the product build):
// FA_FWD_STAMP(k) records s_memtime / s_memrealtime at phase k of dense_fwd_tiled;
// FA_FWD_ABL selects timing-only ablations that compute WRONG results
// (1: no v_exp, 2: no row sum, 4: no row max).
#ifndef FA_FWD_STAMP
#define FA_FWD_STAMP(k)
#endif
#ifndef FA_FWD_ABL
#define FA_FWD_ABL 0
#endif
// FA_FWD_OAUX: cache-policy bits of the LDS-staged O stores (0 plain; A/B builds only)
#ifndef FA_FWD_OAUX
#define FA_FWD_OAUX 0
#endif

namespace fa {

thread_local int g_fwd_variant = 0;
thread_local int g_fwd_last_path = 0;   // fa_debug_fwd_last_path: 30 when the last fast launch ran fa_fwd_p4  // 0: auto; 4..7: forced geometry (benchmark knob, fa_debug_set_fwd_variant)
thread_local float g_fwd_rescale_log2 = kRescaleLog2;  // fa_debug_set_rescale_threshold (accuracy tests)

// FwdParams: fa_fwd_params.h (shared with fa_fwd_pipe.hip)

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

// --------------------------------------------------------------------------
// bf16 / fp16 forward (v_mfma_f32_32x32x16_{bf16,f16})
// --------------------------------------------------------------------------
template <class T, int D, int DV>
__global__ __launch_bounds__(kThreads) void dense_fwd_generic(FwdParams p) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int KROW = kBN * 2;       // K image: [D][64 keys], 128-B rows, 32-B chunk XOR swizzle
    constexpr int VROW = kBN * 2 + 16;  // V image: [DV][64 keys], 144-B rows (pad → conflict-free b128)
    constexpr int KCH = D * 8 / kThreads;   // 16-B K chunks per thread per tile
    constexpr int VCH = DV * 8 / kThreads;
    static_assert(KCH >= 1 && VCH >= 1, "head dim class too small");
    __shared__ __attribute__((aligned(16))) char smem[D * KROW + DV * VROW];
    char* const klds = smem;
    char* const vlds = smem + D * KROW;

    const int lid = xcd_remap(blockIdx.x, p.total_wg);
    const int b = lid / p.nqb;
    const int qb = lid - b * p.nqb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int N = p.N, Nk = p.Nk, d = p.d, dv = p.dv;
    const T* __restrict__ Qb = (const T*)p.Q + (int64_t)b * N * d;
    const T* __restrict__ Kb = (const T*)p.K + (int64_t)b * Nk * d;
    const T* __restrict__ Vb = (const T*)p.V + (int64_t)b * Nk * dv;
    const bool fast = p.fast != 0;

    // Q^T fragments (B operand of S^T = K Q^T), kept in registers:
    // lane (r, h), k-step s holds Q[query qi][features 16s+8h .. 16s+8h+7].
    const int qi = qb * kBM + wave * 32 + r;
    F8 qf[D / 16];
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int f = 16 * s + 8 * h + e;
            qf[s][e] = (qi < N && f < d) ? Qb[(int64_t)f * N + qi] : (T)0.0f;
        }

    // Per-lane LDS offsets of the transposed K reads.  16-lane group g: kh = g&1
    // selects keys 0-15 / 16-31 of a 32-key block; lane 4q+pp supplies feature
    // row q and the 4-key chunk sigma(pp) (sigma swaps 1 and 2 → lane r ends up
    // holding key pi(r) = r with bits 2 and 3 swapped).
    const int g = lane >> 4, kh = g & 1, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
    int koff[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
        koff[kb] = (8 * h + qq) * KROW + (((kb * 2 + kh) ^ (((qq >> 1) & 1) << 1)) * 32) + 8 * sig;
    const int voff = r * VROW + 16 * h;  // + cb*32*VROW + (kb*32+16s)*2

    f32x16 oacc[DV / 32];
#pragma unroll
    for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
        for (int x = 0; x < 16; ++x) oacc[cb][x] = 0.0f;
    float m_run = kNegInf, l_run = 0.0f;
    const float c = p.scale_log2;

    u32x4 kreg[KCH], vreg[VCH];
    auto gload = [&](int j) {
        const int key0 = j * kBN;
#pragma unroll
        for (int it = 0; it < KCH; ++it) {
            const int ch = tid + kThreads * it;
            kreg[it] = load_chunk<T>(Kb, ch >> 3, key0 + (ch & 7) * 8, d, Nk, fast);
        }
#pragma unroll
        for (int it = 0; it < VCH; ++it) {
            const int ch = tid + kThreads * it;
            vreg[it] = load_chunk<T>(Vb, ch >> 3, key0 + (ch & 7) * 8, dv, Nk, fast);
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int it = 0; it < KCH; ++it) {
            const int ch = tid + kThreads * it, f = ch >> 3, pc = ch & 7;
            const int off = f * KROW + (((pc >> 1) ^ (((f >> 1) & 1) << 1)) * 32) + (pc & 1) * 16;
            *(u32x4*)(klds + off) = kreg[it];
        }
#pragma unroll
        for (int it = 0; it < VCH; ++it) {
            const int ch = tid + kThreads * it;
            *(u32x4*)(vlds + (ch >> 3) * VROW + (ch & 7) * 16) = vreg[it];
        }
    };

    const int ntiles = (Nk + kBN - 1) / kBN;
    gload(0);
    lstore();
    __syncthreads();

    for (int j = 0; j < ntiles; ++j) {
        const bool more = j + 1 < ntiles;
        if (more) gload(j + 1);

        // ---- S^T = K Q^T : two 32-key accumulator blocks ----
        f32x16 sacc[2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
            for (int x = 0; x < 16; ++x) sacc[kb][x] = 0.0f;
#pragma unroll
            for (int s = 0; s < D / 16; ++s) {
                const char* a = klds + koff[kb] + 16 * s * KROW;
                const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(a));
                const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(a + 4 * KROW));
                const F8 af = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                sacc[kb] = mfma32x32x16(af, qf[s], sacc[kb]);
            }
        }

        // ---- mask keys >= Nk (last tile only) ----
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

        // ---- online softmax (raw dot-product units; exp2 with folded scale) ----
        float mt = kNegInf;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x) mt = fmaxf(mt, sacc[kb][x]);
        mt = swap_halves_max(mt);
        const float m_new = fmaxf(m_run, mt);
        const float alpha = exp2_fast((m_run - m_new) * c);
        const float mc = m_new * c;
        float ls = 0.0f;
        F8 pf[2][2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const float pv = exp2_fast(fmaf(sacc[kb][x], c, -mc));
                ls += pv;
                pf[kb][x >> 3][x & 7] = (T)pv;
            }
        l_run = l_run * alpha + ls;
        m_run = m_new;
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int x = 0; x < 16; ++x) oacc[cb][x] *= alpha;

        // ---- O^T += V^T P^T ----
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const F8 va = *(const F8*)(vlds + voff + cb * 32 * VROW + (kb * 32 + 16 * s) * 2);
                    oacc[cb] = mfma32x32x16(va, pf[kb][s], oacc[cb]);
                }

        __syncthreads();
        if (more) {
            lstore();
            __syncthreads();
        }
    }

    // ---- epilogue: O = O / l ; l, m in natural-log units ----
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
            p.m[(int64_t)b * N + qi] = m_run * p.scale;
            p.l[(int64_t)b * N + qi] = lt;
        }
    }
}

// --------------------------------------------------------------------------
// fp32 forward (exact f32 MFMA v_mfma_f32_32x32x2_f32)
// --------------------------------------------------------------------------
template <int D, int DV>
__global__ __launch_bounds__(kThreads) void dense_fwd_generic_f32(FwdParams p) {
    constexpr int KROWF = kBN;       // K image [D][64] floats
    constexpr int VROWF = kBN + 1;   // V image [DV][65] floats (pad → conflict-free column reads)
    constexpr int KCH = D * 16 / kThreads;
    constexpr int VCH = DV * 16 / kThreads;
    static_assert(KCH >= 1 && VCH >= 1, "head dim class too small");
    __shared__ __attribute__((aligned(16))) float smem[D * KROWF + DV * VROWF];
    float* const klds = smem;
    float* const vlds = smem + D * KROWF;

    const int lid = xcd_remap(blockIdx.x, p.total_wg);
    const int b = lid / p.nqb;
    const int qb = lid - b * p.nqb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int N = p.N, Nk = p.Nk, d = p.d, dv = p.dv;
    const float* __restrict__ Qb = (const float*)p.Q + (int64_t)b * N * d;
    const float* __restrict__ Kb = (const float*)p.K + (int64_t)b * Nk * d;
    const float* __restrict__ Vb = (const float*)p.V + (int64_t)b * Nk * dv;
    const bool fast = p.fast != 0;

    const int qi = qb * kBM + wave * 32 + r;
    float qf[D / 2];  // lane (r, h), step t: Q[qi][feature 2t+h]
#pragma unroll
    for (int t = 0; t < D / 2; ++t) {
        const int f = 2 * t + h;
        qf[t] = (qi < N && f < d) ? Qb[(int64_t)f * N + qi] : 0.0f;
    }

    f32x16 oacc[DV / 32];
#pragma unroll
    for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
        for (int x = 0; x < 16; ++x) oacc[cb][x] = 0.0f;
    float m_run = kNegInf, l_run = 0.0f;
    const float c = p.scale_log2;

    u32x4 kreg[KCH], vreg[VCH];
    auto gload = [&](int j) {
        const int key0 = j * kBN;
#pragma unroll
        for (int it = 0; it < KCH; ++it) {
            const int ch = tid + kThreads * it;
            kreg[it] = load_chunk<float>(Kb, ch >> 4, key0 + (ch & 15) * 4, d, Nk, fast);
        }
#pragma unroll
        for (int it = 0; it < VCH; ++it) {
            const int ch = tid + kThreads * it;
            vreg[it] = load_chunk<float>(Vb, ch >> 4, key0 + (ch & 15) * 4, dv, Nk, fast);
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int it = 0; it < KCH; ++it) {
            const int ch = tid + kThreads * it;
            *(u32x4*)(klds + (ch >> 4) * KROWF + (ch & 15) * 4) = kreg[it];
        }
#pragma unroll
        for (int it = 0; it < VCH; ++it) {
            const int ch = tid + kThreads * it;
            float* dst = vlds + (ch >> 4) * VROWF + (ch & 15) * 4;
#pragma unroll
            for (int e = 0; e < 4; ++e) dst[e] = __uint_as_float(vreg[it][e]);
        }
    };

    const int ntiles = (Nk + kBN - 1) / kBN;
    gload(0);
    lstore();
    __syncthreads();

    for (int j = 0; j < ntiles; ++j) {
        const bool more = j + 1 < ntiles;
        if (more) gload(j + 1);

        f32x16 sacc[2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
            for (int x = 0; x < 16; ++x) sacc[kb][x] = 0.0f;
#pragma unroll
            for (int t = 0; t < D / 2; ++t)
                sacc[kb] = mfma32x32x2(klds[(2 * t + h) * KROWF + kb * 32 + r], qf[t], sacc[kb]);
        }

        const int key0 = j * kBN;
        if (key0 + kBN > Nk) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int x = 0; x < 16; ++x)
                    if (key0 + kb * 32 + acc_row(x, h) >= Nk) sacc[kb][x] = kNegInf;
        }

        float mt = kNegInf;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x) mt = fmaxf(mt, sacc[kb][x]);
        mt = swap_halves_max(mt);
        const float m_new = fmaxf(m_run, mt);
        const float alpha = exp2_fast((m_run - m_new) * c);
        const float mc = m_new * c;
        float ls = 0.0f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const float pv = exp2_fast(fmaf(sacc[kb][x], c, -mc));
                ls += pv;
                sacc[kb][x] = pv;
            }
        l_run = l_run * alpha + ls;
        m_run = m_new;
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int x = 0; x < 16; ++x) oacc[cb][x] *= alpha;

#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int x = 0; x < 16; ++x)
                    oacc[cb] = mfma32x32x2(vlds[(cb * 32 + r) * VROWF + kb * 32 + acc_row(x, h)],
                                           sacc[kb][x], oacc[cb]);

        __syncthreads();
        if (more) {
            lstore();
            __syncthreads();
        }
    }

    const float lt = swap_halves_sum(l_run);
    const float inv = 1.0f / lt;
    if (qi < N) {
        float* Ob = (float*)p.O + (int64_t)b * N * dv;
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int cc = cb * 32 + acc_row(x, h);
                if (cc < dv) Ob[(int64_t)cc * N + qi] = oacc[cb][x] * inv;
            }
        if (h == 0) {
            p.m[(int64_t)b * N + qi] = m_run * p.scale;
            p.l[(int64_t)b * N + qi] = lt;
        }
    }
}

// --------------------------------------------------------------------------
// bf16 / fp16 fast path: K/V rows 16-B aligned, Nk % 8 == 0, slab < 4 GiB.
//
// Differences from the generic kernel:
//  * every global access is an unconditional buffer load through a per-slab
//    descriptor (num_records = slab bytes): reads of padded feature rows
//    (f >= d) fall outside the slab and return 0, so the loop body has no
//    divergent control flow and hipcc keeps the tile loads in flight across the
//    whole compute phase (no vmcnt(0) next to the issue);
//  * LDS is double-buffered: tile j+1's registers are written into the other
//    buffer right after tile j's compute, one barrier per tile;
//  * lazy rescaling: the running max used for the exponentials (m_used) is
//    only raised when a tile's max exceeds it by more than kRescaleLog2 (in
//    log2 units), so the O / l rescale is a rare, wave-uniform branch; P is then
//    bounded by 2^kRescaleLog2 (bf16 keeps its relative precision), and the
//    exact max is tracked separately for the returned m (and l is converted to
//    it at the end).
// --------------------------------------------------------------------------

// --------------------------------------------------------------------------
// bf16 / fp16 fast path, generalised geometry: NW waves x 32 query rows per
// workgroup, BN keys per tile (the v2 structure: double-buffered LDS, one
// barrier per tile, lazy rescale, branch-free buffer loads).  The partial-tile
// V zeroing runs only on the last tile.
// --------------------------------------------------------------------------
template <class T, int D, int DV, int NW, int BN, int NQB, bool SPLIT = false, bool WIDE = false>
__device__ __forceinline__ void dense_fwd_tiled(const FwdParams& p) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int NTH = 64 * NW;
    constexpr int BM = 32 * NW * NQB;           // query rows per workgroup
    constexpr int NKB = BN / 32;                // 32-key accumulator blocks per tile
    constexpr int KROW = BN * 2;                // K image row (bytes)
    constexpr int VROW = BN * 2 + 16;           // V image row (bytes), padded
    constexpr int KBYTES = D * KROW, VBYTES = DV * VROW, STAGE = KBYTES + VBYTES;
    constexpr int CPR = BN / 8;                 // 16-B chunks per row
    constexpr int KTOT = D * CPR, VTOT = DV * CPR;   // 16-B chunks per tile
    constexpr int KCH = (KTOT + NTH - 1) / NTH;
    constexpr int VCH = (VTOT + NTH - 1) / NTH;
    static_assert(KTOT % NTH == 0 || KTOT < NTH, "tile split");
    static_assert(VTOT % NTH == 0 || VTOT < NTH, "tile split");
    // WIDE: Q arrives by LDS-DMA (16-B coalesced loads, no VGPRs) into a [feature][BM
    // tokens] image read back by transposed reads, and O leaves through the same image
    // as 16-B row stores, instead of 2-byte gathers / scatters (one per feature and
    // query).  The 32-B blocks of image row f are XOR-ed with (f & 3) | (bit 2 of f) << 2:
    // conflict-free transposed reads (4 rows) and b16 writes (rows f, f + 4).
    constexpr int ROWB = BM * 2;
    constexpr int QOOFF = (2 * STAGE + 16 + 255) & ~255;
    constexpr int QOB = WIDE ? (D > DV ? D : DV) * ROWB : 0;
    __shared__ __attribute__((aligned(256))) char smem[QOOFF + QOB];   // +16 past the stages: dump slot
    auto qo_at = [](int f, int byteoff) {
        const int X = (f & 3) | (((f >> 2) & 1) << 2);
        return f * ROWB + (((byteoff >> 5) ^ X) << 5) + (byteoff & 31);
    };
    char* const qoimg = smem + QOOFF;

    // K image swizzle: XOR the 32-B chunk index so that the 4 feature rows a
    // transposed read touches land on distinct banks (128-B rows: rows f and
    // f+1 are 32 banks apart already; 256-B rows need a 2-bit XOR).
    auto kswz = [](int f) { return BN == 64 ? (((f >> 1) & 1) << 1) : ((f & 3) << 1); };

    FA_FWD_STAMP(0);
    int lid = xcd_remap(blockIdx.x, p.total_wg);
    const int split = SPLIT ? lid % p.nsplit : 0;
    if (SPLIT) lid /= p.nsplit;
    const int b = lid / p.nqb;
    const int qb = lid - b * p.nqb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int N = p.N, Nk = p.Nk, d = p.d, dv = p.dv;
    const auto qrs = slab_rsrc((const T*)p.Q + (int64_t)b * N * d, (uint32_t)(N * d * (int)sizeof(T)));
    const int ldk = p.ldk;
    const auto krs = slab_rsrc((const T*)p.K + (int64_t)b * ldk * d, (uint32_t)(ldk * d * (int)sizeof(T)));
    const auto vrs = slab_rsrc((const T*)p.V + (int64_t)b * ldk * dv, (uint32_t)(ldk * dv * (int)sizeof(T)));

    int qiv[NQB];
    F8 qf[NQB][D / 16];
    if constexpr (WIDE) {
        static_assert(D * ROWB % (1024 * NW) == 0, "Q image DMA split");
#pragma unroll
        for (int it = 0; it < D * ROWB / 1024 / NW; ++it) {
            const int k = it * NW + wave;
            const int P = k * 1024 + lane * 16, f = P / ROWB, pb = P - f * ROWB;
            const int X = (f & 3) | (((f >> 2) & 1) << 2);
            const int lb = (((pb >> 5) ^ X) << 5) + (pb & 31);     // logical byte = 2 * token
            __builtin_amdgcn_raw_ptr_buffer_load_lds(qrs, (__attribute__((address_space(3))) void*)(qoimg + k * 1024), 16,
                                                     (f * N + qb * BM) * 2 + lb, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < NQB; ++u) qiv[u] = qb * BM + (wave * NQB + u) * 32 + r;
    }
#pragma unroll
    for (int u = 0; u < NQB && !WIDE; ++u) {
        qiv[u] = qb * BM + (wave * NQB + u) * 32 + r;
#pragma unroll
        for (int s = 0; s < D / 16; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int f = 16 * s + 8 * h + e;
                const unsigned short w = __builtin_amdgcn_raw_buffer_load_b16(qrs, (f * N + qiv[u]) * 2, 0, 0);
                qf[u][s][e] = __builtin_bit_cast(T, w);
            }
    }

    const int g = lane >> 4, kh = g & 1, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
    int koff[NKB];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
        koff[kb] = (8 * h + qq) * KROW + (((kb * 2 + kh) ^ kswz(qq)) * 32) + 8 * sig;
    const int voff = r * VROW + 16 * h;

    int kgo[KCH], kso[KCH], vgo[VCH], vso[VCH];
    // threads past the chunk count (small head dims at 8 waves) load an
    // out-of-range offset (→ 0) and store into a scratch slot past the tile
    const bool kact = KTOT >= NTH || tid < KTOT, vact = VTOT >= NTH || tid < VTOT;
#pragma unroll
    for (int it = 0; it < KCH; ++it) {
        const int ch = tid + NTH * it, f = ch / CPR, pc = ch % CPR;
        kgo[it] = kact ? (f * ldk + pc * 8) * 2 : 0x7FFFFFF0;
        kso[it] = kact ? f * KROW + (((pc >> 1) ^ kswz(f)) * 32) + (pc & 1) * 16 : 2 * STAGE;
    }
#pragma unroll
    for (int it = 0; it < VCH; ++it) {
        const int ch = tid + NTH * it, f = ch / CPR, pc = ch % CPR;
        vgo[it] = vact ? (f * ldk + pc * 8) * 2 : 0x7FFFFFF0;
        vso[it] = vact ? f * VROW + pc * 16 : 2 * STAGE - KBYTES;
    }

    f32x16 oacc[NQB][DV / 32];
#pragma unroll
    for (int u = 0; u < NQB; ++u)
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int x = 0; x < 16; ++x) oacc[u][cb][x] = 0.0f;
    float m_used[NQB], m_true[NQB], l_run[NQB];
#pragma unroll
    for (int u = 0; u < NQB; ++u) { m_used[u] = kNegInf; m_true[u] = kNegInf; l_run[u] = 0.0f; }
    const float c = p.scale_log2;
    const float thr_raw = p.rescale_log2 / c;
    const int NT = (Nk + BN - 1) / BN;
    const bool ragged = (Nk % BN) != 0;

    u32x4 kreg[KCH], vreg[VCH];
    auto gload = [&](int j) {
        const int kb0 = j * BN * 2;
#pragma unroll
        for (int it = 0; it < KCH; ++it) kreg[it] = __builtin_amdgcn_raw_buffer_load_b128(krs, kgo[it] + kb0, 0, 0);
#pragma unroll
        for (int it = 0; it < VCH; ++it) vreg[it] = __builtin_amdgcn_raw_buffer_load_b128(vrs, vgo[it] + kb0, 0, 0);
    };
    auto lstore = [&](char* buf, int j) {
        if (ragged && j == NT - 1) {   // keys >= Nk read the next feature row: zero V there
#pragma unroll
            for (int it = 0; it < VCH; ++it) {
                const int ch = tid + NTH * it;
                if (j * BN + (ch % CPR) * 8 >= Nk) vreg[it] = u32x4{0u, 0u, 0u, 0u};
            }
        }
#pragma unroll
        for (int it = 0; it < KCH; ++it) *(u32x4*)((kact ? buf : smem) + kso[it]) = kreg[it];
#pragma unroll
        for (int it = 0; it < VCH; ++it) *(u32x4*)((vact ? buf : smem) + KBYTES + vso[it]) = vreg[it];
    };

    auto compute = [&](const char* klds, const char* vlds, int j) {
        f32x16 sacc[NQB][NKB];
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
#pragma unroll
            for (int u = 0; u < NQB; ++u)
#pragma unroll
                for (int x = 0; x < 16; ++x) sacc[u][kb][x] = 0.0f;
#pragma unroll
            for (int s = 0; s < D / 16; ++s) {
                const char* a = klds + koff[kb] + 16 * s * KROW;
                const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(a));
                const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(a + 4 * KROW));
                const F8 af = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
                for (int u = 0; u < NQB; ++u) sacc[u][kb] = mfma32x32x16(af, qf[u][s], sacc[u][kb]);
            }
        }
        if (ragged && j == NT - 1) {
            const int key0 = j * BN;
#pragma unroll
            for (int u = 0; u < NQB; ++u)
#pragma unroll
                for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                    for (int x = 0; x < 16; ++x) {
                        const int kt = kb * 32 + (x & 3) + 4 * ((x >> 2) & 1) + 8 * h + 16 * (x >> 3);
                        if (key0 + kt >= Nk) sacc[u][kb][x] = kNegInf;
                    }
        }
        F8 pf[NQB][NKB][2];
#pragma unroll
        for (int u = 0; u < NQB; ++u) {
            // lane-local tile max (this lane's half of the keys): the lazy check needs no
            // cross-lane step, since the query's other half-lane takes part in the same
            // wave-wide ballot; only a rescale combines the halves.  m_true stays
            // lane-local and is combined once after the loop (bitwise the same result).
            const float mt = (FA_FWD_ABL & 4) ? sacc[u][0][0] : lane_max<NKB>(sacc[u]);
            m_true[u] = vmax(m_true[u], mt);
            if (__builtin_amdgcn_ballot_w64(mt > m_used[u] + thr_raw) != 0) {
                const float m_new = fmaxf(m_used[u], swap_halves_max(mt));
                const float alpha = exp2_fast((m_used[u] - m_new) * c);
                l_run[u] *= alpha;
#pragma unroll
                for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                    for (int x = 0; x < 16; ++x) oacc[u][cb][x] *= alpha;
                m_used[u] = m_new;
            }
            const float mc = m_used[u] * c;
            float ps[4];
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int x = 0; x < 16; ++x) {
                    const float arg = fmaf(sacc[u][kb][x], c, -mc);
                    const float pv = (FA_FWD_ABL & 1) ? arg : exp2_fast(arg);
                    // first four seed the partial sums (no `0 + p` adds: without
                    // fast-math the compiler must keep them, -0 + 0 != -0)
                    if (kb == 0 && x < 4) ps[x] = pv; else if (!(FA_FWD_ABL & 2)) ps[x & 3] += pv;
                    pf[u][kb][x >> 3][x & 7] = (T)pv;
                }
            l_run[u] += (ps[0] + ps[1]) + (ps[2] + ps[3]);
        }
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const F8 va = *(const F8*)(vlds + voff + cb * 32 * VROW + (kb * 32 + 16 * s) * 2);
#pragma unroll
                    for (int u = 0; u < NQB; ++u) oacc[u][cb] = mfma32x32x16(va, pf[u][kb][s], oacc[u][cb]);
                }
    };

    char* const buf0 = smem;
    char* const buf1 = smem + STAGE;
    // key tiles [jt0, jt1) of this workgroup (all tiles unless split-KV)
    const int jt0 = SPLIT ? split * p.tps : 0, jt1 = SPLIT ? min(NT, jt0 + p.tps) : NT;
    gload(jt0);
    lstore(buf0, jt0);
    if constexpr (WIDE) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's Q DMA landed
    __syncthreads();
    if constexpr (WIDE) {
#pragma unroll
        for (int u = 0; u < NQB; ++u)
#pragma unroll
            for (int s = 0; s < D / 16; ++s) {
                const int tb = ((wave * NQB + u) * 32 + 16 * kh + 4 * pp) * 2;
                const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(qoimg + qo_at(16 * s + 8 * h + qq, tb)));
                const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(qoimg + qo_at(16 * s + 8 * h + 4 + qq, tb)));
                qf[u][s] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
            }
    }
    FA_FWD_STAMP(1);
    for (int j = jt0; j < jt1; j += 2) {
        gload(min(j + 1, jt1 - 1));
        compute(buf0, buf0 + KBYTES, j);
        lstore(buf1, min(j + 1, jt1 - 1));
        __syncthreads();
        if (j + 1 < jt1) {
            gload(min(j + 2, jt1 - 1));
            compute(buf1, buf1 + KBYTES, j + 1);
            lstore(buf0, min(j + 2, jt1 - 1));
            __syncthreads();
        }
    }
    FA_FWD_STAMP(2);
#pragma unroll
    for (int u = 0; u < NQB; ++u) m_true[u] = swap_halves_max(m_true[u]);   // the query's two half-lanes

    if constexpr (SPLIT) {   // partials: O, l relative to exp2(c (s - m_true)), m_true in raw units
        const int64_t sb = (int64_t)split * p.batch + b;
#pragma unroll
        for (int u = 0; u < NQB; ++u) {
            const int qi = qiv[u];
            const float sc = exp2_fast((m_used[u] - m_true[u]) * c);
            const float lt = swap_halves_sum(l_run[u]) * sc;
            if (qi < N) {
                float* Op = p.opart + sb * N * dv;
#pragma unroll
                for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                    for (int x = 0; x < 16; ++x) {
                        const int cc = cb * 32 + acc_row(x, h);
                        if (cc < dv) Op[(int64_t)cc * N + qi] = oacc[u][cb][x] * sc;
                    }
                if (h == 0) {
                    p.mpart[sb * N + qi] = m_true[u];
                    p.lpart[sb * N + qi] = lt;
                }
            }
        }
        return;
    }

    if constexpr (WIDE) {
        // O (normalised, T) into the Q/O image, then one 16-B store per lane and row chunk
#pragma unroll
        for (int u = 0; u < NQB; ++u) {
            const int qi = qiv[u];
            const float lt = swap_halves_sum(l_run[u]);
            const float inv = 1.0f / lt;
            const int tb = ((wave * NQB + u) * 32 + r) * 2;
#pragma unroll
            for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                for (int x = 0; x < 16; ++x)
                    *(T*)(qoimg + qo_at(cb * 32 + acc_row(x, h), tb)) = (T)(oacc[u][cb][x] * inv);
            if (qi < N && h == 0) {
                p.m[(int64_t)b * N + qi] = m_true[u] * p.scale;
                p.l[(int64_t)b * N + qi] = lt * exp2_fast((m_used[u] - m_true[u]) * c);
            }
        }
        __syncthreads();
        const auto ors = slab_rsrc((T*)p.O + (int64_t)b * N * dv, (uint32_t)(N * dv * (int)sizeof(T)));
        constexpr int CPRO = ROWB / 16;
        static_assert(DV * CPRO % NTH == 0, "O image store split");
#pragma unroll
        for (int it = 0; it < DV * CPRO / NTH; ++it) {
            const int ch = it * NTH + tid, f = ch / CPRO, lb = (ch - f * CPRO) * 16;
            const int q = qb * BM + lb / 2;
            const u32x4 v4 = *(const u32x4*)(qoimg + qo_at(f, lb));
            // branch-free: a chunk outside (dv, N) gets an offset past the slab descriptor's
            // range, which the buffer store drops (no per-store exec-mask branch in the tail)
            const int off = (f < dv && q < N) ? (f * N + q) * 2 : 0x7FFFFFF0;
            __builtin_amdgcn_raw_buffer_store_b128(v4, ors, off, 0, FA_FWD_OAUX);
        }
        FA_FWD_STAMP(3);
        return;
    }
#pragma unroll
    for (int u = 0; u < NQB; ++u) {
        const int qi = qiv[u];
        const float lt = swap_halves_sum(l_run[u]);
        const float inv = 1.0f / lt;
        if (qi < N) {
            T* Ob = (T*)p.O + (int64_t)b * N * dv;
#pragma unroll
            for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                for (int x = 0; x < 16; ++x) {
                    const int cc = cb * 32 + acc_row(x, h);
                    if (cc < dv) Ob[(int64_t)cc * N + qi] = (T)(oacc[u][cb][x] * inv);
                }
            if (h == 0) {
                p.m[(int64_t)b * N + qi] = m_true[u] * p.scale;
                p.l[(int64_t)b * N + qi] = lt * exp2_fast((m_used[u] - m_true[u]) * c);
            }
        }
    }
}

template <class T, int D, int DV>
__global__ __launch_bounds__(512, 1) void dense_fwd_w8b64(FwdParams p) { dense_fwd_tiled<T, D, DV, 8, 64, 1>(p); }
template <class T, int D, int DV>
__global__ __launch_bounds__(512, 1) void dense_fwd_w8q2(FwdParams p) { dense_fwd_tiled<T, D, DV, 8, 64, 2>(p); }
// the default geometries with LDS-staged Q / O (N % 8 == 0, Q and O 16-B aligned)
template <class T, int D, int DV>
__global__ __launch_bounds__(512, 1) void dense_fwd_w8q2_wide(FwdParams p) {
    dense_fwd_tiled<T, D, DV, 8, 64, 2, false, (D <= 64 && DV <= 64)>(p);   // the launcher picks it only there
}
template <class T, int D, int DV>
__global__ __launch_bounds__(512, 1) void dense_fwd_w8b64_wide(FwdParams p) { dense_fwd_tiled<T, D, DV, 8, 64, 1, false, true>(p); }
// split-KV instantiations of the two default geometries (small grids)
template <class T, int D, int DV>
__global__ __launch_bounds__(512, 1) void dense_fwd_w8q2_split(FwdParams p) { dense_fwd_tiled<T, D, DV, 8, 64, 2, true>(p); }
template <class T, int D, int DV>
__global__ __launch_bounds__(512, 1) void dense_fwd_w8b64_split(FwdParams p) { dense_fwd_tiled<T, D, DV, 8, 64, 1, true>(p); }

// Split-KV combine: O = Σ_s o_s·2^(c(m_s − m)) / Σ_s l_s·2^(c(m_s − m)), m = max_s m_s
// (fixed split order: deterministic).  One thread per output element.
template <class T>
__global__ __launch_bounds__(256) void fwd_split_combine(FwdParams p, int64_t total) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    const int N = p.N, dv = p.dv, B = p.batch;
    const int n = (int)(e % N);
    const int64_t rest = e / N;
    const int cc = (int)(rest % dv);
    const int b = (int)(rest / dv);
    const float c = p.scale_log2;
    float mx = kNegInf;
    for (int sp = 0; sp < p.nsplit; ++sp) mx = vmax(mx, p.mpart[((int64_t)sp * B + b) * N + n]);
    float L = 0.0f, acc = 0.0f;
    for (int sp = 0; sp < p.nsplit; ++sp) {
        const int64_t sb = (int64_t)sp * B + b;
        const float w = exp2_fast((p.mpart[sb * N + n] - mx) * c);
        L = fmaf(p.lpart[sb * N + n], w, L);
        acc = fmaf(p.opart[(sb * dv + cc) * N + n], w, acc);
    }
    ((T*)p.O)[((int64_t)b * dv + cc) * N + n] = (T)(acc / L);
    if (cc == 0) {
        p.m[(int64_t)b * N + n] = mx * p.scale;
        p.l[(int64_t)b * N + n] = L;
    }
}

// Split-KV plan for the fast kernels: grids of fewer workgroups than CUs split the
// key range so that ~512 workgroups run (each at least 2 tiles of 64 keys).
struct SplitPlan {
    int nsplit = 1, tps = 0;
    size_t bytes = 0;
};
static SplitPlan split_plan(int dtype, int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch) {
    SplitPlan sp;
    const int Dc = head_dim_class(d), DVc = head_dim_class(dv);
    if (dtype == FA_DTYPE_F32 || dtype == FA_DTYPE_F64 || !Dc || !DVc) return sp;
    const int64_t rows = (Dc <= 64 && DVc <= 64) ? 512 : 256;
    const int64_t wgs = (N + rows - 1) / rows * batch;
    const int64_t NT = (Nk + kBN - 1) / kBN;
    if (wgs >= 256 || NT < 4) return sp;
    int64_t ns = std::min<int64_t>((512 + wgs - 1) / wgs, NT / 2);
    if (ns < 2) return sp;
    const int64_t tps = (NT + ns - 1) / ns;
    ns = (NT + tps - 1) / tps;
    if (ns < 2 || ns * wgs > INT32_MAX) return sp;
    sp.nsplit = (int)ns;
    sp.tps = (int)tps;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    sp.bytes = al((size_t)(ns * batch * N * dv) * 4) + 2 * al((size_t)(ns * batch * N) * 4) + 256;
    return sp;
}

// --------------------------------------------------------------------------
// launcher
// --------------------------------------------------------------------------
bool launch_dense_fwd_p4(const FwdParams& p, int Dc, int DVc, int dtype, hipStream_t s, hipError_t* err);

template <class T, int D>
static hipError_t launch_dv(const FwdParams& p, int DVc, dim3 grid, hipStream_t s) {
    // one wave per SIMD, persistent (fa_fwd_p4.hip): the default at d = dv = 128 (5-8 %
    // over the 8-wave kernel, bitwise equal: profiles/r04_fwd_p4_default_d128_ab.log);
    // at 64 the 8-wave kernel stays (p4 is 15 % slower there); variant 30 forces it
    if (p.fast && (g_fwd_variant == 30 || (g_fwd_variant == 0 && D == 128 && DVc == 128))) {
        hipError_t e = hipSuccess;
        if (launch_dense_fwd_p4(p, D, DVc, std::is_same<T, bf16>::value ? FA_DTYPE_BF16 : FA_DTYPE_F16, s, &e)) {
            g_fwd_last_path = 30;
            return e;
        }
    }
    if (p.fast) {
        // geometry per head-dim class (measured on MI355X):
        // <= 64: 8 waves x 2 query blocks (512 rows / workgroup); 128: 8 waves x 1.
        int v = g_fwd_variant;
        // default geometries stage Q / O through LDS when the shape allows (variant 20:
        // the same geometries with per-element Q gathers / O stores, for A/B)
        const bool wide = p.wide && (v == 0 || v == 5 || v == 7 || v == 30);
        if (v == 0 || v == 20 || v == 30) v = (D <= 64 && DVc <= 64) ? 7 : 5;
        const int nw = 8;
        const int rows = v == 7 ? 512 : 256;   // query rows per workgroup: w8q2 / w8b64
        FwdParams q = p;
        q.nqb = (q.N + rows - 1) / rows;
        q.total_wg = q.nqb * (int)(p.total_wg / p.nqb) * (q.nsplit > 1 ? q.nsplit : 1);
        const dim3 g2((unsigned)q.total_wg);
        const dim3 blk(64 * nw);
#define FA_LAUNCH_T(KER)                                                                \
        switch (DVc) {                                                                  \
            case 32: hipLaunchKernelGGL((KER<T, D, 32>), g2, blk, 0, s, q); break;      \
            case 64: hipLaunchKernelGGL((KER<T, D, 64>), g2, blk, 0, s, q); break;      \
            case 128: hipLaunchKernelGGL((KER<T, D, 128>), g2, blk, 0, s, q); break;    \
            default: return hipErrorInvalidValue;                                       \
        }
        if (q.nsplit > 1 && rows == 256) { FA_LAUNCH_T(dense_fwd_w8b64_split) }
        else if (q.nsplit > 1) { FA_LAUNCH_T(dense_fwd_w8q2_split) }
        else if (v == 5 && wide) { FA_LAUNCH_T(dense_fwd_w8b64_wide) }
        else if (v == 5) { FA_LAUNCH_T(dense_fwd_w8b64) }
        else if (wide) { FA_LAUNCH_T(dense_fwd_w8q2_wide) }
        else { FA_LAUNCH_T(dense_fwd_w8q2) }
#undef FA_LAUNCH_T
        if (q.nsplit > 1) {
            const int64_t total = (int64_t)q.N * q.dv * q.batch;
            hipLaunchKernelGGL(fwd_split_combine<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, q, total);
        }
        return hipGetLastError();
    }
    switch (DVc) {
        case 32: hipLaunchKernelGGL((dense_fwd_generic<T, D, 32>), grid, dim3(kThreads), 0, s, p); break;
        case 64: hipLaunchKernelGGL((dense_fwd_generic<T, D, 64>), grid, dim3(kThreads), 0, s, p); break;
        case 128: hipLaunchKernelGGL((dense_fwd_generic<T, D, 128>), grid, dim3(kThreads), 0, s, p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
template <int D>
static hipError_t launch_dv_f32(const FwdParams& p, int DVc, dim3 grid, hipStream_t s) {
    switch (DVc) {
        case 32: hipLaunchKernelGGL((dense_fwd_generic_f32<D, 32>), grid, dim3(kThreads), 0, s, p); break;
        case 64: hipLaunchKernelGGL((dense_fwd_generic_f32<D, 64>), grid, dim3(kThreads), 0, s, p); break;
        case 128: hipLaunchKernelGGL((dense_fwd_generic_f32<D, 128>), grid, dim3(kThreads), 0, s, p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
template <class T>
static hipError_t launch_typed(const FwdParams& p, int Dc, int DVc, dim3 grid, hipStream_t s) {
    switch (Dc) {
        case 32: return launch_dv<T, 32>(p, DVc, grid, s);
        case 64: return launch_dv<T, 64>(p, DVc, grid, s);
        case 128: return launch_dv<T, 128>(p, DVc, grid, s);
    }
    return hipErrorInvalidValue;
}
static hipError_t launch_f32(const FwdParams& p, int Dc, int DVc, dim3 grid, hipStream_t s) {
    switch (Dc) {
        case 32: return launch_dv_f32<32>(p, DVc, grid, s);
        case 64: return launch_dv_f32<64>(p, DVc, grid, s);
        case 128: return launch_dv_f32<128>(p, DVc, grid, s);
    }
    return hipErrorInvalidValue;
}

static bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15u) == 0; }

// Padded-key fast path: bf16/fp16 K and V are copied into zero-padded slabs of
// row stride Nk8 = roundup(Nk, 8) in the caller's workspace; the fast kernels
// then address rows by ldk = Nk8 and mask keys >= Nk as for any ragged last
// tile.  fa_dense_fwd_workspace reserves that copy only when the SHAPE needs it
// (Nk % 8 != 0): the query has no pointers.  K / V that are not 16-B aligned
// with Nk % 8 == 0 (e.g. a view at an odd element offset) take the same copy
// when the workspace passed is large enough for it (fwd_pad_bytes_any), and the
// generic kernel otherwise.  Without a workspace (fa_dense_fwd) those shapes run
// the generic kernel.
static bool fwd_pad_fits(int dtype, int64_t Nk, int64_t d, int64_t dv, int64_t batch) {
    const int64_t nk8 = (Nk + 7) / 8 * 8;
    return dtype != FA_DTYPE_F32 && dtype != FA_DTYPE_F64 && nk8 * d * 2 < INT32_MAX && nk8 * dv * 2 < INT32_MAX &&
           nk8 * (d > dv ? d : dv) * batch < ((int64_t)1 << 40);
}
static bool fwd_pad_needed(int dtype, int64_t Nk, int64_t d, int64_t dv, int64_t batch) {
    return Nk % 8 != 0 && fwd_pad_fits(dtype, Nk, d, dv, batch);
}
static size_t fwd_pad_bytes_any(int64_t Nk, int64_t d, int64_t dv, int64_t batch) {
    const int64_t nk8 = (Nk + 7) / 8 * 8;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    return al((size_t)(nk8 * d * batch) * 2) + al((size_t)(nk8 * dv * batch) * 2) + 256;
}
static size_t fwd_pad_bytes(int dtype, int64_t Nk, int64_t d, int64_t dv, int64_t batch) {
    if (!fwd_pad_needed(dtype, Nk, d, dv, batch)) return 0;
    return fwd_pad_bytes_any(Nk, d, dv, batch);
}
size_t dense_fwd_workspace(int dtype, int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch) {
    return fwd_pad_bytes(dtype, Nk, d, dv, batch) + split_plan(dtype, N, Nk, d, dv, batch).bytes;
}
// dst (Np, C, B) <- src (N, C, B), zero rows n >= N
template <class T>
__global__ __launch_bounds__(256) void fwd_pad_keys(const T* __restrict__ src, T* __restrict__ dst, int N, int Np,
                                                    int64_t total) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    const int n = (int)(e % Np);
    const int64_t cb = e / Np;                  // c + C·b
    dst[e] = n < N ? src[cb * N + n] : (T)0.0f;
}

int launch_dense_fwd(const DenseArgs& a, hipStream_t s, const char** why) {
    g_fwd_last_path = 0;   // every path below that is not a persistent kernel leaves 0
    if (a.dtype == FA_DTYPE_F64) return launch_dense_fwd_f64(a, s, why);
    const int Dc = head_dim_class(a.d), DVc = head_dim_class(a.dv);
    if (!Dc || !DVc) {
        *why = "head dimension exceeds the compiled maximum (128)";
        return FA_ERR_UNSUPPORTED;
    }
    if (a.N > INT32_MAX / 2 || a.Nk > INT32_MAX / 2 || a.N * a.d > INT32_MAX ||
        a.Nk * a.d > INT32_MAX || a.Nk * a.dv > INT32_MAX || a.N * a.dv > INT32_MAX) {
        *why = "per-slab extent exceeds 2^31 elements";
        return FA_ERR_UNSUPPORTED;
    }
    FwdParams p;
    p.Q = a.Q; p.K = a.K; p.V = a.V; p.O = a.O; p.l = a.l; p.m = a.m;
    p.N = (int)a.N; p.Nk = (int)a.Nk; p.d = (int)a.d; p.dv = (int)a.dv;
    p.nqb = (int)((a.N + kBM - 1) / kBM);
    const int64_t total = (int64_t)p.nqb * a.batch;
    if (total > INT32_MAX) {
        *why = "grid too large";
        return FA_ERR_UNSUPPORTED;
    }
    p.total_wg = (int)total;
    p.scale = a.scale;
    p.scale_log2 = a.scale * kLog2e;
    p.rescale_log2 = g_fwd_rescale_log2;
    p.batch = (int)a.batch;
    p.nsplit = 1; p.tps = 0; p.opart = p.lpart = p.mpart = nullptr;
    const int epc = a.dtype == FA_DTYPE_F32 ? 4 : 8;
    p.ldk = (int)a.Nk;
    p.fast = (a.Nk % epc == 0) && aligned16(a.K) && aligned16(a.V);
    p.wide = a.N % 8 == 0 && aligned16(a.Q) && aligned16(a.O);
    // bytes of the workspace taken by the padded K / V copies (0: none made)
    size_t pad_bytes = 0;
    if (!p.fast && a.workspace && fwd_pad_fits(a.dtype, a.Nk, a.d, a.dv, a.batch) &&
        a.N * a.d * 2 < (int64_t)INT32_MAX &&
        a.workspace_bytes >= fwd_pad_bytes_any(a.Nk, a.d, a.dv, a.batch)) {
        pad_bytes = fwd_pad_bytes_any(a.Nk, a.d, a.dv, a.batch);
        const int64_t nk8 = (a.Nk + 7) / 8 * 8;
        char* w = (char*)(((uintptr_t)a.workspace + 255) & ~(uintptr_t)255);
        char* kp = w;
        char* vp = w + (((size_t)(nk8 * a.d * a.batch) * 2 + 255) & ~(size_t)255);
        const int64_t tk = nk8 * a.d * a.batch, tv = nk8 * a.dv * a.batch;
        if (a.dtype == FA_DTYPE_F16) {
            hipLaunchKernelGGL(fwd_pad_keys<f16>, dim3((unsigned)((tk + 255) / 256)), dim3(256), 0, s, (const f16*)a.K, (f16*)kp, (int)a.Nk, (int)nk8, tk);
            hipLaunchKernelGGL(fwd_pad_keys<f16>, dim3((unsigned)((tv + 255) / 256)), dim3(256), 0, s, (const f16*)a.V, (f16*)vp, (int)a.Nk, (int)nk8, tv);
        } else {
            hipLaunchKernelGGL(fwd_pad_keys<bf16>, dim3((unsigned)((tk + 255) / 256)), dim3(256), 0, s, (const bf16*)a.K, (bf16*)kp, (int)a.Nk, (int)nk8, tk);
            hipLaunchKernelGGL(fwd_pad_keys<bf16>, dim3((unsigned)((tv + 255) / 256)), dim3(256), 0, s, (const bf16*)a.V, (bf16*)vp, (int)a.Nk, (int)nk8, tv);
        }
        p.K = kp;
        p.V = vp;
        p.ldk = (int)nk8;
        p.fast = 1;
    }
    // buffer descriptors address a slab with 32-bit byte offsets
    const int64_t esz = a.dtype == FA_DTYPE_F32 ? 4 : 2;
    if (a.N * a.d * esz >= (int64_t)INT32_MAX || (int64_t)p.ldk * a.d * esz >= (int64_t)INT32_MAX ||
        (int64_t)p.ldk * a.dv * esz >= (int64_t)INT32_MAX)
        p.fast = 0;
    // split-KV for small grids (fast kernels, default geometry, workspace given)
    // (not when fa_fwd_p4's own 256-row blocks already fill the chip)
    const bool p4_fills = (g_fwd_variant == 30 || (g_fwd_variant == 0 && Dc == 128 && DVc == 128)) &&
                          (a.N + 255) / 256 * a.batch >= device_cus(s);
    if (p.fast && (g_fwd_variant == 0 || g_fwd_variant == 30) && !p4_fills && a.workspace) {
        const SplitPlan sp = split_plan(a.dtype, a.N, a.Nk, a.d, a.dv, a.batch);
        if (sp.nsplit > 1 && a.workspace_bytes >= pad_bytes + sp.bytes) {
            auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
            char* w = (char*)(((uintptr_t)a.workspace + 255) & ~(uintptr_t)255) + (pad_bytes ? pad_bytes - 256 : 0);
            w = (char*)(((uintptr_t)w + 255) & ~(uintptr_t)255);
            p.opart = (float*)w;
            w += al((size_t)(sp.nsplit * a.batch * a.N * a.dv) * 4);
            p.lpart = (float*)w;
            w += al((size_t)(sp.nsplit * a.batch * a.N) * 4);
            p.mpart = (float*)w;
            p.nsplit = sp.nsplit;
            p.tps = sp.tps;
        }
    }
    const dim3 grid((unsigned)total);
    hipError_t e;
    switch (a.dtype) {
        case FA_DTYPE_BF16: e = launch_typed<bf16>(p, Dc, DVc, grid, s); break;
        case FA_DTYPE_F16: e = launch_typed<f16>(p, Dc, DVc, grid, s); break;
        case FA_DTYPE_F32: e = launch_f32(p, Dc, DVc, grid, s); break;
        default: *why = "unknown dtype"; return FA_ERR_INVALID_ARG;
    }
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    return FA_OK;
}

}  // namespace fa
