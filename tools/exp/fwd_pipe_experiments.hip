// ARCHIVED EXPERIMENT (round 2) — not built into libfa_hip.so.
// Two forward schedules that were parity-green (bitwise equal to the shipped
// kernel where applicable) but not faster; kept for the record:
//   * dense_fwd_pipe: one wave per SIMD, 32-key steps, QKᵀ(i) | softmax(i-1) |
//     PV(i-2) software pipeline: 709 vs 988 TFLOP/s at configs[1] (the compiler
//     keeps the scores in AGPRs and copies them out, and a single wave exposes
//     every LDS / dependency latency);
//   * dense_fwd_stag: 8 waves, speculative softmax (exponentials against the
//     running max while the tile max is reduced, rare recompute), waves 4-7
//     half an iteration behind: 1010 vs 1012 TFLOP/s (co-executing MFMA/VALU
//     cycles +37 %, VALU instructions +3.5 %: the vector pipe stays the pole).
// To build it for an A/B, add it back to csrc/Makefile's SRCS and restore the
// launcher declarations in fa_fwd_params.h and the dispatch in fa_fwd.hip.
// fa_fwd_pipe.hip — software-pipelined dense forward for gfx950: one wave per
// SIMD, the matrix pipe and the vector pipe of each SIMD fed by ONE wave.
//
// Same result as dense_fa!(O, l, m, Q, K, V) (reference src/dense.jl:21-102) and
// the same layouts, fragments and numerics as dense_fwd_tiled in fa_fwd.hip
// (transposed scores Sᵀ = K·Qᵀ, P kept in registers as the B operand of
// Oᵀ = Vᵀ·Pᵀ, key permutation σ, lazy rescale); what changes is the schedule.
//
// Why: in the 8-wave kernel both waves of a SIMD start each key tile at the
// same barrier, so they run QKᵀ together (matrix pipe busy, vector pipe idle),
// then the softmax together (vector pipe busy, matrix pipe idle), then PV.  At
// d = 64 the softmax costs more vector-issue cycles per tile (≈1264 + 8 per
// MFMA) than the tile's MFMAs take (1024), so the tile time is close to their
// SUM.  Here each wave carries three tiles at once, so the two pipes overlap
// inside the wave:
//
//     step j:   MFMA   Sᵀ(j) = K(j)·Qᵀ           (16 MFMAs at d = 64)
//                      Oᵀ  += V(j-2)ᵀ·P(j-2)ᵀ    (16 MFMAs at dv = 64)
//               VALU   P(j-1) = exp2(c·S(j-1) − c·m_used), row sums, row max
//
// with no dependency between the two streams inside a step, so the compiler
// interleaves them (sched_group_barrier pins the pattern).  The step time is
// then ≈ max(MFMA, VALU + MFMA issue) instead of their sum.
//
// Lazy rescale, speculative form: P(j-1) is exponentiated against the CURRENT
// m_used while its tile max is computed alongside (max and exp are
// independent).  At the end of the step, if any row's tile max exceeds m_used
// by more than the threshold (rare, wave-uniform branch), that tile is
// recomputed against the new max, l is rescaled, and O — which by then holds
// exactly PV(≤ j-2), all at the old max — is rescaled once (cdna guide T13's
// hazard rule: everything still at the old max is scaled exactly once, P(j-1)
// is at the new max).
//
// Workgroup = 4 waves × 64 query rows (two 32-row blocks per wave) = 256 rows
// of one slab; K/V tiles of 64 keys double-buffered in LDS (K image: 128-B
// rows, 32-B XOR swizzle, read by ds_read_b64_tr_b16; V image: 144-B rows,
// read by ds_read_b128), loaded to registers one step ahead and written after
// the step's compute, one barrier per step.
#include "fa_common.h"
#include "fa_internal.h"
#include "fa_fwd_params.h"
#include "../../include/fa_hip.h"

namespace fa {

template <class T, int D, int DV>
__global__ __launch_bounds__(256, 1) void dense_fwd_pipe(FwdParams p) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int NW = 4, QB = 2, BN = 64;
    constexpr int NTH = 64 * NW;
    constexpr int BM = 32 * QB * NW;            // 256 query rows per workgroup
    constexpr int KS = D / 16;                  // k-steps of Sᵀ
    constexpr int NCB = DV / 32;                // 32-row output blocks of Oᵀ
    constexpr int KROW = BN * 2;                // K image row (bytes)
    constexpr int VROW = BN * 2 + 16;           // V image row (bytes), padded
    constexpr int KBYTES = D * KROW, VBYTES = DV * VROW;
    constexpr int SLOT = KBYTES + VBYTES;
    constexpr int CPR = BN / 8;                 // 16-B chunks per row
    constexpr int KTOT = D * CPR, VTOT = DV * CPR;
    constexpr int KCH = (KTOT + NTH - 1) / NTH;
    constexpr int VCH = (VTOT + NTH - 1) / NTH;
    static_assert(KTOT % NTH == 0 || KTOT < NTH, "tile split");
    static_assert(VTOT % NTH == 0 || VTOT < NTH, "tile split");
    __shared__ __attribute__((aligned(16))) char smem[2 * SLOT + 16];   // +16: dump slot

    auto kswz = [](int f) { return ((f >> 1) & 1) << 1; };   // 128-B rows

    const int lid = xcd_remap(blockIdx.x, p.total_wg);
    const int b = lid / p.nqb;
    const int qb = lid - b * p.nqb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int N = p.N, Nk = p.Nk, d = p.d, dv = p.dv;
    const int ldk = p.ldk;
    const auto qrs = slab_rsrc((const T*)p.Q + (int64_t)b * N * d, (uint32_t)(N * d * (int)sizeof(T)));
    const auto krs = slab_rsrc((const T*)p.K + (int64_t)b * ldk * d, (uint32_t)(ldk * d * (int)sizeof(T)));
    const auto vrs = slab_rsrc((const T*)p.V + (int64_t)b * ldk * dv, (uint32_t)(ldk * dv * (int)sizeof(T)));

    // Q fragments (B operand of Sᵀ): query qiv[u], features 16s + 8h + e
    int qiv[QB];
    F8 qf[QB][KS];
#pragma unroll
    for (int u = 0; u < QB; ++u) {
        qiv[u] = qb * BM + (wave * QB + u) * 32 + r;
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int f = 16 * s + 8 * h + e;
                const unsigned short w = __builtin_amdgcn_raw_buffer_load_b16(qrs, (f * N + qiv[u]) * 2, 0, 0);
                qf[u][s][e] = __builtin_bit_cast(T, w);
            }
    }

    // transposed K reads with the key permutation σ (bits 2, 3 of the
    // accumulator row swapped) so each lane's 8 P values are consecutive keys
    const int g = lane >> 4, kh = g & 1, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
    const int koff0 = (8 * h + qq) * KROW + (((0 * 2 + kh) ^ kswz(qq)) * 32) + 8 * sig;
    const int koff1 = (8 * h + qq) * KROW + (((1 * 2 + kh) ^ kswz(qq)) * 32) + 8 * sig;
    const int voff = r * VROW + 16 * h;

    // K / V staging: chunk it of a tile is chunk tid + NTH·it, i.e. feature row
    // f0 + it·(NTH / CPR) at the same column: the per-it offsets are uniform
    // (global: soffset; LDS: immediate), so one lane offset serves every chunk
    static_assert(NTH % CPR == 0, "rows per staging pass");
    constexpr int FPI = NTH / CPR;              // feature rows per staging pass
    const int f0 = tid / CPR, pc0 = tid % CPR;
    const bool kact = KTOT >= NTH || tid < KTOT, vact = VTOT >= NTH || tid < VTOT;
    const int kgo = kact ? (f0 * ldk + pc0 * 8) * 2 : 0x7FFFFFF0;
    const int vgo = vact ? (f0 * ldk + pc0 * 8) * 2 : 0x7FFFFFF0;
    // kswz(f0 + FPI·it) == kswz(f0) (FPI is a multiple of 4)
    const int kso = kact ? f0 * KROW + (((pc0 >> 1) ^ kswz(f0)) * 32) + (pc0 & 1) * 16 : 2 * SLOT;
    const int vso = vact ? KBYTES + f0 * VROW + pc0 * 16 : 2 * SLOT;
    static_assert(FPI % 4 == 0, "swizzle period");

    const float c = p.scale_log2;
    const float thr_raw = p.rescale_log2 / c;
    const int NT = (Nk + BN - 1) / BN;

    f32x16 oacc[QB][NCB];
#pragma unroll
    for (int u = 0; u < QB; ++u)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int x = 0; x < 16; ++x) oacc[u][cb][x] = 0.0f;
    float m_used[QB], m_true[QB], l_run[QB];
#pragma unroll
    for (int u = 0; u < QB; ++u) { m_used[u] = kNegInf; m_true[u] = kNegInf; l_run[u] = 0.0f; }

    // staging registers: K(t+1) is loaded at the start of step 2t and written
    // at its end, V(t) at the start of step 2t+1 and written at its end
    u32x4 kreg[KCH], vreg[VCH];
    auto kload = [&](int t) {
#pragma unroll
        for (int it = 0; it < KCH; ++it)
            kreg[it] = __builtin_amdgcn_raw_buffer_load_b128(krs, kgo, t * BN * 2 + it * FPI * ldk * 2, 0);
    };
    auto vload = [&](int t) {
#pragma unroll
        for (int it = 0; it < VCH; ++it)
            vreg[it] = __builtin_amdgcn_raw_buffer_load_b128(vrs, vgo, t * BN * 2 + it * FPI * ldk * 2, 0);
    };
    auto kstore = [&](int t) {
        char* slot = (kact ? smem + (t & 1) * SLOT : smem) + kso;
#pragma unroll
        for (int it = 0; it < KCH; ++it) *(u32x4*)(slot + it * FPI * KROW) = kreg[it];
    };
    auto vstore = [&](int t) {
        if (t == NT - 1 && (Nk % BN) != 0) {   // keys >= Nk read the next feature row: zero V there
            if (t * BN + pc0 * 8 >= Nk)
#pragma unroll
                for (int it = 0; it < VCH; ++it) vreg[it] = u32x4{0u, 0u, 0u, 0u};
        }
        char* slot = (vact ? smem + ((t + 1) & 1) * SLOT : smem) + vso;
#pragma unroll
        for (int it = 0; it < VCH; ++it) *(u32x4*)(slot + it * FPI * VROW) = vreg[it];
    };

    // 32-key sub-tiles: S[u] = Sᵀ block (32 keys x 32 queries), P[u][s] its
    // bf16 P as two 16-key B fragments.  Two register sets (sub-tile parity).
    f32x16 S0[QB], S1[QB];
    F8 P0[QB][2], P1[QB][2];
    float mt[QB], ps[QB][2];

    // Sᵀ of sub-tile kb of the K tile in `slot`
    auto qk = [&](f32x16 (&S)[QB], const char* slot, int koff) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const char* a = slot + koff + 16 * s * KROW;
            const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(a));
            const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(a + 4 * KROW));
            const F8 af = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
            for (int u = 0; u < QB; ++u)
                S[u] = (s == 0) ? mfma32x32x16(af, qf[u][s], f32x16{}) : mfma32x32x16(af, qf[u][s], S[u]);
        }
    };
    // Oᵀ += Vᵀ·Pᵀ over sub-tile kb of the V tile in `slot`
    auto pv = [&](const F8 (&P)[QB][2], const char* slot, int kb) {
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const F8 va = *(const F8*)(slot + KBYTES + voff + cb * 32 * VROW + (kb * 32 + 16 * s) * 2);
#pragma unroll
                for (int u = 0; u < QB; ++u) oacc[u][cb] = mfma32x32x16(va, P[u][s], oacc[u][cb]);
            }
    };
    // keys >= Nk of sub-tile i: score -inf
    auto mask = [&](f32x16 (&S)[QB], int i) {
        if (32 * i + 32 <= Nk) return;
#pragma unroll
        for (int u = 0; u < QB; ++u)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int kt = (x & 3) + 4 * ((x >> 2) & 1) + 8 * h + 16 * (x >> 3);
                if (32 * i + kt >= Nk) S[u][x] = kNegInf;
            }
    };
    // speculative softmax of S against m_used: P, partial row sums, tile max
    auto smx = [&](const f32x16 (&S)[QB], F8 (&P)[QB][2]) {
#pragma unroll
        for (int u = 0; u < QB; ++u) {
            const float mc = m_used[u] * c;
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const float pv_ = exp2_fast(fmaf(S[u][x], c, -mc));
                if (x < 2) ps[u][x] = pv_; else ps[u][x & 1] += pv_;
                P[u][x >> 3][x & 7] = (T)pv_;
            }
            mt[u] = lane_max<1>(*(const f32x16(*)[1]) & S[u]);
        }
    };
    // end of a step: row max across the half-waves, rescale decision (rare
    // uniform branch: recompute P against the new max, rescale l and O)
    auto finish = [&](const f32x16 (&S)[QB], F8 (&P)[QB][2]) {
        // the speculative P and sums are computed HERE, beside the step's MFMAs:
        // without these opaque uses the compiler sinks them into the branch
        // below (past the MFMAs), which serialises the two pipes again
#pragma unroll
        for (int u = 0; u < QB; ++u) {
            asm volatile("" : "+v"(P[u][0]), "+v"(P[u][1]), "+v"(ps[u][0]), "+v"(ps[u][1]));
        }
        bool need = false;
#pragma unroll
        for (int u = 0; u < QB; ++u) {
            mt[u] = swap_halves_max(mt[u]);
            m_true[u] = vmax(m_true[u], mt[u]);
            need |= mt[u] > m_used[u] + thr_raw;
        }
        if (__builtin_amdgcn_ballot_w64(need) != 0) {
#pragma unroll
            for (int u = 0; u < QB; ++u) {
                const float m_new = fmaxf(m_used[u], mt[u]);
                const float alpha = exp2_fast((m_used[u] - m_new) * c);
                m_used[u] = m_new;
                const float mc = m_new * c;
                float q4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int x = 0; x < 16; ++x) {
                    const float pv_ = exp2_fast(fmaf(S[u][x], c, -mc));
                    q4[x & 3] += pv_;
                    P[u][x >> 3][x & 7] = (T)pv_;
                }
                l_run[u] = l_run[u] * alpha + ((q4[0] + q4[1]) + (q4[2] + q4[3]));
#pragma unroll
                for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
                    for (int x = 0; x < 16; ++x) oacc[u][cb][x] *= alpha;
            }
        } else {
#pragma unroll
            for (int u = 0; u < QB; ++u) l_run[u] += ps[u][0] + ps[u][1];
        }
    };

    // ---- pipeline over 32-key sub-tiles i: step i = QK(i) | SM(i-1) | PV(i-2)
    // Sub-tiles 2t, 2t+1 read K(t) and V(t-1) from LDS slot t&1; the step pair
    // also loads K(t+1), V(t) and writes them into slot (t+1)&1, one barrier
    // per pair.  Even steps: S new = S0, S cur = S1, P cur = P1, P old = P0.
    kload(0);
    kstore(0);
    __syncthreads();
    {   // t = 0: steps 0 (QK(0)) and 1 (QK(1) | SM(0))
        const char* slot = smem;
        if (NT > 1) kload(1);
        qk(S0, slot, koff0);
        if (NT > 1) kstore(1);
        vload(0);
        qk(S1, slot, koff1);
        mask(S0, 0);
        smx(S0, P0);
        finish(S0, P0);
        vstore(0);
        __syncthreads();
    }
    // steady tiles t = 1 .. NT-2: no conditionals in the body, so each step's
    // QK / SM / PV streams form one basic block the scheduler can interleave
    for (int t = 1; t < NT - 1; ++t) {
        const char* slot = smem + (t & 1) * SLOT;
        // step 2t: QK(2t) | SM(2t-1) | PV(2t-2)
        kload(t + 1);
        qk(S0, slot, koff0);
        smx(S1, P1);
        pv(P0, slot, 0);
        finish(S1, P1);
        kstore(t + 1);
        // step 2t+1: QK(2t+1) | SM(2t) | PV(2t-1)
        vload(t);
        qk(S1, slot, koff1);
        smx(S0, P0);
        pv(P1, slot, 1);
        finish(S0, P0);
        vstore(t);
        __syncthreads();
    }
    if (NT > 1) {   // last tile t = NT-1: no K(t+1); its first half may be ragged
        const int t = NT - 1;
        const char* slot = smem + (t & 1) * SLOT;
        qk(S0, slot, koff0);
        smx(S1, P1);
        pv(P0, slot, 0);
        finish(S1, P1);
        vload(t);
        qk(S1, slot, koff1);
        mask(S0, 2 * t);
        smx(S0, P0);
        pv(P1, slot, 1);
        finish(S0, P0);
        vstore(t);
        __syncthreads();
    }
    {   // drain: step 2NT: SM(2NT-1) | PV(2NT-2); step 2NT+1: PV(2NT-1)
        const char* slot = smem + (NT & 1) * SLOT;
        mask(S1, 2 * NT - 1);
        smx(S1, P1);
        pv(P0, slot, 0);
        finish(S1, P1);
        pv(P1, slot, 1);
    }

#pragma unroll
    for (int u = 0; u < QB; ++u) {
        const int qi = qiv[u];
        const float lt = swap_halves_sum(l_run[u]);
        const float inv = 1.0f / lt;
        if (qi < N) {
            T* Ob = (T*)p.O + (int64_t)b * N * dv;
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb)
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

// --------------------------------------------------------------------------
// 8-wave kernel with a staggered second half and a speculative softmax.
//
// The 8-wave kernel (fa_fwd.hip dense_fwd_tiled) runs both waves of a SIMD in
// lockstep: they pass each tile's barrier together, so they run QKᵀ together
// (matrix pipe busy, vector pipe idle), then the softmax together, then PV.
// Here waves 4-7 (the second wave of every SIMD) run half an iteration behind:
//
//     waves 0-3, iteration j:   QKᵀ(j) + softmax(j)  |  PV(j)
//     waves 4-7, iteration j:   PV(j-1)              |  QKᵀ(j) + softmax(j)
//
// so while one wave of a SIMD is in its vector-heavy softmax the other is in
// matrix work.  PV(j-1) of the late waves reads tile j-1 after the early waves
// have started on tile j, so the LDS ring has three slots (tile t in slot t%3).
//
// Speculative softmax: P(j) is exponentiated against the current m_used while
// the tile max is reduced alongside (the two chains are independent); only if
// a row's max exceeds m_used by more than the threshold (rare, wave-uniform)
// is the tile recomputed against the new max, with l and O — which hold tiles
// < j only — rescaled once (cdna guide T13 hazard rule).  The max-then-exp
// serialisation of the textbook order is gone from the common path.
// --------------------------------------------------------------------------
template <class T, int D, int DV, int NQB, bool STAG, bool SPEC>
__global__ __launch_bounds__(512, 1) void dense_fwd_stag(FwdParams p) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int NW = 8, BN = 64, NKB = 2;
    constexpr int NTH = 64 * NW;
    constexpr int BM = 32 * NW * NQB;           // query rows per workgroup
    constexpr int KROW = BN * 2;                // K image row (bytes)
    constexpr int VROW = BN * 2 + 16;           // V image row (bytes), padded
    constexpr int KBYTES = D * KROW, VBYTES = DV * VROW, STAGE = KBYTES + VBYTES;
    constexpr int NSLOT = STAG ? 3 : 2;
    constexpr int CPR = BN / 8;
    constexpr int KTOT = D * CPR, VTOT = DV * CPR;
    constexpr int KCH = (KTOT + NTH - 1) / NTH;
    constexpr int VCH = (VTOT + NTH - 1) / NTH;
    static_assert(KTOT % NTH == 0 || KTOT < NTH, "tile split");
    static_assert(VTOT % NTH == 0 || VTOT < NTH, "tile split");
    __shared__ __attribute__((aligned(16))) char smem[NSLOT * STAGE + 16];   // +16: dump slot

    auto kswz = [](int f) { return ((f >> 1) & 1) << 1; };

    const int lid = xcd_remap(blockIdx.x, p.total_wg);
    const int b = lid / p.nqb;
    const int qb = lid - b * p.nqb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int N = p.N, Nk = p.Nk, d = p.d, dv = p.dv;
    const auto qrs = slab_rsrc((const T*)p.Q + (int64_t)b * N * d, (uint32_t)(N * d * (int)sizeof(T)));
    const int ldk = p.ldk;
    const auto krs = slab_rsrc((const T*)p.K + (int64_t)b * ldk * d, (uint32_t)(ldk * d * (int)sizeof(T)));
    const auto vrs = slab_rsrc((const T*)p.V + (int64_t)b * ldk * dv, (uint32_t)(ldk * dv * (int)sizeof(T)));
    const bool late = STAG && __builtin_amdgcn_readfirstlane(wave) >= 4;

    int qiv[NQB];
    F8 qf[NQB][D / 16];
#pragma unroll
    for (int u = 0; u < NQB; ++u) {
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
    const bool kact = KTOT >= NTH || tid < KTOT, vact = VTOT >= NTH || tid < VTOT;
#pragma unroll
    for (int it = 0; it < KCH; ++it) {
        const int ch = tid + NTH * it, f = ch / CPR, pc = ch % CPR;
        kgo[it] = kact ? (f * ldk + pc * 8) * 2 : 0x7FFFFFF0;
        kso[it] = kact ? f * KROW + (((pc >> 1) ^ kswz(f)) * 32) + (pc & 1) * 16 : NSLOT * STAGE;
    }
#pragma unroll
    for (int it = 0; it < VCH; ++it) {
        const int ch = tid + NTH * it, f = ch / CPR, pc = ch % CPR;
        vgo[it] = vact ? (f * ldk + pc * 8) * 2 : 0x7FFFFFF0;
        vso[it] = vact ? f * VROW + pc * 16 : NSLOT * STAGE - KBYTES;
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
    auto lstore = [&](char* buf, int j, auto) {
        if (ragged && j == NT - 1) {
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

    F8 pf[NQB][NKB][2];
    // Sᵀ(j) = K(j)·Qᵀ (keys past Nk: -inf)
    auto scores = [&](f32x16 (&sacc)[NQB][NKB], const char* klds, int j, auto maskc) {
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
#pragma unroll
            for (int s = 0; s < D / 16; ++s) {
                const char* a = klds + koff[kb] + 16 * s * KROW;
                const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(a));
                const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(a + 4 * KROW));
                const F8 af = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
                for (int u = 0; u < NQB; ++u)
                    sacc[u][kb] = (s == 0) ? mfma32x32x16(af, qf[u][s], f32x16{}) : mfma32x32x16(af, qf[u][s], sacc[u][kb]);
            }
        }
        if (decltype(maskc)::value && ragged) {
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
    };
    // QKᵀ(j) + speculative softmax -> pf.  P(j) is exponentiated against the
    // current m_used while the tile max is reduced alongside; if a row's max
    // exceeds m_used by more than the threshold (rare, wave-uniform), l and O
    // (tiles < j only) are rescaled and the pass is repeated against the new
    // max.  Written as a loop so that the rare path holds no second copy of
    // the scores: they are recomputed from the tile, which stays in its LDS
    // slot for the whole iteration.
    auto qksm = [&](const char* klds, int j, auto maskc) {
        float ps[NQB][4];
        bool again;
        do {
            // re-read the tile on a repeat (no CSE of the LDS reads across passes)
            asm volatile("" ::: "memory");
            float mt[NQB];
            {
                f32x16 sacc[NQB][NKB];
                scores(sacc, klds, j, maskc);
#pragma unroll
                for (int u = 0; u < NQB; ++u) {
                    const float mc = m_used[u] * c;
                    mt[u] = lane_max<NKB>(sacc[u]);
#pragma unroll
                    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                        for (int x = 0; x < 16; ++x) {
                            const float pv = exp2_fast(fmaf(sacc[u][kb][x], c, -mc));
                            if (kb == 0 && x < 4) ps[u][x] = pv; else ps[u][x & 3] += pv;
                            pf[u][kb][x >> 3][x & 7] = (T)pv;
                        }
                }
            }
            // keep the speculative P and sums ahead of the branch (else the
            // compiler sinks them below it, behind the max chain again)
#pragma unroll
            for (int u = 0; u < NQB; ++u)
#pragma unroll
                for (int kb = 0; kb < NKB; ++kb)
                    asm volatile("" : "+v"(pf[u][kb][0]), "+v"(pf[u][kb][1]));
#pragma unroll
            for (int u = 0; u < NQB; ++u) asm volatile("" : "+v"(ps[u][0]), "+v"(ps[u][1]), "+v"(ps[u][2]), "+v"(ps[u][3]));
            bool need = false;
#pragma unroll
            for (int u = 0; u < NQB; ++u) {
                mt[u] = swap_halves_max(mt[u]);
                m_true[u] = vmax(m_true[u], mt[u]);
                need |= mt[u] > m_used[u] + thr_raw;
            }
            again = __builtin_amdgcn_ballot_w64(need) != 0;
            if (again) {
#pragma unroll
                for (int u = 0; u < NQB; ++u) {
                    const float m_new = fmaxf(m_used[u], mt[u]);
                    const float alpha = exp2_fast((m_used[u] - m_new) * c);
                    m_used[u] = m_new;
                    l_run[u] *= alpha;
#pragma unroll
                    for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                        for (int x = 0; x < 16; ++x) oacc[u][cb][x] *= alpha;
                }
            }
        } while (again);
#pragma unroll
        for (int u = 0; u < NQB; ++u) l_run[u] += (ps[u][0] + ps[u][1]) + (ps[u][2] + ps[u][3]);
    };
    // textbook order (SPEC = false): tile max first, rescale decision, then P
    auto qksm_tb = [&](const char* klds, int j, auto maskc) {
        f32x16 sacc[NQB][NKB];
        scores(sacc, klds, j, maskc);
#pragma unroll
        for (int u = 0; u < NQB; ++u) {
            const float mt = swap_halves_max(lane_max<NKB>(sacc[u]));
            m_true[u] = vmax(m_true[u], mt);
            if (__builtin_amdgcn_ballot_w64(mt > m_used[u] + thr_raw) != 0) {
                const float m_new = fmaxf(m_used[u], mt);
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
                    const float pv = exp2_fast(fmaf(sacc[u][kb][x], c, -mc));
                    if (kb == 0 && x < 4) ps[x] = pv; else ps[x & 3] += pv;
                    pf[u][kb][x >> 3][x & 7] = (T)pv;
                }
            l_run[u] += (ps[0] + ps[1]) + (ps[2] + ps[3]);
        }
    };
    auto pvm = [&](const char* vlds) {
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

    // Both halves run the same instruction stream  QKᵀ+softmax(j), PV(j), ...;
    // only their barrier moves: waves 0-3 pass barrier j after PV(j), waves
    // 4-7 right after QKᵀ+softmax(j).  Between barriers j and j+1 the early
    // half then runs QKᵀ+softmax(j+1), PV(j+1) while the late half runs PV(j),
    // QKᵀ+softmax(j+1): the two waves of a SIMD are half an iteration apart.
    // Tile j+1 is written (slot (j+1)%3, which held tile j-2, last read by the
    // late half's PV(j-2) before barrier j-1) right before each wave's barrier j.
    int cur = 0;
    auto nxt = [&](int s_) { return s_ + 1 == NSLOT ? 0 : s_ + 1; };
    gload(0);
    lstore(smem, 0, std::true_type{});
    __syncthreads();
    // the last tile (masked keys, zeroed V rows) is peeled: the loop body
    // carries no per-tile mask selects
    auto iter = [&](int j, auto maskc) {
        const int n1 = nxt(cur);
        gload(min(j + 1, NT - 1));
        char* cs = smem + cur * STAGE;
        if constexpr (SPEC) qksm(cs, j, maskc); else qksm_tb(cs, j, maskc);
        if (late) {
            lstore(smem + n1 * STAGE, min(j + 1, NT - 1), maskc);
            __syncthreads();
        }
        pvm(cs + KBYTES);
        if (!late) {
            lstore(smem + n1 * STAGE, min(j + 1, NT - 1), maskc);
            __syncthreads();
        }
        cur = n1;
    };
    for (int j = 0; j < NT - 1; ++j) iter(j, std::false_type{});
    iter(NT - 1, std::true_type{});

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

template <class T, int D, int NQB, bool STAG, bool SPEC>
static hipError_t launch_stag_dv(const FwdParams& p0, int DVc, hipStream_t s) {
    FwdParams q = p0;
    const int rows = 32 * 8 * NQB;
    q.nqb = (q.N + rows - 1) / rows;
    q.total_wg = q.nqb * q.batch;
    const dim3 g((unsigned)q.total_wg), blk(512);
    switch (DVc) {
        case 32: hipLaunchKernelGGL((dense_fwd_stag<T, D, 32, NQB, STAG, SPEC>), g, blk, 0, s, q); break;
        case 64: hipLaunchKernelGGL((dense_fwd_stag<T, D, 64, NQB, STAG, SPEC>), g, blk, 0, s, q); break;
        case 128:
            if constexpr (NQB == 1) { hipLaunchKernelGGL((dense_fwd_stag<T, D, 128, 1, STAG, SPEC>), g, blk, 0, s, q); break; }
            return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// variant 11: speculative softmax, lockstep; 12: speculative + staggered;
// 13: textbook softmax + staggered.  Geometry as the default (d, dv <= 64:
// 2 query blocks per wave; else 1).
template <class T, bool STAG, bool SPEC>
static hipError_t launch_stag_typed(const FwdParams& p, int Dc, int DVc, hipStream_t s) {
    const bool q2 = Dc <= 64 && DVc <= 64;
    switch (Dc) {
        case 32: return q2 ? launch_stag_dv<T, 32, 2, STAG, SPEC>(p, DVc, s) : launch_stag_dv<T, 32, 1, STAG, SPEC>(p, DVc, s);
        case 64: return q2 ? launch_stag_dv<T, 64, 2, STAG, SPEC>(p, DVc, s) : launch_stag_dv<T, 64, 1, STAG, SPEC>(p, DVc, s);
        case 128: return launch_stag_dv<T, 128, 1, STAG, SPEC>(p, DVc, s);
    }
    return hipErrorInvalidValue;
}

template <class T>
static hipError_t launch_stag_v(const FwdParams& p, int Dc, int DVc, int variant, hipStream_t s) {
    switch (variant) {
        case 11: return launch_stag_typed<T, false, true>(p, Dc, DVc, s);
        case 12: return launch_stag_typed<T, true, true>(p, Dc, DVc, s);
        default: return launch_stag_typed<T, true, false>(p, Dc, DVc, s);
    }
}

hipError_t launch_fwd_stag(const FwdParams& p, int dtype, int Dc, int DVc, int variant, hipStream_t s) {
    return dtype == FA_DTYPE_F16 ? launch_stag_v<f16>(p, Dc, DVc, variant, s) : launch_stag_v<bf16>(p, Dc, DVc, variant, s);
}

template <class T, int D>
static hipError_t launch_pipe_dv(const FwdParams& p0, int DVc, hipStream_t s) {
    FwdParams q = p0;
    q.nqb = (q.N + 255) / 256;
    q.total_wg = q.nqb * q.batch;
    const dim3 g((unsigned)q.total_wg), blk(256);
    switch (DVc) {
        case 32: hipLaunchKernelGGL((dense_fwd_pipe<T, D, 32>), g, blk, 0, s, q); break;
        case 64: hipLaunchKernelGGL((dense_fwd_pipe<T, D, 64>), g, blk, 0, s, q); break;
        case 128: hipLaunchKernelGGL((dense_fwd_pipe<T, D, 128>), g, blk, 0, s, q); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <class T>
static hipError_t launch_pipe_typed(const FwdParams& p, int Dc, int DVc, hipStream_t s) {
    switch (Dc) {
        case 32: return launch_pipe_dv<T, 32>(p, DVc, s);
        case 64: return launch_pipe_dv<T, 64>(p, DVc, s);
        case 128: return launch_pipe_dv<T, 128>(p, DVc, s);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_fwd_pipe(const FwdParams& p, int dtype, int Dc, int DVc, hipStream_t s) {
    if ((int64_t)p.total_wg > INT32_MAX) return hipErrorInvalidValue;
    return dtype == FA_DTYPE_F16 ? launch_pipe_typed<f16>(p, Dc, DVc, s) : launch_pipe_typed<bf16>(p, Dc, DVc, s);
}

}  // namespace fa
