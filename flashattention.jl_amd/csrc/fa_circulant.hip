// fa_circulant.hip — circulant (periodic banded) flash attention for gfx950.
//
// Replaces circulant_fa!(O, l, m, Q, K, V, W) (reference src/circulant.jl:9-118;
// naive form circulant_dpa! src/naive/circulant.jl:8-36).  Query i (0-based)
// attends the W band entries key(i, t) = (i − p + t) mod N, t = 0..W−1,
// p = (W−1) ÷ 2 — the set cartesian_circulant (src/utils.jl:6-17) enumerates
// for column i+1 (its circshift only re-orders the band so that the sparse
// matrix's row indices come out sorted).  W > N repeats keys, each band entry
// counting once, as in the reference loops.  O, l, m as in dense_fa!:
// m = τ·max over the band, l = Σ exp(τ s − m), O = softmax(τ s)·V.
//
// The reference wrapper circulant_fa(Q, K, V, W) (src/circulant.jl:1-7) calls
// circulant_fa! without W and allocates O like Q (breaks for dv ≠ d); the C ABI
// takes W and dv explicitly.
//
// Kernels:
//  * circ_fwd_tiled (bf16/fp16, N % 8 == 0, 16-B aligned K/V): a workgroup of
//    4 waves owns 128 consecutive queries; the union of their bands is
//    BM + W − 1 consecutive circular key positions (start rounded down to a
//    16-B chunk).  That union streams through the same double-buffered,
//    swizzled LDS images and MFMA fragments as the dense forward (fa_fwd.hip):
//    Sᵀ = K·Qᵀ, P from registers, Oᵀ += Vᵀ·Pᵀ.  Each wave computes only the
//    64-key tiles that intersect its own 32 bands and masks per element
//    (0 <= u − r − off < W) only on tiles that are not inside every band.
//    Roofline: HBM for W below ≈600 (intensity ≈ W/2 FLOP/B).
//  * circ_fwd_simt (every dtype incl. fp32, any N / alignment): one thread per
//    query, LDS-tiled key union, exact fp32 arithmetic (below).
//  * circ_fwd_generic: one wave per query, lanes over features — kept only as a
//    reference path behind fa_debug_set_circ_generic.
#include <type_traits>

#include "fa_common.h"
#include "fa_internal.h"
#include "../../include/fa_hip.h"

namespace fa {

thread_local int g_circ_force_generic = 0;   // debug knob: 1 = one-wave-per-query kernel, 2 = LDS-tiled SIMT kernel (non-MFMA shapes)

struct CircParams {
    const void* Q;
    const void* K;
    const void* V;
    void* O;
    float* l;
    float* m;
    int N, d, dv, W, p;
    int nqb, total_wg;
    float scale, scale_log2;
};

// --------------------------------------------------------------------------
// generic: one wave per (query, slab); lanes own features f = lane, lane + 64
// --------------------------------------------------------------------------
template <class T>
__global__ __launch_bounds__(256) void circ_fwd_generic(CircParams P) {
    const int lane = threadIdx.x & 63;
    const int64_t gq = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int N = P.N, d = P.d, dv = P.dv, W = P.W;
    if (gq >= (int64_t)N * P.total_wg) return;   // total_wg carries the batch here
    const int b = (int)(gq / N), i = (int)(gq - (int64_t)b * N);
    const T* Q = (const T*)P.Q + (int64_t)b * N * d;
    const T* K = (const T*)P.K + (int64_t)b * N * d;
    const T* V = (const T*)P.V + (int64_t)b * N * dv;
    float qv[2], acc[2] = {0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int f = lane + 64 * u;
        qv[u] = f < d ? (float)Q[(int64_t)f * N + i] : 0.f;
    }
    const float c = P.scale_log2;
    float m = kNegInf, l = 0.f;
    int key = ((i - P.p) % N + N) % N;
    for (int t = 0; t < W; ++t) {
        float s = 0.f;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int f = lane + 64 * u;
            if (f < d) s = fmaf(qv[u], (float)K[(int64_t)f * N + key], s);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
        const float mn = fmaxf(m, s);
        const float a = exp2_fast((m - mn) * c);          // m = −inf first: exp2(−inf) = 0
        const float pr = exp2_fast((s - mn) * c);
        l = l * a + pr;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int cc = lane + 64 * u;
            acc[u] = acc[u] * a + (cc < dv ? pr * (float)V[(int64_t)cc * N + key] : 0.f);
        }
        m = mn;
        key = key + 1 == N ? 0 : key + 1;
    }
    T* O = (T*)P.O + (int64_t)b * N * dv;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int cc = lane + 64 * u;
        if (cc < dv) O[(int64_t)cc * N + i] = (T)(acc[u] / l);
    }
    if (lane == 0) {
        P.m[(int64_t)b * N + i] = m * P.scale;
        P.l[(int64_t)b * N + i] = l;
    }
}

// Float64 (the reference's test element type): the same one-wave-per-query sweep
// in double, exact online softmax (no lazy rescale), τ resolved in double.
__global__ __launch_bounds__(256) void circ_fwd_f64(CircParams P, double scale, int64_t batch) {
    const int lane = threadIdx.x & 63;
    const int64_t gq = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int N = P.N, d = P.d, dv = P.dv, W = P.W;
    if (gq >= (int64_t)N * batch) return;
    const int b = (int)(gq / N), i = (int)(gq - (int64_t)b * N);
    const double* Q = (const double*)P.Q + (int64_t)b * N * d;
    const double* K = (const double*)P.K + (int64_t)b * N * d;
    const double* V = (const double*)P.V + (int64_t)b * N * dv;
    double qv[2], acc[2] = {0.0, 0.0};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int f = lane + 64 * u;
        qv[u] = f < d ? Q[(int64_t)f * N + i] : 0.0;
    }
    double m = -__builtin_huge_val(), l = 0.0;
    int key = ((i - P.p) % N + N) % N;
    for (int t = 0; t < W; ++t) {
        double s = 0.0;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int f = lane + 64 * u;
            if (f < d) s = fma(qv[u], K[(int64_t)f * N + key], s);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
        s *= scale;
        const double mn = __builtin_elementwise_maximum(m, s);
        const double a = exp(m - mn);   // m = −inf first: exp(−inf) = 0
        const double pr = exp(s - mn);
        l = l * a + pr;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int cc = lane + 64 * u;
            acc[u] = acc[u] * a + (cc < dv ? pr * V[(int64_t)cc * N + key] : 0.0);
        }
        m = mn;
        key = key + 1 == N ? 0 : key + 1;
    }
    double* O = (double*)P.O + (int64_t)b * N * dv;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int cc = lane + 64 * u;
        if (cc < dv) O[(int64_t)cc * N + i] = acc[u] / l;
    }
    if (lane == 0) {
        P.m[(int64_t)b * N + i] = (float)m;
        P.l[(int64_t)b * N + i] = (float)l;
    }
}

// --------------------------------------------------------------------------
// LDS-tiled SIMT kernel (every dtype incl. fp32, any N / alignment): one thread
// per query, 256 consecutive queries per workgroup.  The union of their bands,
// 256 + W − 1 consecutive circular key positions, streams through LDS in tiles
// of KT keys stored [key][feature] (fp32, rows padded by 4 floats: the per-lane
// float4 reads of different keys hit distinct banks).  Each lane scores its
// in-band keys (exact fp32 dot products) with the lazy online rescale of the
// MFMA kernels (threshold 2^8) and accumulates O in registers.  Tiles outside a
// wave's band union are skipped.
// Replaces one-wave-per-query: ragged N (16383) 35.7 ms -> ~1 ms, fp32 likewise.
// --------------------------------------------------------------------------
template <class T, int D, int DV, int KT>
__global__ __launch_bounds__(256) void circ_fwd_simt(CircParams P) {
    constexpr int DR = D + 4, VR = DV + 4;
    __shared__ __attribute__((aligned(16))) float sk[KT * DR], sv[KT * VR];
    const int N = P.N, d = P.d, dv = P.dv, W = P.W;
    const int nq = (N + 255) / 256;
    const int lid = xcd_remap(blockIdx.x, P.total_wg);
    const int b = lid / nq, q0 = (lid - b * nq) * 256;
    const int tid = threadIdx.x, r = tid, i = q0 + tid;
    const T* Qb = (const T*)P.Q + (int64_t)b * N * d;
    const T* Kb = (const T*)P.K + (int64_t)b * N * d;
    const T* Vb = (const T*)P.V + (int64_t)b * N * dv;
    float qv[D], o[DV];
#pragma unroll
    for (int f = 0; f < D; ++f) qv[f] = (i < N && f < d) ? (float)Qb[(int64_t)f * N + i] : 0.0f;
#pragma unroll
    for (int f = 0; f < DV; ++f) o[f] = 0.0f;
    const float c = P.scale_log2;
    const float thr_raw = kRescaleLog2 / c;
    float m_used = kNegInf, m_true = kNegInf, l = 0.0f;
    const int U = 256 + W - 1;
    const int ntile = (U + KT - 1) / KT;
    const int base = ((q0 - P.p) % N + N) % N;        // union position u <-> key (base + u) mod N
    const int w0 = tid & ~63;                          // this wave's band union: u in [w0, w0 + 63 + W - 1]
    for (int tt = 0; tt < ntile; ++tt) {
        const int u0 = tt * KT;
        __syncthreads();
        // stage KT keys x features (consecutive threads -> consecutive keys: coalesced)
        for (int e = tid; e < KT * D; e += 256) {
            const int kk = e % KT, f = e / KT;
            const int key = (int)(((int64_t)base + u0 + kk) % N);
            sk[kk * DR + f] = f < d ? (float)Kb[(int64_t)f * N + key] : 0.0f;
        }
        for (int e = tid; e < KT * DV; e += 256) {
            const int kk = e % KT, f = e / KT;
            const int key = (int)(((int64_t)base + u0 + kk) % N);
            sv[kk * VR + f] = f < dv ? (float)Vb[(int64_t)f * N + key] : 0.0f;
        }
        __syncthreads();
        if (u0 + KT <= w0 || u0 > w0 + 63 + W - 1) continue;   // wave-uniform
#pragma unroll 2
        for (int kk = 0; kk < KT; ++kk) {
            const int u = u0 + kk;
            if (u < r || u >= r + W) continue;
            const float4* kr = (const float4*)(sk + kk * DR);
            float a0 = 0.0f, a1 = 0.0f;
#pragma unroll
            for (int f4 = 0; f4 < D / 4; ++f4) {
                const float4 kv = kr[f4];
                a0 = fmaf(qv[4 * f4], kv.x, a0);
                a1 = fmaf(qv[4 * f4 + 1], kv.y, a1);
                a0 = fmaf(qv[4 * f4 + 2], kv.z, a0);
                a1 = fmaf(qv[4 * f4 + 3], kv.w, a1);
            }
            const float sc = a0 + a1;
            m_true = vmax(m_true, sc);
            if (sc > m_used + thr_raw) {               // lazy rescale (rare; always on the first key)
                const float a = exp2_fast((m_used - sc) * c);
                l *= a;
#pragma unroll
                for (int f = 0; f < DV; ++f) o[f] *= a;
                m_used = sc;
            }
            const float pr = exp2_fast((sc - m_used) * c);
            l += pr;
            const float4* vr = (const float4*)(sv + kk * VR);
#pragma unroll
            for (int f4 = 0; f4 < DV / 4; ++f4) {
                const float4 vv = vr[f4];
                o[4 * f4] = fmaf(pr, vv.x, o[4 * f4]);
                o[4 * f4 + 1] = fmaf(pr, vv.y, o[4 * f4 + 1]);
                o[4 * f4 + 2] = fmaf(pr, vv.z, o[4 * f4 + 2]);
                o[4 * f4 + 3] = fmaf(pr, vv.w, o[4 * f4 + 3]);
            }
        }
    }
    // l, O are relative to 2^(c·m_used); the returned l is relative to the exact max
    l *= exp2_fast((m_used - m_true) * c);
    const float osc = exp2_fast((m_used - m_true) * c);
#pragma unroll
    for (int f = 0; f < DV; ++f) o[f] *= osc;
    const float m = m_true;
    if (i < N) {
        T* Ob = (T*)P.O + (int64_t)b * N * dv;
        const float inv = 1.0f / l;
#pragma unroll
        for (int f = 0; f < DV; ++f)
            if (f < dv) Ob[(int64_t)f * N + i] = (T)(o[f] * inv);
        P.m[(int64_t)b * N + i] = m * P.scale;
        P.l[(int64_t)b * N + i] = l;
    }
}

// --------------------------------------------------------------------------
// tiled MFMA kernel (bf16 / fp16)
// --------------------------------------------------------------------------
template <class T, int D, int DV>
__global__ __launch_bounds__(256, 2) void circ_fwd_tiled(CircParams P) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int NTH = 256, BM = 128, BN = 64, NKB = 2;   // 4 waves x 32 queries
    constexpr int KROW = BN * 2, VROW = BN * 2 + 16;
    constexpr int KBYTES = D * KROW, VBYTES = DV * VROW, STAGE = KBYTES + VBYTES;
    constexpr int CPR = BN / 8;
    constexpr int KTOT = D * CPR, VTOT = DV * CPR;
    constexpr int KCH = (KTOT + NTH - 1) / NTH, VCH = (VTOT + NTH - 1) / NTH;
    static_assert(KTOT % NTH == 0 || KTOT < NTH, "tile split");
    static_assert(VTOT % NTH == 0 || VTOT < NTH, "tile split");
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 16];
    auto kswz = [](int f) { return ((f >> 1) & 1) << 1; };

    const int lid = xcd_remap(blockIdx.x, P.total_wg);
    const int b = lid / P.nqb;
    const int qb = lid - b * P.nqb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int N = P.N, d = P.d, dv = P.dv, W = P.W;
    const auto qrs = slab_rsrc((const T*)P.Q + (int64_t)b * N * d, (uint32_t)(N * d * (int)sizeof(T)));
    const auto krs = slab_rsrc((const T*)P.K + (int64_t)b * N * d, (uint32_t)(N * d * (int)sizeof(T)));
    const auto vrs = slab_rsrc((const T*)P.V + (int64_t)b * N * dv, (uint32_t)(N * dv * (int)sizeof(T)));

    // union of the workgroup's bands: positions u = 0..U-1 <-> keys (k0 + u) mod N
    const int q0 = qb * BM;
    const int s0 = ((q0 - P.p) % N + N) % N;
    const int k0 = s0 & ~7, off = s0 - k0;
    const int NT = (BM + off + W - 1 + BN - 1) / BN;
    // this wave's queries r' = 32·wave + r attend u in [r' + off, r' + off + W − 1]
    const int tlo = (32 * wave + off) / BN;
    const int thi = min(NT - 1, (32 * wave + 31 + off + W - 1) / BN);

    const int qi = q0 + wave * 32 + r;
    F8 qf[D / 16];
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e)
            qf[s][e] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b16(qrs, ((16 * s + 8 * h + e) * N + qi) * 2, 0, 0));

    const int g = lane >> 4, kh = g & 1, qq = (lane & 15) >> 2, pp = lane & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
    int koff[NKB];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
        koff[kb] = (8 * h + qq) * KROW + (((kb * 2 + kh) ^ kswz(qq)) * 32) + 8 * sig;
    const int voff = r * VROW + 16 * h;

    const bool kact = KTOT >= NTH || tid < KTOT, vact = VTOT >= NTH || tid < VTOT;
    int kf[KCH], kpc[KCH], kso[KCH], vf[VCH], vpc[VCH], vso[VCH];
#pragma unroll
    for (int it = 0; it < KCH; ++it) {
        const int ch = tid + NTH * it;
        kf[it] = ch / CPR; kpc[it] = ch % CPR;
        kso[it] = kact ? kf[it] * KROW + (((kpc[it] >> 1) ^ kswz(kf[it])) * 32) + (kpc[it] & 1) * 16 : 2 * STAGE;
    }
#pragma unroll
    for (int it = 0; it < VCH; ++it) {
        const int ch = tid + NTH * it;
        vf[it] = ch / CPR; vpc[it] = ch % CPR;
        vso[it] = vact ? KBYTES + vf[it] * VROW + vpc[it] * 16 : 2 * STAGE;
    }

    // two register sets: a tile's global loads are issued two iterations before
    // its LDS store, so the (latency-bound) short band loop overlaps them
    u32x4 kreg[2][KCH], vreg[2][VCH];
    auto gload = [&](int t, int set) {   // 8-key chunks never straddle N (k0 % 8 == 0, N % 8 == 0)
#pragma unroll
        for (int it = 0; it < KCH; ++it) {
            const int key = (k0 + t * BN + 8 * kpc[it]) % N;
            kreg[set][it] = __builtin_amdgcn_raw_buffer_load_b128(krs, kact ? (kf[it] * N + key) * 2 : 0x7FFFFFF0, 0, 0);
        }
#pragma unroll
        for (int it = 0; it < VCH; ++it) {
            const int key = (k0 + t * BN + 8 * vpc[it]) % N;
            vreg[set][it] = __builtin_amdgcn_raw_buffer_load_b128(vrs, vact ? (vf[it] * N + key) * 2 : 0x7FFFFFF0, 0, 0);
        }
    };
    auto lstore = [&](char* buf, int set) {
#pragma unroll
        for (int it = 0; it < KCH; ++it) *(u32x4*)((kact ? buf : smem) + kso[it]) = kreg[set][it];
#pragma unroll
        for (int it = 0; it < VCH; ++it) *(u32x4*)((vact ? buf : smem) + vso[it]) = vreg[set][it];
    };

    f32x16 oacc[DV / 32];
#pragma unroll
    for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
        for (int x = 0; x < 16; ++x) oacc[cb][x] = 0.0f;
    float m_used = kNegInf, m_true = kNegInf, l_run = 0.0f;
    const float c = P.scale_log2;
    const float thr_raw = kRescaleLog2 / c;
    const int rq = 32 * wave + r + off;   // first band position of this lane's query

    auto compute = [&](const char* klds, int t) {
        f32x16 sacc[NKB];
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
#pragma unroll
            for (int x = 0; x < 16; ++x) sacc[kb][x] = 0.0f;
#pragma unroll
            for (int s = 0; s < D / 16; ++s) {
                const char* a = klds + koff[kb] + 16 * s * KROW;
                const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(a));
                const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(a + 4 * KROW));
                sacc[kb] = mfma32x32x16(__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7), qf[s], sacc[kb]);
            }
        }
        // inside every band of the wave: [t·BN, t·BN + BN) ⊂ [32w + 31 + off, 32w + off + W − 1]
        const bool full = t * BN >= 32 * wave + 31 + off && t * BN + BN - 1 <= 32 * wave + off + W - 1;
        if (!full) {
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int x = 0; x < 16; ++x) {
                    const int kt = kb * 32 + (x & 3) + 4 * ((x >> 2) & 1) + 8 * h + 16 * (x >> 3);
                    if ((unsigned)(t * BN + kt - rq) >= (unsigned)W) sacc[kb][x] = kNegInf;
                }
        }
        const float mt = swap_halves_max(lane_max<NKB>(sacc));
        m_true = vmax(m_true, mt);
        if (__builtin_amdgcn_ballot_w64(mt > m_used + thr_raw) != 0) {
            // a band edge can leave a query without any key in this tile (mt = −inf)
            const float m_new = fmaxf(m_used, mt);
            const float alpha = m_new == kNegInf ? 1.0f : exp2_fast((m_used - m_new) * c);
            l_run *= alpha;
#pragma unroll
            for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                for (int x = 0; x < 16; ++x) oacc[cb][x] *= alpha;
            m_used = m_new;
        }
        const float mc = m_used == kNegInf ? 0.0f : m_used * c;
        F8 pf[NKB][2];
        float ps[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const float pv = exp2_fast(fmaf(sacc[kb][x], c, -mc));
                ps[x & 3] += pv;
                pf[kb][x >> 3][x & 7] = (T)pv;
            }
        l_run += (ps[0] + ps[1]) + (ps[2] + ps[3]);
        const char* vl = klds + KBYTES + voff;
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const F8 va = *(const F8*)(vl + cb * 32 * VROW + (kb * 32 + 16 * s) * 2);
                    oacc[cb] = mfma32x32x16(va, pf[kb][s], oacc[cb]);
                }
    };

    char* const buf0 = smem;
    char* const buf1 = smem + STAGE;
    // tile t: registers set t % 2 (loaded at iteration t-2), LDS buffer t % 2
    gload(0, 0);
    if (NT > 1) gload(1, 1);
    lstore(buf0, 0);
    if (NT > 2) gload(2, 0);
    __syncthreads();
    for (int t = 0; t < NT; t += 2) {
        if (t >= tlo && t <= thi) compute(buf0, t);
        if (t + 1 < NT) {
            lstore(buf1, 1);
            if (t + 3 < NT) gload(t + 3, 1);
        }
        __syncthreads();
        if (t + 1 < NT) {
            if (t + 1 >= tlo && t + 1 <= thi) compute(buf1, t + 1);
            if (t + 2 < NT) {
                lstore(buf0, 0);
                if (t + 4 < NT) gload(t + 4, 0);
            }
            __syncthreads();
        }
    }

    const float lt = swap_halves_sum(l_run);
    if (qi < N) {
        const float inv = 1.0f / lt;
        T* Ob = (T*)P.O + (int64_t)b * N * dv;
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int cc = cb * 32 + acc_row(x, h);
                if (cc < dv) Ob[(int64_t)cc * N + qi] = (T)(oacc[cb][x] * inv);
            }
        if (h == 0) {
            P.m[(int64_t)b * N + qi] = m_true * P.scale;
            P.l[(int64_t)b * N + qi] = lt * exp2_fast((m_used - m_true) * c);
        }
    }
}

// --------------------------------------------------------------------------
// launcher
// --------------------------------------------------------------------------
static bool circ_aligned16(const void* ptr) { return ((uintptr_t)ptr & 15u) == 0; }

template <class T, int D>
static void launch_circ_tiled(const CircParams& p, int DVc, hipStream_t s) {
    const dim3 grid((unsigned)p.total_wg), blk(256);
    switch (DVc) {
        case 32: hipLaunchKernelGGL((circ_fwd_tiled<T, D, 32>), grid, blk, 0, s, p); break;
        case 64: hipLaunchKernelGGL((circ_fwd_tiled<T, D, 64>), grid, blk, 0, s, p); break;
        default: hipLaunchKernelGGL((circ_fwd_tiled<T, D, 128>), grid, blk, 0, s, p); break;
    }
}

template <class T>
static void launch_circ_typed(CircParams p, int64_t batch, bool fast, hipStream_t s) {
    if constexpr (!std::is_same<T, float>::value) {
        if (fast) {
            const int Dc = head_dim_class(p.d), DVc = head_dim_class(p.dv);
            p.nqb = (p.N + 127) / 128;
            p.total_wg = (int)(p.nqb * batch);
            switch (Dc) {
                case 32: launch_circ_tiled<T, 32>(p, DVc, s); break;
                case 64: launch_circ_tiled<T, 64>(p, DVc, s); break;
                default: launch_circ_tiled<T, 128>(p, DVc, s); break;
            }
            return;
        }
    }
    // small grids (< 128 workgroups of 256 queries) keep one wave per query: more
    // parallelism there (N 4096, d 32, one slab, W 129 fp32: 72 vs 137 us)
    if (g_circ_force_generic == 1 || (g_circ_force_generic != 2 && (int64_t)(p.N + 255) / 256 * batch < 128)) {
        p.total_wg = (int)batch;   // one-wave-per-query kernel: slab count
        const int64_t waves = (int64_t)p.N * batch;
        hipLaunchKernelGGL((circ_fwd_generic<T>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, p);
        return;
    }
    p.total_wg = (int)((p.N + 255) / 256 * batch);
    const dim3 grid((unsigned)p.total_wg);
    const int Dc = head_dim_class(p.d), DVc = head_dim_class(p.dv);
#define FA_CS(DD, DVV, KTT) hipLaunchKernelGGL((circ_fwd_simt<T, DD, DVV, KTT>), grid, dim3(256), 0, s, p)
    if (Dc <= 32 && DVc <= 32) FA_CS(32, 32, 32);
    else if (Dc <= 64 && DVc <= 64) FA_CS(64, 64, 32);
    else FA_CS(128, 128, 8);
#undef FA_CS
}

int launch_circulant_fwd(const CircArgs& a, hipStream_t s, const char** why) {
    if (!head_dim_class(a.d) || !head_dim_class(a.dv)) {
        *why = "head dimension exceeds the compiled maximum (128)";
        return FA_ERR_UNSUPPORTED;
    }
    const int64_t esz = (int64_t)dtype_size(a.dtype);
    if (a.N * a.d * esz >= (int64_t)INT32_MAX || a.N * a.dv * esz >= (int64_t)INT32_MAX ||
        a.W > INT32_MAX / 2 || a.N * a.batch > (int64_t)INT32_MAX * 2) {
        *why = "per-slab extent or band width exceeds the 32-bit addressing of the kernels";
        return FA_ERR_UNSUPPORTED;
    }
    CircParams p;
    p.Q = a.Q; p.K = a.K; p.V = a.V; p.O = a.O; p.l = a.l; p.m = a.m;
    p.N = (int)a.N; p.d = (int)a.d; p.dv = (int)a.dv; p.W = (int)a.W; p.p = (int)((a.W - 1) / 2);
    p.nqb = 0; p.total_wg = 0;
    p.scale = a.scale;
    p.scale_log2 = a.scale * kLog2e;
    const bool fast = (a.dtype == FA_DTYPE_BF16 || a.dtype == FA_DTYPE_F16) && a.N % 8 == 0 && circ_aligned16(a.K) && circ_aligned16(a.V) &&
                      ((a.N + 127) / 128) * a.batch <= INT32_MAX && g_circ_force_generic == 0;
    switch (a.dtype) {
        case FA_DTYPE_BF16: launch_circ_typed<bf16>(p, a.batch, fast, s); break;
        case FA_DTYPE_F16: launch_circ_typed<f16>(p, a.batch, fast, s); break;
        case FA_DTYPE_F32: launch_circ_typed<float>(p, a.batch, false, s); break;
        case FA_DTYPE_F64: {
            const int64_t waves = a.N * a.batch;
            hipLaunchKernelGGL(circ_fwd_f64, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, p,
                               a.scale64 > 0.0 ? a.scale64 : (double)a.scale, a.batch);
            break;
        }
        default: *why = "unknown dtype"; return FA_ERR_INVALID_ARG;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    return FA_OK;
}

}  // namespace fa
