// fa_bwd.hip — dense flash-attention backward for gfx950.
//
// Replaces dense_fa_backward(Q, K, V, O, dO, l, m) (reference
// src/dense.jl:104-167, not executable as committed — Appendix A.2; the
// executable spec is OneDFastBack, src_cpp/FlashAttention.cpp:194-252):
//   P = exp(τ Q Kᵀ − m)/l,  dV = Pᵀ dO,  dP = dO Vᵀ,  D = rowsum(dO ∘ O),
//   dS = P ∘ (dP − D),  dQ = τ dS K,  dK = τ dSᵀ Q.
//
// Structure (FA-2 style, deterministic: no float atomics):
//   1. pre-pass   : D[b][n] = Σ_c dO∘O (fp32) and lse2[b][n] = (m + ln l)·log2 e
//                   into the caller's workspace (8·N·B bytes);
//   2. dK/dV pass : each wave owns 32 keys, sweeps all query tiles; dKᵀ, dVᵀ
//                   accumulate in registers and are written once;
//   3. dQ pass    : each wave owns 32 queries, sweeps all key tiles (the
//                   forward's shape); dQᵀ accumulates in registers.
// P is recomputed from lse, so neither pass needs an online max.
//
// Two implementations: the MFMA fast path (bf16/fp16, aligned, Nk % 8 == 0,
// N % 8 == 0) and a generic LDS-tiled SIMT path (fp32, ragged or unaligned
// shapes) used for parity on every dtype.
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "fa_common.h"
#include "fa_internal.h"
#include "../../include/fa_hip.h"

namespace fa {

// bwd_fused: a poll gives up only when the whole launch has published nothing for this
// long (fa_debug_set_bwd_stall_us): a safety net, not a scheduling decision (§ bwd_fused).
// The boundary header states the same bound (tests/test_abi.py checks they agree).
constexpr int kStallUs = FA_BWD_HANDOFF_STALL_US;

// Single-pass hand-off words in the workspace (zeroed per call), in 32-bit words from
// BwdParams::flags, for `batch` slabs of NS slices and KM members:
struct FusedFlags {
    int64_t cnt;    // [2 chains][batch][NS]: members of the chain that have published slice t
    int64_t fin;    // [batch][NS]: tails of a wrapped slice's two chains that stored their sums
    int64_t serr;   // [batch]: the slab gave up (its dQ is recomputed by bwd_dq_fast)
    int64_t xcc;    // [batch][KM]: XCD of each member + 1 (L2-local hand-off)
    int64_t prog;   // [batch][KM]: each member's count of publishes (plain stores, no contention)
    int64_t garr;   // the launch's arrival count (one add per workgroup)
    int64_t words;  // (a wrapped slice left to bwd_dq_fast's combine is flagged in hdr[3])
};
__host__ __device__ inline FusedFlags fused_flags(int64_t batch, int64_t NS, int64_t KM) {
    FusedFlags f;
    f.cnt = 0;
    f.fin = 2 * batch * NS;
    f.serr = 3 * batch * NS;
    f.xcc = f.serr + batch;
    f.prog = f.xcc + batch * KM;
    f.garr = f.prog + batch * KM;
    f.words = f.garr + 1;
    return f;
}

struct BwdParams {
    const void *Q, *K, *V, *O, *dO;
    const float *l, *m;
    void *dQ, *dK, *dV;
    float* nD;     // workspace: −rowsum(dO ∘ O)          [batch][N]
    float* nlse;   // workspace: −(m + ln l)/τ (raw units) [batch][N]
    int N, Nk, d, dv, batch;
    int nblk, total_wg;          // fast path: row blocks per slab, workgroups
    float scale, scale_log2;
    double scale64 = 0.0;        // Float64 generic path: τ in double
    // single-pass kernel (bwd_fused): dQ hand-off state, all in the caller's workspace
    unsigned* flags = nullptr;   // hand-off words (FusedFlags, zeroed per call)
    unsigned* err = nullptr;     // hand-off timeout word = hdr[1] (set per call by the pre-pass)
    // workspace header (first 256 B of the aligned workspace; fa_dense_bwd_handoff_status):
    // hdr[0] = kBwdHdrMagic | plan (1 = single pass), hdr[1] = the timeout word,
    // hdr[2] = give-ups counted over every call on this workspace (never reset here),
    // hdr[3] = some chain-B tail of this call left its slice to bwd_dq_fast's combine
    unsigned* hdr = nullptr;
    unsigned hdr_plan = 0, hdr_err = 0;
    float* part = nullptr;       // [batch][2 chains][nqt][D/16 tiles][16 x 64] fp32 running dQ sums
    int nkb = 0, nqt = 0, hoff = 3, xcd = 0;   // key blocks, 64-query slices, step offset, XCD mapping
    int stall_ticks = kStallUs * 100;   // no-progress bound of a poll in s_memrealtime ticks (100 MHz)
    int nodirect = 0;                   // tests: chain-B tails store, bwd_dq_fast adds A + B (fa_debug_set_bwd_nodirect)
    int l2local = 0;  // 1: hand the running sums over in the XCD's L2 when a slab's members share one
    int ablate = 0;   // timing-only ablations (wrong dQ): 1 no waits, 2 no sum traffic, 8 no sum loads, 16 no sum stores, 32 no dS image writes
    const unsigned* guard = nullptr;           // bwd_dq_fast runs only if *guard != 0 (nullptr: always)
    const unsigned* sguard = nullptr;          // ... and then only on the slabs b with sguard[b] != 0
    const unsigned* cguard = nullptr;          // bwd_dq_fast: combine the wrapped slices bwd_fused left (*cguard != 0)
    const unsigned* fin = nullptr;             // ... those with fin[b][t] == 2
};

template <class T> __device__ __forceinline__ float to_f(T x) { return (float)x; }

constexpr unsigned kBwdHdrMagic = 0x46414200u;   // "FAB\0"
constexpr size_t kBwdHdrBytes = 256;

// The pre-pass runs first on the stream in every 16/32-bit backward: its thread 0
// (re)writes the workspace header, so the timeout word starts each call at hdr_err.
__device__ __forceinline__ void write_bwd_header(const BwdParams& p) {
    if (p.hdr) {
        p.hdr[0] = kBwdHdrMagic | p.hdr_plan;
        p.hdr[1] = p.hdr_err;
        p.hdr[3] = 0u;   // set by a chain-B tail that left its slice to the combine (read by tests)
    }
}

// --------------------------------------------------------------------------
// 1. pre-pass (HBM-bound): one thread per (b, n), coalesced along n.
// --------------------------------------------------------------------------
template <class T>
__global__ __launch_bounds__(256) void bwd_prepass(BwdParams p) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t total = (int64_t)p.N * p.batch;
    if (idx >= total) return;
    if (idx == 0) write_bwd_header(p);
    const int64_t b = idx / p.N, n = idx - b * p.N;
    const T* O = (const T*)p.O + b * (int64_t)p.N * p.dv + n;
    const T* dO = (const T*)p.dO + b * (int64_t)p.N * p.dv + n;
    float acc = 0.0f;
    for (int c = 0; c < p.dv; ++c) acc = fmaf(to_f(dO[(int64_t)c * p.N]), to_f(O[(int64_t)c * p.N]), acc);
    p.nD[idx] = -acc;
    p.nlse[idx] = -(p.m[idx] + logf(p.l[idx])) / p.scale;
}

// 16-B variant (bf16 / fp16, N % 8 == 0, O and dO 16-B aligned): a thread owns 8
// consecutive queries and keeps 16 row loads in flight; the scalar kernel above
// issues one 2-byte load pair per feature and leaves HBM half idle (88 µs at
// configs[3]).
template <class T>
__global__ __launch_bounds__(256) void bwd_prepass_v(BwdParams p) {
    constexpr int U = 8;
    const int64_t g8 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g8 >= (int64_t)p.N * p.batch / 8) return;
    if (g8 == 0) write_bwd_header(p);
    const int64_t idx = g8 * 8, b = idx / p.N, n = idx - b * p.N;
    const T* O = (const T*)p.O + b * (int64_t)p.N * p.dv + n;
    const T* dO = (const T*)p.dO + b * (int64_t)p.N * p.dv + n;
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.0f;
    auto fma8 = [&](const u32x4& a, const u32x4& c) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned wa = a[k], wc = c[k];
            acc[2 * k] = fmaf(to_f(__builtin_bit_cast(T, (unsigned short)(wa & 0xFFFFu))),
                              to_f(__builtin_bit_cast(T, (unsigned short)(wc & 0xFFFFu))), acc[2 * k]);
            acc[2 * k + 1] = fmaf(to_f(__builtin_bit_cast(T, (unsigned short)(wa >> 16))),
                                  to_f(__builtin_bit_cast(T, (unsigned short)(wc >> 16))), acc[2 * k + 1]);
        }
    };
    int c = 0;
    for (; c + U <= p.dv; c += U) {
        u32x4 ro[U], rd[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ro[u] = *(const u32x4*)(O + (int64_t)(c + u) * p.N);
            rd[u] = *(const u32x4*)(dO + (int64_t)(c + u) * p.N);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) fma8(rd[u], ro[u]);
    }
    for (; c < p.dv; ++c) fma8(*(const u32x4*)(dO + (int64_t)c * p.N), *(const u32x4*)(O + (int64_t)c * p.N));
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        p.nD[idx + k] = -acc[k];
        p.nlse[idx + k] = -(p.m[idx + k] + logf(p.l[idx + k])) / p.scale;
    }
}

// --------------------------------------------------------------------------
// 2./3. generic SIMT path.  Tiles of 32 queries x 32 keys in LDS, arithmetic in
// A: float for the 16/32-bit types, double for Float64 (whose row statistics
// nD / nlse are double too, fa_f64.hip).  LDS rows hold d + 1 (dv + 1) elements,
// so the per-key / per-query row reads of 32 lanes fall in distinct banks.
// --------------------------------------------------------------------------
constexpr int kGT = 32;          // tile edge
constexpr int kGThreads = 256;

__device__ __forceinline__ float fma_a(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ double fma_a(double a, double b, double c) { return fma(a, b, c); }
__device__ __forceinline__ float exp2_a(float x) { return exp2f(x); }
__device__ __forceinline__ double exp2_a(double x) { return exp2(x); }
template <class A> __device__ __forceinline__ A bscale(const BwdParams& p) {
    if constexpr (sizeof(A) == 8) return p.scale64; else return p.scale;
}
template <class A> __device__ __forceinline__ A bscale_log2(const BwdParams& p) {
    if constexpr (sizeof(A) == 8) return p.scale64 * 1.4426950408889634074; else return p.scale_log2;
}

// dQ: one block per (b, 32-query tile).
template <class T, class A>
__global__ __launch_bounds__(kGThreads) void bwd_generic_dq(BwdParams p) {
    extern __shared__ __attribute__((aligned(16))) char gsm_raw[];
    A* const gsm = (A*)gsm_raw;
    const int d = p.d, dv = p.dv, N = p.N, Nk = p.Nk, ld = d + 1, ldv = dv + 1;
    A* sQ = gsm;                         // [32][d+1]
    A* sdO = sQ + kGT * ld;              // [32][dv+1]
    A* sK = sdO + kGT * ldv;             // [32][d+1]
    A* sV = sK + kGT * ld;               // [32][dv+1]
    A* sdS = sV + kGT * ldv;             // [32 q][33]
    const int nqt = (N + kGT - 1) / kGT;
    const int b = blockIdx.x / nqt, q0 = (blockIdx.x % nqt) * kGT;
    const int tid = threadIdx.x;
    const T* Qb = (const T*)p.Q + (int64_t)b * N * d;
    const T* Kb = (const T*)p.K + (int64_t)b * Nk * d;
    const T* Vb = (const T*)p.V + (int64_t)b * Nk * dv;
    const T* dOb = (const T*)p.dO + (int64_t)b * N * dv;
    for (int i = tid; i < kGT * d; i += kGThreads) {
        const int q = i % kGT, f = i / kGT;
        sQ[q * ld + f] = (q0 + q < N) ? (A)Qb[(int64_t)f * N + q0 + q] : (A)0;
    }
    for (int i = tid; i < kGT * dv; i += kGThreads) {
        const int q = i % kGT, f = i / kGT;
        sdO[q * ldv + f] = (q0 + q < N) ? (A)dOb[(int64_t)f * N + q0 + q] : (A)0;
    }
    // each thread owns dQ entries (q, f) = (i % 32, i / 32) for i = tid + 256·t
    constexpr int kMaxPer = 128 * kGT / kGThreads;   // d <= 128
    A acc[kMaxPer];
#pragma unroll
    for (int t = 0; t < kMaxPer; ++t) acc[t] = (A)0;
    const A* nD = (const A*)p.nD + (int64_t)b * N;
    const A* nL = (const A*)p.nlse + (int64_t)b * N;
    const A sl2 = bscale_log2<A>(p);
    for (int k0 = 0; k0 < Nk; k0 += kGT) {
        __syncthreads();
        for (int i = tid; i < kGT * d; i += kGThreads) {
            const int k = i % kGT, f = i / kGT;
            sK[k * ld + f] = (k0 + k < Nk) ? (A)Kb[(int64_t)f * Nk + k0 + k] : (A)0;
        }
        for (int i = tid; i < kGT * dv; i += kGThreads) {
            const int k = i % kGT, f = i / kGT;
            sV[k * ldv + f] = (k0 + k < Nk) ? (A)Vb[(int64_t)f * Nk + k0 + k] : (A)0;
        }
        __syncthreads();
        for (int e = tid; e < kGT * kGT; e += kGThreads) {
            const int q = e / kGT, k = e % kGT;
            A ds = (A)0;
            if (q0 + q < N && k0 + k < Nk) {
                A s = (A)0, dp = (A)0;
                for (int f = 0; f < d; ++f) s = fma_a(sQ[q * ld + f], sK[k * ld + f], s);
                for (int f = 0; f < dv; ++f) dp = fma_a(sdO[q * ldv + f], sV[k * ldv + f], dp);
                const A pr = exp2_a((s + nL[q0 + q]) * sl2);
                ds = pr * (dp + nD[q0 + q]);
            }
            sdS[q * (kGT + 1) + k] = ds;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < kMaxPer; ++t) {
            const int i = tid + kGThreads * t, q = i % kGT, f = i / kGT;
            if (f < d) {
                A a = acc[t];
                for (int k = 0; k < kGT; ++k) a = fma_a(sdS[q * (kGT + 1) + k], sK[k * ld + f], a);
                acc[t] = a;
            }
        }
    }
    T* dQb = (T*)p.dQ + (int64_t)b * N * d;
    const A sc = bscale<A>(p);
#pragma unroll
    for (int t = 0; t < kMaxPer; ++t) {
        const int i = tid + kGThreads * t, q = i % kGT, f = i / kGT;
        if (f < d && q0 + q < N) dQb[(int64_t)f * N + q0 + q] = (T)(acc[t] * sc);
    }
}

// dK, dV: one block per (b, 32-key tile).
template <class T, class A>
__global__ __launch_bounds__(kGThreads) void bwd_generic_dkdv(BwdParams p) {
    extern __shared__ __attribute__((aligned(16))) char gsm_raw[];
    A* const gsm = (A*)gsm_raw;
    const int d = p.d, dv = p.dv, N = p.N, Nk = p.Nk, ld = d + 1, ldv = dv + 1;
    A* sK = gsm;                         // [32][d+1]
    A* sV = sK + kGT * ld;               // [32][dv+1]
    A* sQ = sV + kGT * ldv;              // [32][d+1]
    A* sdO = sQ + kGT * ld;              // [32][dv+1]
    A* sP = sdO + kGT * ldv;             // [32 q][33]
    A* sdS = sP + kGT * (kGT + 1);       // [32 q][33]
    const int nkt = (Nk + kGT - 1) / kGT;
    const int b = blockIdx.x / nkt, k0 = (blockIdx.x % nkt) * kGT;
    const int tid = threadIdx.x;
    const T* Qb = (const T*)p.Q + (int64_t)b * N * d;
    const T* Kb = (const T*)p.K + (int64_t)b * Nk * d;
    const T* Vb = (const T*)p.V + (int64_t)b * Nk * dv;
    const T* dOb = (const T*)p.dO + (int64_t)b * N * dv;
    for (int i = tid; i < kGT * d; i += kGThreads) {
        const int k = i % kGT, f = i / kGT;
        sK[k * ld + f] = (k0 + k < Nk) ? (A)Kb[(int64_t)f * Nk + k0 + k] : (A)0;
    }
    for (int i = tid; i < kGT * dv; i += kGThreads) {
        const int k = i % kGT, f = i / kGT;
        sV[k * ldv + f] = (k0 + k < Nk) ? (A)Vb[(int64_t)f * Nk + k0 + k] : (A)0;
    }
    constexpr int kMaxPer = 128 * kGT / kGThreads;
    A accK[kMaxPer], accV[kMaxPer];
#pragma unroll
    for (int t = 0; t < kMaxPer; ++t) { accK[t] = (A)0; accV[t] = (A)0; }
    const A* nD = (const A*)p.nD + (int64_t)b * N;
    const A* nL = (const A*)p.nlse + (int64_t)b * N;
    const A sl2 = bscale_log2<A>(p);
    for (int q0 = 0; q0 < N; q0 += kGT) {
        __syncthreads();
        for (int i = tid; i < kGT * d; i += kGThreads) {
            const int q = i % kGT, f = i / kGT;
            sQ[q * ld + f] = (q0 + q < N) ? (A)Qb[(int64_t)f * N + q0 + q] : (A)0;
        }
        for (int i = tid; i < kGT * dv; i += kGThreads) {
            const int q = i % kGT, f = i / kGT;
            sdO[q * ldv + f] = (q0 + q < N) ? (A)dOb[(int64_t)f * N + q0 + q] : (A)0;
        }
        __syncthreads();
        for (int e = tid; e < kGT * kGT; e += kGThreads) {
            const int q = e / kGT, k = e % kGT;
            A pr = (A)0, ds = (A)0;
            if (q0 + q < N && k0 + k < Nk) {
                A s = (A)0, dp = (A)0;
                for (int f = 0; f < d; ++f) s = fma_a(sQ[q * ld + f], sK[k * ld + f], s);
                for (int f = 0; f < dv; ++f) dp = fma_a(sdO[q * ldv + f], sV[k * ldv + f], dp);
                pr = exp2_a((s + nL[q0 + q]) * sl2);
                ds = pr * (dp + nD[q0 + q]);
            }
            sP[q * (kGT + 1) + k] = pr;
            sdS[q * (kGT + 1) + k] = ds;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < kMaxPer; ++t) {
            const int i = tid + kGThreads * t, k = i % kGT, f = i / kGT;
            if (f < d) {
                A a = accK[t];
                for (int q = 0; q < kGT; ++q) a = fma_a(sdS[q * (kGT + 1) + k], sQ[q * ld + f], a);
                accK[t] = a;
            }
            if (f < dv) {
                A a = accV[t];
                for (int q = 0; q < kGT; ++q) a = fma_a(sP[q * (kGT + 1) + k], sdO[q * ldv + f], a);
                accV[t] = a;
            }
        }
    }
    T* dKb = (T*)p.dK + (int64_t)b * Nk * d;
    T* dVb = (T*)p.dV + (int64_t)b * Nk * dv;
    const A sc = bscale<A>(p);
#pragma unroll
    for (int t = 0; t < kMaxPer; ++t) {
        const int i = tid + kGThreads * t, k = i % kGT, f = i / kGT;
        if (k0 + k < Nk) {
            if (f < d) dKb[(int64_t)f * Nk + k0 + k] = (T)(accK[t] * sc);
            if (f < dv) dVb[(int64_t)f * Nk + k0 + k] = (T)accV[t];
        }
    }
}


// --------------------------------------------------------------------------
// 2./3. fp32 MFMA path (v_mfma_f32_32x32x2_f32: exact fp32 products, the same
// arithmetic as an fmaf chain; d, dv <= 128 (classes 32 / 64 / 128), any N, Nk).  Each lane keeps its
// own key's (dK/dV kernel) or query's (dQ kernel) K, V (resp. Q, dO) features in
// registers as the B operand of the score products; the tile of the other side
// sits in LDS ([feature][33] rows: conflict-free for both the column and the
// row access).  The score accumulators are used directly as the B operand of
// the gradient products: register x of lane (r, h) holds row acc_row(x, h), which
// is exactly what a 32x32x2 B operand with k = h needs (cf. the fp32 forward).
//   dK/dV: S = Q Kᵀ (queries on rows, keys on lanes), dVᵀ += dOᵀ P, dKᵀ += Qᵀ dS;
//   dQ   : Sᵀ = K Qᵀ (keys on rows, queries on lanes), dQᵀ += Kᵀ dSᵀ.
// Keys past Nk are zero rows: their own rows are not stored and their K = 0
// adds nothing to dQ; queries past N carry nlse = −inf (P = 0) and dO = 0.
// --------------------------------------------------------------------------
constexpr int kF32T = 32;   // tile of the streamed side
constexpr int kF32R = 33;   // LDS row (floats)

template <int D, int DV>
__global__ __launch_bounds__(256) void bwd_dkdv_f32(BwdParams p) {
    __shared__ float sQ[D * kF32R], sdO[DV * kF32R], sL[kF32T], sD[kF32T];
    const int N = p.N, Nk = p.Nk, d = p.d, dv = p.dv;
    const int nkb = (Nk + 127) / 128;
    const int b = blockIdx.x / nkb, k0 = (blockIdx.x % nkb) * 128;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const float* Qb = (const float*)p.Q + (int64_t)b * N * d;
    const float* dOb = (const float*)p.dO + (int64_t)b * N * dv;
    const float* Kb = (const float*)p.K + (int64_t)b * Nk * d;
    const float* Vb = (const float*)p.V + (int64_t)b * Nk * dv;
    const int key = k0 + wave * 32 + r;
    float kf[D / 2], vf[DV / 2];
#pragma unroll
    for (int t = 0; t < D / 2; ++t) kf[t] = (key < Nk && 2 * t + h < d) ? Kb[(int64_t)(2 * t + h) * Nk + key] : 0.0f;
#pragma unroll
    for (int t = 0; t < DV / 2; ++t) vf[t] = (key < Nk && 2 * t + h < dv) ? Vb[(int64_t)(2 * t + h) * Nk + key] : 0.0f;
    f32x16 aK[D / 32], aV[DV / 32];
#pragma unroll
    for (int i = 0; i < D / 32; ++i)
#pragma unroll
        for (int x = 0; x < 16; ++x) aK[i][x] = 0.0f;
#pragma unroll
    for (int i = 0; i < DV / 32; ++i)
#pragma unroll
        for (int x = 0; x < 16; ++x) aV[i][x] = 0.0f;
    const float c = p.scale_log2;
    const float* nD = p.nD + (int64_t)b * N;
    const float* nL = p.nlse + (int64_t)b * N;
    for (int q0 = 0; q0 < N; q0 += kF32T) {
        __syncthreads();
        for (int i = tid; i < D * kF32T; i += 256) {
            const int q = i % kF32T, f = i / kF32T;
            sQ[f * kF32R + q] = (q0 + q < N && f < d) ? Qb[(int64_t)f * N + q0 + q] : 0.0f;
        }
        for (int i = tid; i < DV * kF32T; i += 256) {
            const int q = i % kF32T, f = i / kF32T;
            sdO[f * kF32R + q] = (q0 + q < N && f < dv) ? dOb[(int64_t)f * N + q0 + q] : 0.0f;
        }
        if (tid < kF32T) {
            sL[tid] = q0 + tid < N ? nL[q0 + tid] : kNegInf;
            sD[tid] = q0 + tid < N ? nD[q0 + tid] : 0.0f;
        }
        __syncthreads();
        f32x16 sa, pa;
#pragma unroll
        for (int x = 0; x < 16; ++x) { sa[x] = 0.0f; pa[x] = 0.0f; }
#pragma unroll
        for (int t = 0; t < D / 2; ++t) sa = mfma32x32x2(sQ[(2 * t + h) * kF32R + r], kf[t], sa);
#pragma unroll
        for (int t = 0; t < DV / 2; ++t) pa = mfma32x32x2(sdO[(2 * t + h) * kF32R + r], vf[t], pa);
        // lane (r, h): key r; register x: query acc_row(x, h)
#pragma unroll
        for (int x = 0; x < 16; ++x) {
            const int q = acc_row(x, h);
            const float pr = exp2f((sa[x] + sL[q]) * c);
            sa[x] = pr;                          // P
            pa[x] = pr * (pa[x] + sD[q]);        // dS
        }
#pragma unroll
        for (int x = 0; x < 16; ++x) {
            const int q = acc_row(x, h);
#pragma unroll
            for (int i = 0; i < DV / 32; ++i) aV[i] = mfma32x32x2(sdO[(i * 32 + r) * kF32R + q], sa[x], aV[i]);
#pragma unroll
            for (int i = 0; i < D / 32; ++i) aK[i] = mfma32x32x2(sQ[(i * 32 + r) * kF32R + q], pa[x], aK[i]);
        }
    }
    if (key < Nk) {
        float* dKb = (float*)p.dK + (int64_t)b * Nk * d;
        float* dVb = (float*)p.dV + (int64_t)b * Nk * dv;
#pragma unroll
        for (int i = 0; i < D / 32; ++i)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int f = i * 32 + acc_row(x, h);
                if (f < d) dKb[(int64_t)f * Nk + key] = aK[i][x] * p.scale;
            }
#pragma unroll
        for (int i = 0; i < DV / 32; ++i)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int f = i * 32 + acc_row(x, h);
                if (f < dv) dVb[(int64_t)f * Nk + key] = aV[i][x];
            }
    }
}

template <int D, int DV>
__global__ __launch_bounds__(256) void bwd_dq_f32(BwdParams p) {
    __shared__ float sK[D * kF32R], sV[DV * kF32R];
    const int N = p.N, Nk = p.Nk, d = p.d, dv = p.dv;
    const int nqb = (N + 127) / 128;
    const int b = blockIdx.x / nqb, q0 = (blockIdx.x % nqb) * 128;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const float* Qb = (const float*)p.Q + (int64_t)b * N * d;
    const float* dOb = (const float*)p.dO + (int64_t)b * N * dv;
    const float* Kb = (const float*)p.K + (int64_t)b * Nk * d;
    const float* Vb = (const float*)p.V + (int64_t)b * Nk * dv;
    const int qi = q0 + wave * 32 + r;
    float qf[D / 2], df[DV / 2];
#pragma unroll
    for (int t = 0; t < D / 2; ++t) qf[t] = (qi < N && 2 * t + h < d) ? Qb[(int64_t)(2 * t + h) * N + qi] : 0.0f;
#pragma unroll
    for (int t = 0; t < DV / 2; ++t) df[t] = (qi < N && 2 * t + h < dv) ? dOb[(int64_t)(2 * t + h) * N + qi] : 0.0f;
    const float nlq = qi < N ? p.nlse[(int64_t)b * N + qi] : kNegInf;
    const float ndq = qi < N ? p.nD[(int64_t)b * N + qi] : 0.0f;
    const float c = p.scale_log2;
    f32x16 aQ[D / 32];
#pragma unroll
    for (int i = 0; i < D / 32; ++i)
#pragma unroll
        for (int x = 0; x < 16; ++x) aQ[i][x] = 0.0f;
    for (int k0 = 0; k0 < Nk; k0 += kF32T) {
        __syncthreads();
        for (int i = tid; i < D * kF32T; i += 256) {
            const int k = i % kF32T, f = i / kF32T;
            sK[f * kF32R + k] = (k0 + k < Nk && f < d) ? Kb[(int64_t)f * Nk + k0 + k] : 0.0f;
        }
        for (int i = tid; i < DV * kF32T; i += 256) {
            const int k = i % kF32T, f = i / kF32T;
            sV[f * kF32R + k] = (k0 + k < Nk && f < dv) ? Vb[(int64_t)f * Nk + k0 + k] : 0.0f;
        }
        __syncthreads();
        f32x16 sa, pa;
#pragma unroll
        for (int x = 0; x < 16; ++x) { sa[x] = 0.0f; pa[x] = 0.0f; }
#pragma unroll
        for (int t = 0; t < D / 2; ++t) sa = mfma32x32x2(sK[(2 * t + h) * kF32R + r], qf[t], sa);
#pragma unroll
        for (int t = 0; t < DV / 2; ++t) pa = mfma32x32x2(sV[(2 * t + h) * kF32R + r], df[t], pa);
        // lane (r, h): query r; register x: key acc_row(x, h)
#pragma unroll
        for (int x = 0; x < 16; ++x) {
            const float pr = exp2f((sa[x] + nlq) * c);
            pa[x] = pr * (pa[x] + ndq);          // dSᵀ
        }
#pragma unroll
        for (int x = 0; x < 16; ++x) {
            const int k = acc_row(x, h);
#pragma unroll
            for (int i = 0; i < D / 32; ++i) aQ[i] = mfma32x32x2(sK[(i * 32 + r) * kF32R + k], pa[x], aQ[i]);
        }
    }
    if (qi < N) {
        float* dQb = (float*)p.dQ + (int64_t)b * N * d;
#pragma unroll
        for (int i = 0; i < D / 32; ++i)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int f = i * 32 + acc_row(x, h);
                if (f < d) dQb[(int64_t)f * N + qi] = aQ[i][x] * p.scale;
            }
    }
}

template <int D, int DV>
static hipError_t launch_f32_dd(const BwdParams& p, hipStream_t s) {
    const int64_t nq = ((int64_t)p.N + 127) / 128 * p.batch, nk = ((int64_t)p.Nk + 127) / 128 * p.batch;
    hipLaunchKernelGGL((bwd_dq_f32<D, DV>), dim3((unsigned)nq), dim3(256), 0, s, p);
    hipLaunchKernelGGL((bwd_dkdv_f32<D, DV>), dim3((unsigned)nk), dim3(256), 0, s, p);
    return hipGetLastError();
}
static hipError_t launch_f32_mfma(const BwdParams& p, hipStream_t s) {
    if (p.d > 64 || p.dv > 64) return launch_f32_dd<128, 128>(p, s);
    const int Dc = p.d <= 32 ? 32 : 64, DVc = p.dv <= 32 ? 32 : 64;
    if (Dc == 32 && DVc == 32) return launch_f32_dd<32, 32>(p, s);
    if (Dc == 32) return launch_f32_dd<32, 64>(p, s);
    if (DVc == 32) return launch_f32_dd<64, 32>(p, s);
    return launch_f32_dd<64, 64>(p, s);
}

// --------------------------------------------------------------------------
// 2./3. MFMA fast path (bf16 / fp16; d, dv in {32, 64, 128}; N, Nk % 8 == 0;
// 16-B aligned).  Token tiles of 64 are staged by LDS-DMA (buffer_load … lds)
// into [rows][64 tokens] images with 128-B rows and a 16-B XOR swizzle
// g(f) = ((f>>3)&3) | ((f>>1)&1)<<2 that makes BOTH access patterns
// conflict-free: the transposed reads ds_read_b64_tr_b16 (A operands of the
// score / dP products: 4 consecutive rows × 64 B per half-wave) and the
// ds_read_b128 row reads (A operands of the gradient products: 16 rows per
// lane group, one 16-B chunk each).
// --------------------------------------------------------------------------
__device__ __forceinline__ int swz16(int f) { return ((f >> 3) & 3) | (((f >> 1) & 1) << 2); }

template <class T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bslab(const void* base, int64_t off_elems, int64_t elems) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)((const T*)base + off_elems), (short)0,
                                             (int)(elems * (int64_t)sizeof(T)), 0x00020000);
}

// LDS-DMA one [R rows][64 tokens] image (R*128 bytes) from a [*][ntok] slab at
// token t0.  4 waves; each wave-instruction fills 1 KiB (8 rows) lane-linearly,
// so the swizzle is applied to the per-lane GLOBAL address (cdna guide rule 21).
template <int R>
__device__ __forceinline__ void dma_image(__amdgpu_buffer_rsrc_t rs, char* img, int ntok, int t0, int wave, int lane) {
#pragma unroll
    for (int it = 0; it < R / 32; ++it) {
        const int blk = it * 4 + wave;                 // 1-KiB block of the image
        const int P = blk * 64 + lane;                 // 16-B chunk index (linear in LDS)
        const int f = P >> 3, c = (P & 7) ^ swz16(f);  // logical chunk at that position
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(img + blk * 1024), 16,
            (f * ntok + t0 + 8 * c) * 2, 0, 0, 0);
    }
}

// Inter-workgroup words of the single-pass kernel: global (never flat), agent
// scope, relaxed (global_load / global_store ... sc1).
typedef __attribute__((address_space(1))) unsigned gu32;
__device__ __forceinline__ unsigned ld_agent(gu32* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(gu32* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-lane constant parts of the two fragment reads of an image.
struct FragAddr {
    int tr[2][2];   // [token block tb][s & 1] byte offset of the transposed read (half2 = 0)
    int row[2];     // [h-independent] b128 row read: swizzled chunk offsets need (r, chunk)
};

__device__ __forceinline__ int sig32(int r) { return (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1); }

// dQ of the wrapped slices of query block qb (slices 2qb, 2qb + 1) of slab b whose two
// chain tails both stored their totals (fin == 2, bwd_fused): dQ = (A + B)·τ, the same
// single add — so the same bits — as chain B's tail makes when A is done first.  The
// totals are in bwd_fused's running-sum layout: per slice NTQ tiles of 32 x 32 fp32,
// lane l's 16-B pieces c4 at l·16 + c4·1024, element 4 c4 + e = dQᵀ row (feature)
// 32 cb + acc_row(4 c4 + e, l >> 5), column (query) 32 u + sig32(l & 31), tile = u·D/32 + cb.
template <class T, int D>
__device__ void fused_combine(const BwdParams& p, int b, int qb) {
    constexpr int NTQ = D / 16;
    const int NS = p.nqt, N = p.N;
    const float* const partb = p.part + (int64_t)b * 2 * NS * NTQ * 1024;
    const int64_t pchain = (int64_t)NS * NTQ * 1024;
    T* const dQb = (T*)p.dQ + (int64_t)b * N * D;
    for (int t = 2 * qb; t < 2 * qb + 2 && t < NS; ++t) {
        if (ld_agent((gu32*)(uintptr_t)(p.fin + (int64_t)b * NS + t)) != 2u) continue;
        for (int idx = threadIdx.x; idx < NTQ * 64; idx += 256) {
            const int w = idx >> 6, l = idx & 63;
            const int cb = w % (D / 32), u = w / (D / 32);
            const int q = t * 64 + 32 * u + sig32(l & 31);
            const float* a = partb + (int64_t)(t * NTQ + w) * 1024 + l * 4;
            const float* bb = a + pchain;
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4) {
                const f32x4 va = *(const f32x4*)(a + c4 * 256), vb = *(const f32x4*)(bb + c4 * 256);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int x = 4 * c4 + e;
                    const int f = cb * 32 + acc_row(x, l >> 5);
                    if (q < N) dQb[(int64_t)f * N + q] = (T)((va[e] + vb[e]) * p.scale);
                }
            }
        }
    }
}

template <class T, int D, int DV>
__global__ __launch_bounds__(256, 2) void bwd_dq_fast(BwdParams p) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int KB = D * 128, VB = DV * 128, STAGE = KB + VB;
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
    // after bwd_fused: recompute dQ only on the slabs whose hand-off gave up, and make
    // dQ = A + B of the wrapped slices whose two chain tails both stored their totals
    const bool give_up = p.guard && ld_agent((gu32*)(uintptr_t)p.guard) != 0u;
    const bool combine = p.cguard && ld_agent((gu32*)(uintptr_t)p.cguard) != 0u;
    if (p.guard && !give_up && !combine) return;
    const int lid = xcd_remap(blockIdx.x, p.total_wg);
    const int b = lid / p.nblk, qb = lid - b * p.nblk;
    if (p.sguard && (!give_up || ld_agent((gu32*)(uintptr_t)(p.sguard + b)) == 0u)) {
        if (combine) fused_combine<T, D>(p, b, qb);
        return;
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const int N = p.N, Nk = p.Nk;
    const auto qrs = bslab<T>(p.Q, (int64_t)b * N * D, (int64_t)N * D);
    const auto ors = bslab<T>(p.dO, (int64_t)b * N * DV, (int64_t)N * DV);
    const auto krs = bslab<T>(p.K, (int64_t)b * Nk * D, (int64_t)Nk * D);
    const auto vrs = bslab<T>(p.V, (int64_t)b * Nk * DV, (int64_t)Nk * DV);
    const int qi = qb * 128 + wave * 32 + r;
    F8 qf[D / 16], df[DV / 16];
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e)
            qf[s][e] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b16(qrs, ((16 * s + 8 * h + e) * N + qi) * 2, 0, 0));
#pragma unroll
    for (int s = 0; s < DV / 16; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e)
            df[s][e] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b16(ors, ((16 * s + 8 * h + e) * N + qi) * 2, 0, 0));
    const int qc = qi < N ? qi : N - 1;
    const float c = p.scale_log2;
    const float cnl = c * p.nlse[(int64_t)b * N + qc];
    const float nDq = p.nD[(int64_t)b * N + qc];

    // transposed-read lane offsets (see fa_fwd.hip): lane 4q+pp of 16-lane group g
    const int g = lane >> 4, kh = g & 1, qq = (lane & 15) >> 2, pp = lane & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
    int tro[2][2];
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
            const int sw = ((sp << 1) | h) | (((qq >> 1) & 1) << 2);
            tro[tb][sp] = (8 * h + qq) * 128 + (((tb * 4 + kh * 2 + (sig >> 1)) ^ sw) * 16) + (sig & 1) * 8;
        }
    const int rsw = swz16(r);
    auto trfrag = [&](const char* img, int tb, int s) -> F8 {
        const char* a = img + tro[tb][s & 1] + 16 * s * 128;
        const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(a));
        const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(a + 4 * 128));
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    auto rowfrag = [&](const char* img, int cb, int tb, int s2) -> F8 {
        return *(const F8*)(img + (cb * 32 + r) * 128 + (((tb * 4 + 2 * s2 + h) ^ rsw) * 16));
    };

    f32x16 dq[D / 32];
#pragma unroll
    for (int cb = 0; cb < D / 32; ++cb)
#pragma unroll
        for (int x = 0; x < 16; ++x) dq[cb][x] = 0.0f;

    auto fill = [&](char* st, int t) {
        dma_image<D>(krs, st, Nk, t * 64, wave, lane);
        dma_image<DV>(vrs, st + KB, Nk, t * 64, wave, lane);
    };
    auto compute = [&](const char* st, int t) {
        const char* kimg = st;
        const char* vimg = st + KB;
        const bool partial = (t + 1) * 64 > Nk;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            f32x16 sa, dp;
#pragma unroll
            for (int x = 0; x < 16; ++x) { sa[x] = 0.0f; dp[x] = 0.0f; }
#pragma unroll
            for (int s = 0; s < D / 16; ++s) sa = mfma32x32x16(trfrag(kimg, kb, s), qf[s], sa);
#pragma unroll
            for (int s = 0; s < DV / 16; ++s) dp = mfma32x32x16(trfrag(vimg, kb, s), df[s], dp);
            if (partial) {
#pragma unroll
                for (int x = 0; x < 16; ++x)
                    if (t * 64 + kb * 32 + (x & 7) + 8 * h + 16 * (x >> 3) >= Nk) sa[x] = kNegInf;
            }
            F8 dsf[2];
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const float pr = exp2_fast(fmaf(sa[x], c, cnl));
                dsf[x >> 3][x & 7] = (T)(pr * (dp[x] + nDq));
            }
#pragma unroll
            for (int cb = 0; cb < D / 32; ++cb)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) dq[cb] = mfma32x32x16(rowfrag(kimg, cb, kb, s2), dsf[s2], dq[cb]);
        }
    };

    const int NT = (Nk + 63) / 64;
    char* const st0 = smem;
    char* const st1 = smem + STAGE;
    fill(st0, 0);
    __syncthreads();
    for (int t = 0; t < NT; t += 2) {
        fill(st1, min(t + 1, NT - 1));
        compute(st0, t);
        __syncthreads();
        if (t + 1 < NT) {
            fill(st0, min(t + 2, NT - 1));
            compute(st1, t + 1);
            __syncthreads();
        }
    }
    if (qi < N) {
        T* dQb = (T*)p.dQ + (int64_t)b * N * D;
#pragma unroll
        for (int cb = 0; cb < D / 32; ++cb)
#pragma unroll
            for (int x = 0; x < 16; ++x)
                dQb[(int64_t)(cb * 32 + acc_row(x, h)) * N + qi] = (T)(dq[cb][x] * p.scale);
    }
}

template <class T, int D, int DV>
__global__ __launch_bounds__(256, 2) void bwd_dkdv_fast(BwdParams p) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int QB = D * 128, OB = DV * 128, STAGE = QB + OB + 512;
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
    const int lid = xcd_remap(blockIdx.x, p.total_wg);
    const int b = lid / p.nblk, kblk = lid - b * p.nblk;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const int N = p.N, Nk = p.Nk;
    const auto qrs = bslab<T>(p.Q, (int64_t)b * N * D, (int64_t)N * D);
    const auto ors = bslab<T>(p.dO, (int64_t)b * N * DV, (int64_t)N * DV);
    const auto krs = bslab<T>(p.K, (int64_t)b * Nk * D, (int64_t)Nk * D);
    const auto vrs = bslab<T>(p.V, (int64_t)b * Nk * DV, (int64_t)Nk * DV);
    const int kj = kblk * 128 + wave * 32 + r;   // this lane's key (column of S, dP)
    F8 kf[D / 16], vf[DV / 16];
#pragma unroll
    for (int s = 0; s < D / 16; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e)
            kf[s][e] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b16(krs, ((16 * s + 8 * h + e) * Nk + kj) * 2, 0, 0));
#pragma unroll
    for (int s = 0; s < DV / 16; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e)
            vf[s][e] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b16(vrs, ((16 * s + 8 * h + e) * Nk + kj) * 2, 0, 0));
    const float c = p.scale_log2;
    const float* nlse = p.nlse + (int64_t)b * N;
    const float* nDg = p.nD + (int64_t)b * N;

    const int g = lane >> 4, kh = g & 1, qq = (lane & 15) >> 2, pp = lane & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
    int tro[2][2];
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
            const int sw = ((sp << 1) | h) | (((qq >> 1) & 1) << 2);
            tro[tb][sp] = (8 * h + qq) * 128 + (((tb * 4 + kh * 2 + (sig >> 1)) ^ sw) * 16) + (sig & 1) * 8;
        }
    const int rsw = swz16(r);
    auto trfrag = [&](const char* img, int tb, int s) -> F8 {
        const char* a = img + tro[tb][s & 1] + 16 * s * 128;
        const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(a));
        const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(a + 4 * 128));
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    auto rowfrag = [&](const char* img, int cb, int tb, int s2) -> F8 {
        return *(const F8*)(img + (cb * 32 + r) * 128 + (((tb * 4 + 2 * s2 + h) ^ rsw) * 16));
    };

    f32x16 dk[D / 32], dv[DV / 32];
#pragma unroll
    for (int cb = 0; cb < D / 32; ++cb)
#pragma unroll
        for (int x = 0; x < 16; ++x) dk[cb][x] = 0.0f;
#pragma unroll
    for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
        for (int x = 0; x < 16; ++x) dv[cb][x] = 0.0f;

    // per-tile row constants: threads 0-63 carry −lse (−inf past N), 64-127 −D
    float rowc = 0.0f;
    auto load_rowc = [&](int t) {
        const int q = t * 64 + (tid & 63);
        if (tid < 64) rowc = q < N ? nlse[q] : kNegInf;
        else if (tid < 128) rowc = q < N ? nDg[q] : 0.0f;
    };
    auto store_rowc = [&](char* st) {
        if (tid < 128) ((float*)(st + QB + OB))[tid] = rowc;
    };
    auto fill = [&](char* st, int t) {
        dma_image<D>(qrs, st, N, t * 64, wave, lane);
        dma_image<DV>(ors, st + QB, N, t * 64, wave, lane);
    };
    auto compute = [&](const char* st) {
        const char* qimg = st;
        const char* oimg = st + QB;
        const float* rl = (const float*)(st + QB + OB);      // −lse[64], then −D[64]
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            // rows of S / dP (queries) map to 8h + {0..7} and 16 + 8h + {0..7}
            f32x16 sa, dp;
            const f32x4* Lq = (const f32x4*)(rl + u * 32 + 8 * h);
            const f32x4* Dq = (const f32x4*)(rl + 64 + u * 32 + 8 * h);
            const f32x4 l0 = Lq[0], l1 = Lq[1], l2 = Lq[4], l3 = Lq[5];
            const f32x4 d0 = Dq[0], d1 = Dq[1], d2 = Dq[4], d3 = Dq[5];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                sa[e] = l0[e]; sa[4 + e] = l1[e]; sa[8 + e] = l2[e]; sa[12 + e] = l3[e];
                dp[e] = d0[e]; dp[4 + e] = d1[e]; dp[8 + e] = d2[e]; dp[12 + e] = d3[e];
            }
#pragma unroll
            for (int s = 0; s < D / 16; ++s) sa = mfma32x32x16(trfrag(qimg, u, s), kf[s], sa);
#pragma unroll
            for (int s = 0; s < DV / 16; ++s) dp = mfma32x32x16(trfrag(oimg, u, s), vf[s], dp);
            F8 pf[2], dsf[2];
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const float pr = exp2_fast(sa[x] * c);
                pf[x >> 3][x & 7] = (T)pr;
                dsf[x >> 3][x & 7] = (T)(pr * dp[x]);
            }
#pragma unroll
            for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) dv[cb] = mfma32x32x16(rowfrag(oimg, cb, u, s2), pf[s2], dv[cb]);
#pragma unroll
            for (int cb = 0; cb < D / 32; ++cb)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) dk[cb] = mfma32x32x16(rowfrag(qimg, cb, u, s2), dsf[s2], dk[cb]);
        }
    };

    const int NT = (N + 63) / 64;
    char* const st0 = smem;
    char* const st1 = smem + STAGE;
    load_rowc(0);
    fill(st0, 0);
    store_rowc(st0);
    __syncthreads();
    for (int t = 0; t < NT; t += 2) {
        load_rowc(min(t + 1, NT - 1));
        fill(st1, min(t + 1, NT - 1));
        compute(st0);
        store_rowc(st1);
        __syncthreads();
        if (t + 1 < NT) {
            load_rowc(min(t + 2, NT - 1));
            fill(st0, min(t + 2, NT - 1));
            compute(st1);
            store_rowc(st0);
            __syncthreads();
        }
    }
    if (kj < Nk) {
        T* dKb = (T*)p.dK + (int64_t)b * Nk * D;
        T* dVb = (T*)p.dV + (int64_t)b * Nk * DV;
#pragma unroll
        for (int cb = 0; cb < D / 32; ++cb)
#pragma unroll
            for (int x = 0; x < 16; ++x)
                dKb[(int64_t)(cb * 32 + acc_row(x, h)) * Nk + kj] = (T)(dk[cb][x] * p.scale);
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int x = 0; x < 16; ++x)
                dVb[(int64_t)(cb * 32 + acc_row(x, h)) * Nk + kj] = (T)dv[cb][x];
    }
}

// --------------------------------------------------------------------------
// Single-pass backward: the five MFMA products of OneDFastBack
// (src_cpp/FlashAttention.cpp:221-251) — S, dP, dVᵀ += dOᵀP, dKᵀ += QᵀdS and
// dQᵀ += KᵀdSᵀ — in one sweep, instead of the dK/dV pass plus a dQ pass that
// recomputes S and dP (7 products).
//
// A workgroup = 8 waves = 256 keys of one slab (member j of the slab's K = Nk/256
// workgroups); wave w keeps dKᵀ, dVᵀ of its 32 keys in registers (the dK/dV pass's
// layout) and the workgroup sweeps the slab's 64-query slices.  Per slice, dS goes
// through LDS once as a [key][query] image, and wave w computes one 32 x 32 tile of
// dQᵀ over all 256 keys from it and the K image.  The slab's K workgroups sum each
// slice's dQ in a FIXED order (deterministic, no float atomics): member j sweeps the
// slices rotated by 3j (step i: slice (i − 3j) mod T), so the member that adds to a
// slice after member j does so three steps later.  Where that order wraps from member
// K−1 to member 0 it is cut: a slice's members form chain A (the ones that reach it
// first, w0 .. K−1) and chain B (0 .. w0−1), each summed upwards, and dQ = A + B — one
// add, commutative, so the same bits whoever makes it.  Every member therefore waits
// only on the member before it, j − 1, dispatched before it.  The running fp32 sum is
// handed over through the workspace with sc1 stores, a per-slice counter (one lane,
// sc1) that the next member polls (one lane) before a barrier, and sc1 loads
// (MI355X_MICROARCH § visibility, first row of the sc1 hand-off table; 1 WG per CU).
// Chain A's tail stores its total; chain B's tail adds it in when A has finished by
// then (always, solo: A runs ≥ 3 steps earlier) and writes dQ, else stores its own
// total and leaves the add to bwd_dq_fast, which runs after every single pass (the
// slice's fin word, an agent-scope counter both tails add to, reads 2 then).
// Step i of a member, in issue order: B1 (vmcnt(4): slice i's Q/dO DMA landed, step
// i-1's four sum stores may still fly) | phase A, u = 0 | vmcnt(0): step i-1's sums
// stored | u = 1 | lane 0 polls the count of step i+1's slice; the sum loads of step i
// | B2; lane 0 publishes step i-1's count | the row constants and Q/dO DMA of step
// i+1 | the dQ tile (asm LDS reads) | vmcnt(NDMA): the sums landed, added | the sum
// stores (or the tail's dQ stores).  So no barrier waits on a store, and the only
// vmcnt(0) of a step is the one in the middle of phase A.
// No member needs another to be resident: dispatch within an XCD is in launch order,
// so the lowest unfinished workgroup is always on a CU or next in line, and it waits on
// nothing unfinished.  A co-tenant (another stream or process) can slow the chains but
// not strand them.  A poll gives up only if the whole launch publishes nothing for
// 100 ms (see wait_count); it then sets the slab's trip word and the call's status
// word `err`, the slab's other polls stop at once, and the guarded bwd_dq_fast that
// follows recomputes dQ of the slabs that tripped (dK, dV do not depend on the
// hand-off).
// --------------------------------------------------------------------------
// 16-B swizzle of the dSᵀ image, which is written by ds_write_b128 (8 groups of 8
// contiguous lanes, banks mod 128 B) at rows sig32(r) and read only transposed.  A
// write group covers rows {0..3} + {0, 8} (+ 4, 16, 20): the swizzle is a bijection of
// row bits {0, 1, 3}, so its 8 slots differ; its bit 2 = row bit 1, so rows q and
// q ^ 2 of a transposed read sit in opposite 64-B halves of their bank row.  (swz16
// gives rows 0 and 4 the same slot: measured 6.7e7 conflict cycles at N = 8192.)
__device__ __forceinline__ int swzds(int f) { return ((f >> 3) & 1) | ((f & 1) << 1) | (((f >> 1) & 1) << 2); }

// [R rows][64 tokens] LDS image written by 8 waves (cf. dma_image).
template <int R>
__device__ __forceinline__ void dma_image8(__amdgpu_buffer_rsrc_t rs, char* img, int ntok, int t0, int wave, int lane) {
    constexpr int NB = R / 8;                          // 1-KiB blocks
#pragma unroll
    for (int it = 0; it < (NB + 7) / 8; ++it) {
        const int blk = it * 8 + wave;
        if (NB % 8 == 0 || blk < NB) {
            const int P = blk * 64 + lane;
            const int f = P >> 3, c = (P & 7) ^ swz16(f);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void*)(img + blk * 1024), 16,
                (f * ntok + t0 + 8 * c) * 2, 0, 0, 0);
        }
    }
}

__device__ __forceinline__ void arrive(gu32* p) {
    __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One lane waits until *f >= want (its predecessor in a chain has published).  Every
// such wait is on the previous member of the slab, of lower launch id, so it cannot
// strand (see bwd_fused).  The poll gives up — the slab's trip word *serr and the
// call's status word *herr are set, the slab's other polls stop — only when neither
// the launch's arrival count *garr nor any publish count of the slab's KM members
// (prog[], one plain store per member and step: a single launch-wide counter bumped
// per publish measured 5 % slower, its atomics queueing on one address) has moved for
// stall_ticks (100 ms): a safety net for a dispatcher that broke launch order, not a
// scheduling decision.  A co-tenant that holds CUs for longer than that costs a
// recompute of the slab's dQ, never a wrong result.
__device__ __forceinline__ void wait_count(gu32* f, unsigned want, gu32* serr, gu32* herr, gu32* garr, gu32* prog,
                                           int KM, uint64_t stall_ticks) {
    if (ld_agent(f) >= want) return;
    auto progress = [&]() {
        unsigned sum = ld_agent(garr);
        for (int k = 0; k < KM; ++k) sum += ld_agent(prog + k);
        return sum;
    };
    // the progress counts are first read after 20 us of waiting (not at entry: a
    // short wait — the common case — then costs no more than the polls themselves)
    uint64_t tw = __builtin_amdgcn_s_memrealtime(), tc = tw;
    unsigned seen = 0u;
    bool have = false;
    for (;;) {
        __builtin_amdgcn_s_sleep(1);
        if (ld_agent(f) >= want || ld_agent(serr) != 0u) return;
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (now - tc < 2000) continue;   // look at the progress counts every 20 us
        tc = now;
        const unsigned pg = progress();
        if (!have || pg != seen) {
            have = true;
            seen = pg;
            tw = now;
        } else if (now - tw > stall_ticks) {
            st_agent(serr, 1u);
            st_agent(herr, 1u);
            // hdr[2]: a count of give-ups the pre-pass never resets (callers read it
            // around a series of calls: fa_hip.backward_handoff_trips)
            __hip_atomic_fetch_add(herr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
}

// LDS reads hidden from the compiler, with an immediate offset.  hipcc makes every
// LDS access it can see after a `buffer_load ... lds` wait for ALL outstanding
// vector-memory operations (s_waitcnt vmcnt(0): it cannot tell which buffer a DMA
// writes), which in bwd_fused put the next slice's Q/dO DMA and the running-sum
// loads in front of the dQ phase.  A result is not ready until an lgkmcnt wait;
// pass it through reg_fence() after that wait, before any use.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
template <int OFF>
__device__ __forceinline__ u32x4 lds_b128_at(uint32_t a) {
    u32x4 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF) : "memory");
    return r;
}
template <int OFF>
__device__ __forceinline__ s16x4 lds_tr16_at(uint32_t a) {
    s16x4 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF) : "memory");
    return r;
}
__device__ __forceinline__ void lds_w32(void* p, float v) {
    asm volatile("ds_write_b32 %0, %1" : : "v"(lds_addr(p)), "v"(v) : "memory");
}
template <int N>
__device__ __forceinline__ void lgkm_wait() { asm volatile("s_waitcnt lgkmcnt(%0)" : : "i"(N) : "memory"); }
template <class X>
__device__ __forceinline__ void reg_fence(X& x) { asm volatile("" : "+v"(x)); }
// A copy of x the compiler cannot see through: values derived from it inside a loop
// are not hoisted (hoisted per-lane addresses stay live across the loop and spill).
__device__ __forceinline__ int opaque(int x) { asm volatile("" : "+v"(x)); return x; }
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) { static_for_impl(f, std::make_integer_sequence<int, N>{}); }

// Buffer descriptor as four SGPRs for inline asm (raw buffer, stride 0, the
// make_buffer_rsrc flags used everywhere here).
__device__ __forceinline__ u32x4 desc_of(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)base;
    return u32x4{(unsigned)a, (unsigned)(a >> 32), bytes, 0x00020000u};
}
// Vector-memory operations hidden from the compiler's waitcnt model: the caller
// counts vmcnt for them (they retire in issue order) and fences the results.
__device__ __forceinline__ void dma16_asm(const u32x4& desc, uint32_t lds_base, int voff) {
    // s_nop 4: five wait states between a VALU write of the descriptor SGPRs (v_readlane
    // of a spilled SGPR, which the hazard recognizer cannot see past the asm) and the read
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" : : "v"(voff), "s"(desc), "{m0}"(lds_base) : "memory");
}
template <int OFF>
__device__ __forceinline__ u32x4 load16_sc1_asm(const u32x4& desc, int voff) {
    u32x4 r;
    // no s_nop here: no spill restore lands in front of these (tools/vmem_sgpr_hazards.py,
    // tests/test_code_hazards.py); one per load cost 2 % at configs[3]
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3 sc1" : "=v"(r) : "v"(voff), "s"(desc), "i"(OFF) : "memory");
    return r;
}
// dma_image8 through dma16_asm; returns nothing, issues (R/8 + 7)/8 ops or fewer per wave
template <int R>
__device__ __forceinline__ void dma_image8_asm(const u32x4& desc, char* img, int ntok, int t0, int wave, int lane) {
    constexpr int NB = R / 8;
#pragma unroll
    for (int it = 0; it < (NB + 7) / 8; ++it) {
        const int blk = it * 8 + wave;
        if (NB % 8 == 0 || blk < NB) {
            const int P = blk * 64 + lane;
            const int f = P >> 3, c = (P & 7) ^ swz16(f);
            dma16_asm(desc, lds_addr(img + blk * 1024), (f * ntok + t0 + 8 * c) * 2);
        }
    }
}
__device__ __forceinline__ float load4_asm(const float* p) {
    float r;
    asm volatile("global_load_dword %0, %1, off" : "=v"(r) : "v"(p) : "memory");
    return r;
}
// vmcnt immediates (gfx9 encoding: vmcnt[3:0] + [15:14], expcnt[6:4] = 7, lgkmcnt[11:8] = 15)
template <int N>
__device__ __forceinline__ void vm_wait() {
    static_assert(N >= 0 && N < 16, "vmcnt");
    __builtin_amdgcn_s_waitcnt(0x0F70 | N);
}

// Diagnostic phase stamps (tools/exp/bwd4_stamp.py; empty in the product build):
// -DFA_BWD_STAMP4=w records s_memtime of workgroup w's first lane at phase points of
// its first 128 steps (0 after B1, 8 end of phase A, 9 after B2, 10 end of the dQ phase).
#ifdef FA_BWD_STAMP4
__device__ unsigned long long g_bwd_stamp[128 * 16];
#define BWD_STAMP(pt)                                                                          \
    do {                                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        if (blockIdx.x == FA_BWD_STAMP4 && threadIdx.x == 0 && i < 128)                        \
            g_bwd_stamp[i * 16 + (pt)] = __builtin_amdgcn_s_memtime();                         \
        __builtin_amdgcn_sched_barrier(0);                                                     \
    } while (0)
#else
#define BWD_STAMP(pt)
#endif

template <class T, int D, int DV>
__global__ __launch_bounds__(512, 1) void bwd_fused(BwdParams p) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int KSUB = D * 128;                  // K image of 64 keys: [D][64]
    constexpr int QB = D * 128, OB = DV * 128;
    constexpr int STAGE = QB + OB + 512;           // Q, dO images + (−lse, −D) of one slice
    constexpr int DSB = 256 * 128;                 // dSᵀ image [256 keys][64 queries]
    constexpr int NTQ = D / 16;                    // 32 x 32 dQᵀ tiles per slice (<= 8 waves)
    __shared__ __attribute__((aligned(16))) char smem[4 * KSUB + STAGE + DSB];
    char* const kimg = smem;
    char* const qimg = smem + 4 * KSUB;
    char* const oimg = qimg + QB;
    float* const rowc = (float*)(oimg + OB);       // −lse[64] (raw units), −D[64]
    char* const dsimg = qimg + STAGE;

#ifdef FA_BWD_ABL
    const int abl = p.ablate;
#else
    constexpr int abl = 0;   // the timing-only ablations exist only in -DFA_BWD_ABL builds
#endif
    const int lid = p.xcd ? xcd_remap(blockIdx.x, p.total_wg) : (int)blockIdx.x;
    const int KM = p.nkb, NS = p.nqt, OFF = p.hoff;   // members per slab, slices
    const int b = lid / KM, j = lid - b * KM;
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int N = p.N, Nk = p.Nk;
    const auto qrs = bslab<T>(p.Q, (int64_t)b * N * D, (int64_t)N * D);
    const auto ors = bslab<T>(p.dO, (int64_t)b * N * DV, (int64_t)N * DV);
    const auto krs = bslab<T>(p.K, (int64_t)b * Nk * D, (int64_t)Nk * D);
    const auto vrs = bslab<T>(p.V, (int64_t)b * Nk * DV, (int64_t)Nk * DV);
    const int key0 = j * 256;
    const int kj = key0 + 32 * wave + sig32(r);   // this lane's key (column of S, dP, dKᵀ, dVᵀ)
    const bool key_ok = kj < Nk;
    const float c = p.scale_log2;
    const float* nlse = p.nlse + (int64_t)b * N;
    const float* nDg = p.nD + (int64_t)b * N;
    const int64_t pslab = (int64_t)2 * NS * NTQ * 1024;   // floats of running sums per slab (two chains)
    const int pchain4 = NS * NTQ * 4096;                  // bytes of one chain's sums
    const auto prs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.part + b * pslab), (short)0, (int)(pslab * 4),
                                                       0x00020000);
    const u32x4 pdesc = desc_of(p.part + b * pslab, (uint32_t)(pslab * 4));
    const u32x4 qdesc = desc_of((const T*)p.Q + (int64_t)b * N * D, (uint32_t)(N * D * 2));
    const u32x4 odesc = desc_of((const T*)p.dO + (int64_t)b * N * DV, (uint32_t)(N * DV * 2));
    // this wave's loop DMA ops per slice (dma_image8_asm), >= for every wave: a lower bound
    constexpr int NDMA = (D / 8 >= 8 ? D / 64 : 0) + (DV / 8 >= 8 ? DV / 64 : 0);
    // The hand-off's bookkeeping (polls, publishes, the XCD words) is lane 0's alone, so
    // its pointers and state live in LDS, read where they are used through an address
    // the compiler cannot see through (hc(): never hoisted into registers).  Held in
    // SGPRs across the loop they spilled, and their v_readlane restores ran in every
    // step of every wave (35 more SGPR spills than round 4's single chain, 4 times the
    // restores in the loop, 6-13 % slower).
    struct HoffCtx {
        gu32* cnt[2];      // chains A, B: [NS] members of the chain that have published slice t
        gu32* fin;         // [NS] tails of a wrapped slice's two chains that stored their sums
        gu32* serr;        // this slab's trip word
        gu32* err;         // the call's status word (err[1]: the sticky give-up count)
        gu32* garr;        // the launch's arrival count
        gu32* prog;        // [KM] the slab's publish progress
        gu32* xccw;        // [KM] its members' XCDs + 1
        gu32* comb;        // a wrapped slice is left to bwd_dq_fast's combine
        uint64_t stall;    // no-progress bound of a poll
        unsigned next_known;   // j + 1's XCD seen (or not needed)
        unsigned pub;      // the last step's publish: kind | ch << 2 | pos << 3 | t << 12
                           // (pos < K <= CUs < 512; t < 2^20, fused_plan)
        unsigned nodirect; // tests: a chain-B tail never takes the direct add (p.nodirect)
    };
    __shared__ HoffCtx s_hc;
    typedef __attribute__((address_space(3))) HoffCtx LHoff;
    auto hc = [&]() {
        uint32_t a = lds_addr(&s_hc);
        asm volatile("" : "+v"(a));
        return (LHoff*)(uintptr_t)a;
    };
    auto my_xcc = []() { return (__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) & 7u) + 1u; };   // HW_REG_XCC_ID[3:0]
    if (tid == 0) {
        const FusedFlags ff = fused_flags(p.batch, NS, KM);
        s_hc.cnt[0] = (gu32*)(p.flags + ff.cnt + (int64_t)b * NS);
        s_hc.cnt[1] = (gu32*)(p.flags + ff.cnt + (int64_t)(p.batch + b) * NS);
        s_hc.fin = (gu32*)(p.flags + ff.fin + (int64_t)b * NS);
        s_hc.serr = (gu32*)(p.flags + ff.serr + b);
        s_hc.err = (gu32*)p.err;
        s_hc.garr = (gu32*)(p.flags + ff.garr);
        s_hc.prog = (gu32*)(p.flags + ff.prog + (int64_t)b * KM);
        s_hc.xccw = (gu32*)(p.flags + ff.xcc + (int64_t)b * KM);
        s_hc.comb = (gu32*)(p.hdr + 3);
        s_hc.stall = (uint64_t)p.stall_ticks;
        s_hc.next_known = (!p.l2local || j + 1 >= KM) ? 1u : 0u;
        s_hc.pub = 0u;
        s_hc.nodirect = p.nodirect ? 1u : 0u;
        st_agent(s_hc.xccw + j, my_xcc());
        arrive(s_hc.garr);
    }
    // lane 0: wait until chain ch's member pos - 1 has published slice t
    auto poll = [&](int ch, int t, int pos) {
        LHoff* const h = hc();
        wait_count(h->cnt[ch] + t, (unsigned)pos, h->serr, h->err, h->garr, h->prog, KM, h->stall);
    };

    const int g = lane >> 4, kh = g & 1, qq = (lane & 15) >> 2, pp = lane & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
    int tro[2][2];
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
            const int sw = ((sp << 1) | h) | (((qq >> 1) & 1) << 2);
            tro[tb][sp] = (8 * h + qq) * 128 + (((tb * 4 + kh * 2 + (sig >> 1)) ^ sw) * 16) + (sig & 1) * 8;
        }
    const int rsw = swz16(r);
    auto trfrag = [&](const char* img, int tb, int s) -> F8 {
        const char* a = img + tro[tb][s & 1] + 16 * s * 128;
        const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(a));
        const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(a + 4 * 128));
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    auto rowfrag = [&](const char* img, int cb, int tb, int s2) -> F8 {
        return *(const F8*)(img + (cb * 32 + r) * 128 + (((tb * 4 + 2 * s2 + h) ^ rsw) * 16));
    };
    auto slice_of = [&](int i) {
        int t = (i - OFF * j) % NS;
        return t < 0 ? t + NS : t;
    };
    // this member's link in slice t's chains: the members that reach t first (steps
    // (t + OFF·j') mod NS ascending) are j' >= w0 = ceil((NS − t)/OFF); when w0 < KM the
    // order wraps and is cut there into chain A = w0 .. KM−1 (ch 0) and B = 0 .. w0−1
    // (ch 1), else one chain 0 .. KM−1
    struct Link {
        int ch, pos, len;
        bool wrap;
    };
    // Walked without divisions (a runtime % NS and / OFF per use cost ~50 SALU
    // instructions each, in every wave): the step's slice t and w0 = ceil((NS − t)/OFF)
    // as w0 and r0 = NS − t − (w0 − 1)·OFF in [1, OFF], advanced by one slice per step.
    struct Walk {
        int t, w0, r0;
    };
    const int w0_at0 = (NS + OFF - 1) / OFF, r0_at0 = NS - (w0_at0 - 1) * OFF;   // slice 0
    auto walk_at = [&](int t) {
        Walk s;
        s.t = t;
        s.w0 = (NS - t + OFF - 1) / OFF;
        s.r0 = NS - t - (s.w0 - 1) * OFF;
        return s;
    };
    auto advance = [&](const Walk& s) {
        Walk n;
        if (s.t + 1 == NS) {
            n.t = 0;
            n.w0 = w0_at0;
            n.r0 = r0_at0;
        } else {
            n.t = s.t + 1;
            n.w0 = s.r0 == 1 ? s.w0 - 1 : s.w0;
            n.r0 = s.r0 == 1 ? OFF : s.r0 - 1;
        }
        return n;
    };
    auto link_of = [&](const Walk& s) {
        const int w0 = s.w0;
        Link L;
        L.wrap = w0 < KM;
        L.ch = L.wrap && j < w0 ? 1 : 0;
        L.pos = L.wrap && j >= w0 ? j - w0 : j;
        L.len = !L.wrap ? KM : L.ch ? w0 : KM - w0;
        return L;
    };
    // a publish after the step's sums left: the chain's count, or for the tail of a
    // wrapped slice's chain an add to the slice's fin word (no return value: a returning
    // atomic would make this wave wait for the step's running-sum loads).  fin == 2
    // after the launch means both tails stored their totals: chain B's tail found A
    // unfinished, stored instead of writing dQ, and flagged the launch (comb) so that
    // bwd_dq_fast adds them.  Every publish counts as progress of the slab: prog[j] takes
    // the number of steps done, which grows with every publish (lane 0, s_hc.pub).
    auto publish = [&](unsigned steps) {
        // every word read at once (one LDS round trip on wave 0 after B2, not a chain)
        LHoff* const h = hc();
        const unsigned pk = h->pub;
        gu32* const c0 = h->cnt[0];
        gu32* const c1 = h->cnt[1];
        gu32* const fn = h->fin;
        gu32* const cm = h->comb;
        gu32* const pg = h->prog;
        const int kind = pk & 3u, chp = (pk >> 2) & 1u, posp = (pk >> 3) & 511u, tp = pk >> 12;
        if (kind == 1) {
            st_agent((chp ? c1 : c0) + tp, (unsigned)(posp + 1));
        } else if (kind == 2) {
            __hip_atomic_fetch_add(fn + tp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (chp == 1) st_agent(cm, 1u);
        }
        if (kind != 0) st_agent(pg + j, steps);
    };
    auto load_rowc = [&](int t) {
        const int q = t * 64 + (tid & 63);
        float v = 0.0f;
        if (tid < 64) v = q < N ? nlse[q] : kNegInf;
        else if (tid < 128) v = q < N ? nDg[q] : 0.0f;
        return v;
    };

    // ---- prologue: K images (once), the first slice, V fragments of this lane's key ----
    Walk cur = walk_at(slice_of(0));
    int t = cur.t;
    {
        const float rc = load_rowc(t);
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4) dma_image8<D>(krs, kimg + i4 * KSUB, Nk, key0 + 64 * i4, wave, lane);
        dma_image8<D>(qrs, qimg, N, t * 64, wave, lane);
        dma_image8<DV>(ors, oimg, N, t * 64, wave, lane);
        if (tid < 128) rowc[tid] = rc;
    }
    F8 vf[DV / 16];
#pragma unroll
    for (int s = 0; s < DV / 16; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const T x = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b16(vrs, ((16 * s + 8 * h + e) * Nk + kj) * 2, 0, 0));
            vf[s][e] = key_ok ? x : (T)0.0f;
        }
    f32x16 dk[D / 32], dv[DV / 32];
#pragma unroll
    for (int cb = 0; cb < D / 32; ++cb)
#pragma unroll
        for (int x = 0; x < 16; ++x) dk[cb][x] = 0.0f;
#pragma unroll
    for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
        for (int x = 0; x < 16; ++x) dv[cb][x] = 0.0f;
    const char* const kmine = kimg + (wave >> 1) * KSUB;   // the 64-key image holding this wave's keys
    const int ktb = wave & 1;
    const int dsrow = 32 * wave + sig32(r);                  // this lane's dSᵀ row
    const int cbq = wave % (D / 32), uq = wave / (D / 32);   // this wave's dQᵀ tile (wave < NTQ)

    // the prologue's loads have landed: no LDS-DMA the compiler knows of is pending in
    // the loop (its DMA is asm), so it adds no vmcnt(0) before the loop's LDS reads
    vm_wait<0>();
    // L2-local hand-off: once the next member (j + 1, the reader of every running sum
    // this one hands on) is known to run on this member's XCD, the sums are stored
    // plainly and stay in that XCD's L2, where its sc1 loads (L1 bypass, L2-served) find
    // them; until then — nothing waits for it: lane 0 looks for its XCD word once per
    // step while it is missing — sc1 stores (L2 write-through, dropped) as everywhere
    // else.  A chain's tail stores sc1 always.
    __shared__ unsigned s_local;       // read after B2 of each step
    __shared__ unsigned s_direct[2];   // chain B's tail of step i's slice: A had finished (slot i & 1)
    auto look_next = [&]() {           // lane 0
        LHoff* const h = hc();
        if (h->next_known) return;
        const unsigned x = ld_agent(h->xccw + j + 1);
        if (x != 0u) {
            h->next_known = 1u;
            s_local = x == my_xcc() ? 1u : 0u;
        }
    };
    if (tid == 0) {
        s_local = 0u;
        look_next();
    }

    bool pub_prev = false;   // the last step left a publish for lane 0 (kind in s_hc.pub)
    for (int i = 0; i < NS; ++i) {
        t = cur.t;
        const Link lk = link_of(cur);
        const Walk nxt = advance(cur);
        const int pos = lk.pos;
        const int tq = opaque(tid), lq = tq & 63, rq = lq & 31, hq = lq >> 5;   // re-derived per step
        const bool tail = pos == lk.len - 1;
        const bool btail = lk.wrap && tail && lk.ch == 1;   // chain B's tail: makes A + B when A is done
        // B1: this slice's images landed; lane 0 has seen the predecessor's count for
        // slice t (polled at the end of the previous step's dQ phase, or here for the
        // first step; the barrier releases the other waves' sum loads).  The previous
        // step's running-sum stores (this wave's last >= 4 vector-memory ops) may still
        // be in flight: every wave drains them in the middle of phase A and their count
        // is published after B2.  (vmcnt retires in issue order; a poll load behind
        // those stores would wait for them, hence the poll's place.)
        const bool has_tile = NTQ >= 8 || wave < NTQ;
        if (has_tile && i > 0 && !(abl & 18)) __builtin_amdgcn_s_waitcnt(0x0F74);   // vmcnt(4)
        else __builtin_amdgcn_s_waitcnt(0x0F70);                                    // vmcnt(0)
        if (i == 0 && tid == 0 && !(abl & 1)) {
            if (pos > 0) poll(lk.ch, t, pos);
            if (btail) s_direct[0] = !hc()->nodirect && ld_agent(hc()->fin + t) >= 1u ? 1u : 0u;
        }
        __syncthreads();
        BWD_STAMP(0);

        // ---- S, dP, P, dS; dVᵀ, dKᵀ updates; dSᵀ into LDS ----
        const int pofs = lk.ch * pchain4 + (t * NTQ + wave) * 4096 + lq * 16;
        const bool ldpin = pos > 0 && has_tile && !(abl & 10);
        u32x4 pin[4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            f32x16 sa, dp;
            const f32x4* Lq = (const f32x4*)(rowc + u * 32 + 8 * h);
            const f32x4* Dq = (const f32x4*)(rowc + 64 + u * 32 + 8 * h);
            const f32x4 l0 = Lq[0], l1 = Lq[1], l2 = Lq[4], l3 = Lq[5];
            const f32x4 d0 = Dq[0], d1 = Dq[1], d2 = Dq[4], d3 = Dq[5];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                sa[e] = l0[e]; sa[4 + e] = l1[e]; sa[8 + e] = l2[e]; sa[12 + e] = l3[e];
                dp[e] = d0[e]; dp[4 + e] = d1[e]; dp[8 + e] = d2[e]; dp[12 + e] = d3[e];
            }
#pragma unroll
            for (int s = 0; s < D / 16; ++s) sa = mfma32x32x16(trfrag(qimg, u, s), trfrag(kmine, ktb, s), sa);
#pragma unroll
            for (int s = 0; s < DV / 16; ++s) dp = mfma32x32x16(trfrag(oimg, u, s), vf[s], dp);
            if (u == 1) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): last step's sums stored
            F8 pf[2], dsf[2];
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const float pr = key_ok ? exp2_fast(sa[x] * c) : 0.0f;
                pf[x >> 3][x & 7] = (T)pr;
                dsf[x >> 3][x & 7] = (T)(pr * dp[x]);
            }
#pragma unroll
            for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) dv[cb] = mfma32x32x16(rowfrag(oimg, cb, u, s2), pf[s2], dv[cb]);
#pragma unroll
            for (int cb = 0; cb < D / 32; ++cb)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) dk[cb] = mfma32x32x16(rowfrag(qimg, cb, u, s2), dsf[s2], dk[cb]);
            // dSᵀ row kj: queries 32u + 16 s2 + 8h + {0..7}
#pragma unroll
            for (int s2 = 0; s2 < 2 && !(abl & 32); ++s2)
                *(F8*)(dsimg + dsrow * 128 + (((4 * u + 2 * s2 + h) ^ swzds(dsrow)) * 16)) = dsf[s2];
        }

        BWD_STAMP(8);
        // running sum of the members before this one (sc1 loads, after B1).  Loaded
        // whether or not this member is the chain's head (which adds nothing), and the
        // DMA and row constants below are unconditional too: a straight-line step
        // lets the compiler count vmcnt for the sums past the DMA instead of vmcnt(0).
        // lane 0 polls for the NEXT step's slice here: every wave's queue is empty
        // (drained in the middle of this phase), so the poll pays only its own latency,
        // and barriers B2 and B1 order it before every wave's sum loads of that step
        if (wave == 0 && i + 1 < NS && !(abl & 1)) {
            const int tn = nxt.t;
            const Link ln = link_of(nxt);
            if (tq == 0) {
                look_next();
                // a chain-B tail reads chain A's fin word with its poll (one round
                // trip for both; read again if A was not done then)
                const bool bt = ln.wrap && ln.ch == 1 && ln.pos == ln.len - 1;
                gu32* const fw = hc()->fin + tn;
                const unsigned f0 = bt ? ld_agent(fw) : 0u;
                if (ln.pos > 0) poll(ln.ch, tn, ln.pos);
                if (bt) s_direct[(i + 1) & 1] = !hc()->nodirect && (f0 >= 1u || ld_agent(fw) >= 1u) ? 1u : 0u;
            }
        }
        if (has_tile && !(abl & 10)) {
            pin[0] = load16_sc1_asm<0>(pdesc, pofs);
            pin[1] = load16_sc1_asm<1024>(pdesc, pofs);
            pin[2] = load16_sc1_asm<2048>(pdesc, pofs);
            pin[3] = load16_sc1_asm<3072>(pdesc, pofs);
        }
        // a chain-B tail at d, dv <= 64 loads chain A's total here too, before it knows
        // (after B2) whether A had finished at its poll: used only if it had (then the
        // poll, earlier in program order, saw A's publish, which follows A's stores),
        // and counted with the running sum (vm_wait<NDMA>).  At 128 its 16 registers
        // would spill across the dQ phase: loaded after that phase instead.
        constexpr bool kPrefA = D <= 64 && DV <= 64;
        u32x4 pa[4];
        if (kPrefA && has_tile && btail && !(abl & 10)) {
            const int pofa = pofs - pchain4;
            pa[0] = load16_sc1_asm<0>(pdesc, pofa);
            pa[1] = load16_sc1_asm<1024>(pdesc, pofa);
            pa[2] = load16_sc1_asm<2048>(pdesc, pofa);
            pa[3] = load16_sc1_asm<3072>(pdesc, pofa);
        }
        __syncthreads();   // B2: dSᵀ complete, the slice's images free, last step's sums stored
        BWD_STAMP(9);
        // chain B's tail: whether A's total was there at the poll (lane 0's word, ordered
        // by B2).  Read and waited for here: the dQ phase below counts its own LDS reads
        // by hand (lgkm_wait), so no compiler-issued LDS read may land among them.
        const unsigned dword = btail ? s_direct[i & 1] : 0u;
        const unsigned lword = s_local;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const bool direct = btail && __builtin_amdgcn_readfirstlane(dword) != 0u;
        const bool local = __builtin_amdgcn_readfirstlane(lword) != 0u;
        if (pub_prev && tid == 0) publish((unsigned)i);

        // next slice's images and row constants (land before the next B1)
        // (the last step reloads its own slice: harmless, nothing reads it)
        float rc;
        bool rc_in;
        {
            const int tn = i + 1 < NS ? nxt.t : t;
            const int q = tn * 64 + lq;
            rc = load4_asm((tq < 64 ? nlse : nDg) + (q < N ? q : N - 1));   // asm: counted below
            rc_in = q < N;
            if (!(abl & 64)) {
                dma_image8_asm<D>(qdesc, qimg, N, tn * 64, wave, lq);
                dma_image8_asm<DV>(odesc, oimg, N, tn * 64, wave, lq);
            }
        }

        // ---- dQᵀ tile (features 32 cbq.., queries 32 uq..) over the 256 keys ----
        if (has_tile) {
            f32x16 acc;
#pragma unroll
            for (int x = 0; x < 16; ++x) acc[x] = 0.0f;
            // asm LDS reads (see lds_b128_at), one step ahead of the MFMA: the DMA
            // just issued and the running-sum loads stay in flight meanwhile
            uint32_t ka[4];
            const int rswq = swz16(rq);
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4)
                ka[q4] = lds_addr(kimg + (cbq * 32 + rq) * 128 + ((((q4 >> 1) * 4 + 2 * (q4 & 1) + hq) ^ rswq) * 16));
            const int qqq = (lq & 15) >> 2, ppq = lq & 3, khq = (lq >> 4) & 1;
            const int sgq = (ppq == 1) ? 2 : (ppq == 2) ? 1 : ppq;
            const uint32_t da = lds_addr(dsimg + (8 * hq + qqq) * 128 +
                                         (((uq * 4 + khq * 2 + (sgq >> 1)) ^ swzds(8 * hq + qqq)) * 16) + (sgq & 1) * 8);
            u32x4 fa[2];
            s16x4 flo[2], fhi[2];
            auto issue = [&](auto kc) {
                constexpr int kk = decltype(kc)::value;
                fa[kk & 1] = lds_b128_at<(kk >> 2) * KSUB>(ka[kk & 3]);
                flo[kk & 1] = lds_tr16_at<2048 * kk>(da);
                fhi[kk & 1] = lds_tr16_at<2048 * kk + 512>(da);
            };
            issue(std::integral_constant<int, 0>{});
            static_for<16>([&](auto kc) {
                constexpr int kk = decltype(kc)::value;
                if constexpr (kk + 1 < 16) {
                    issue(std::integral_constant<int, kk + 1>{});
                    lgkm_wait<3>();
                } else {
                    lgkm_wait<0>();
                }
                reg_fence(fa[kk & 1]);
                reg_fence(flo[kk & 1]);
                reg_fence(fhi[kk & 1]);
                const F4 lo = __builtin_bit_cast(F4, flo[kk & 1]);
                const F4 hi = __builtin_bit_cast(F4, fhi[kk & 1]);
                acc = mfma32x32x16(__builtin_bit_cast(F8, fa[kk & 1]), __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7),
                                   acc);
            });
            // the sums (asm loads): all but this wave's NDMA DMA ops retired
            if (!(abl & 64)) vm_wait<NDMA>(); else vm_wait<0>();
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4) reg_fence(pin[c4]);
            reg_fence(rc);
            // the next slice's row constants (phase A's reads of rowc ended at B2)
            if (tq < 128) lds_w32(rowc + tq, rc_in ? rc : (tq < 64 ? kNegInf : 0.0f));
            if (ldpin) {
#pragma unroll
                for (int c4 = 0; c4 < 4; ++c4)
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[4 * c4 + e] += __uint_as_float(pin[c4][e]);
            }
            // chain B's tail with A finished: A's total (its tail's sc1 stores, published
            // through fin before this step's poll) in, after this chain's own sum
            if (direct) {
                if constexpr (!kPrefA) {
                    const int pofa = pofs - pchain4;
                    pa[0] = load16_sc1_asm<0>(pdesc, pofa);
                    pa[1] = load16_sc1_asm<1024>(pdesc, pofa);
                    pa[2] = load16_sc1_asm<2048>(pdesc, pofa);
                    pa[3] = load16_sc1_asm<3072>(pdesc, pofa);
                    vm_wait<0>();
                }
#pragma unroll
                for (int c4 = 0; c4 < 4; ++c4) {
                    reg_fence(pa[c4]);
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[4 * c4 + e] += __uint_as_float(pa[c4][e]);
                }
            }
            if ((tail && !lk.wrap) || direct) {
                // 32-bit lane offset + scalar row offset (no hoisted 64-bit addresses)
                const int q = t * 64 + 32 * uq + sig32(rq);
                const auto qo = bslab<T>(p.dQ, (int64_t)b * N * D, (int64_t)N * D);
                const int vo = q < N ? ((cbq * 32 + 4 * hq) * N + q) * 2 : N * D * 2;   // past N: dropped
#pragma unroll
                for (int x = 0; x < 16; ++x)
                    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (T)(acc[x] * p.scale)), qo, vo,
                                                          ((x & 3) + 8 * (x >> 2)) * N * 2, 0);
            } else if (!(abl & 18)) {
#pragma unroll
                for (int c4 = 0; c4 < 4; ++c4) {
                    const u32x4 v4 = {__float_as_uint(acc[4 * c4]), __float_as_uint(acc[4 * c4 + 1]),
                                      __float_as_uint(acc[4 * c4 + 2]), __float_as_uint(acc[4 * c4 + 3])};
                    if (local && !tail) __builtin_amdgcn_raw_buffer_store_b128(v4, prs, pofs + c4 * 1024, 0, 0);
                    else __builtin_amdgcn_raw_buffer_store_b128(v4, prs, pofs + c4 * 1024, 0, 16);   // sc1
                }
            }
        }
        BWD_STAMP(10);
        // publish kind: 0 none (dQ written), 1 chain count, 2 fin word (a wrapped chain's tail)
        const unsigned kind = (tail && !lk.wrap) || direct ? 0u : tail ? 2u : 1u;
        pub_prev = kind != 0u;
        if (tid == 0) hc()->pub = kind | (unsigned)lk.ch << 2 | (unsigned)pos << 3 | (unsigned)t << 12;
        cur = nxt;
    }
    if (pub_prev) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) publish((unsigned)NS);
    }
    if (key_ok) {
        const auto ko = bslab<T>(p.dK, (int64_t)b * Nk * D, (int64_t)Nk * D);
        const auto vo = bslab<T>(p.dV, (int64_t)b * Nk * DV, (int64_t)Nk * DV);
        const int lo = (4 * h * Nk + kj) * 2;
#pragma unroll
        for (int cb = 0; cb < D / 32; ++cb)
#pragma unroll
            for (int x = 0; x < 16; ++x)
                __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (T)(dk[cb][x] * p.scale)), ko, lo,
                                                      (cb * 32 + (x & 3) + 8 * (x >> 2)) * Nk * 2, 0);
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int x = 0; x < 16; ++x)
                __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (T)dv[cb][x]), vo, lo,
                                                      (cb * 32 + (x & 3) + 8 * (x >> 2)) * Nk * 2, 0);
    }
}

#ifdef FA_BWD_STAMP4
extern "C" int fa_debug_bwd_stamps(unsigned long long* out, int n) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bwd_stamp), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif
thread_local int g_bwd_force_generic = 0;   // benchmark knob
thread_local int g_bwd_mode = 0;            // 0 auto, 1 split passes, 2 single pass where the shape allows
thread_local int g_bwd_l2local = -1;        // bwd_fused: L2-local hand-off when a slab sits on one XCD
                                            // (-1 auto: at d, dv <= 64; 0 never; 1 always)
thread_local int g_bwd_hoff = 3;            // bwd_fused: step offset between consecutive members
thread_local int g_bwd_stall_us = kStallUs; // bwd_fused: no-progress bound of a poll (us)
thread_local int g_bwd_nodirect = 0;         // bwd_fused (tests): every wrapped slice left to bwd_dq_fast's combine
thread_local int g_bwd_xcd = -1;            // bwd_fused: one XCD per slab where eligible (-1 auto, 0 never)

template <class T, int D, int DV>
static hipError_t launch_fast_dd(BwdParams p, hipStream_t s) {
    const bool fused = p.part != nullptr;
    if (fused) {   // single pass; dQ pass below only after a hand-off timeout
        p.total_wg = p.nkb * p.batch;
        hipLaunchKernelGGL((bwd_fused<T, D, DV>), dim3((unsigned)p.total_wg), dim3(512), 0, s, p);
        const FusedFlags ff = fused_flags(p.batch, p.nqt, p.nkb);
        p.guard = p.err;
        p.sguard = p.flags + ff.serr;
        p.cguard = p.hdr + 3;
        p.fin = p.flags + ff.fin;
    }
    p.nblk = (p.N + 127) / 128;
    p.total_wg = p.nblk * p.batch;
    hipLaunchKernelGGL((bwd_dq_fast<T, D, DV>), dim3((unsigned)p.total_wg), dim3(256), 0, s, p);
    if (!fused) {
        p.nblk = (p.Nk + 127) / 128;
        p.total_wg = p.nblk * p.batch;
        hipLaunchKernelGGL((bwd_dkdv_fast<T, D, DV>), dim3((unsigned)p.total_wg), dim3(256), 0, s, p);
    }
    return hipGetLastError();
}
template <class T, int D>
static hipError_t launch_fast_d(const BwdParams& p, hipStream_t s) {
    switch (p.dv) {
        case 32: return launch_fast_dd<T, D, 32>(p, s);
        case 64: return launch_fast_dd<T, D, 64>(p, s);
        case 128: return launch_fast_dd<T, D, 128>(p, s);
    }
    return hipErrorInvalidValue;
}
template <class T>
static hipError_t launch_fast(const BwdParams& p, hipStream_t s) {
    switch (p.d) {
        case 32: return launch_fast_d<T, 32>(p, s);
        case 64: return launch_fast_d<T, 64>(p, s);
        case 128: return launch_fast_d<T, 128>(p, s);
    }
    return hipErrorInvalidValue;
}

// --------------------------------------------------------------------------
// launcher
// --------------------------------------------------------------------------
// --------------------------------------------------------------------------
// Padded fast path: 16-bit shapes the MFMA kernels do not take directly (N or
// Nk not a multiple of 8, d or dv not 32 / 64 / 128) are copied into zero-padded
// workspace slabs (N -> N8, Nk -> Nk8, d, dv -> their class) and run on the fast
// kernels.  Zero keys and values are exact there: with the forward's lse they add
// P·0 to dP and dS·0 to dQ, and their own dK / dV rows are dropped; padded
// queries carry dO = O = 0 (so dS = 0) and l = 1, m = 0 (finite P, no NaN).
// --------------------------------------------------------------------------
static bool cls_dim(int64_t x) { return x == 32 || x == 64 || x == 128; }
static bool shape_fast(int dtype, int64_t N, int64_t Nk, int64_t d, int64_t dv) {
    return dtype != FA_DTYPE_F32 && dtype != FA_DTYPE_F64 && cls_dim(d) && cls_dim(dv) && N % 8 == 0 && Nk % 8 == 0 &&
           N * d * 2 < INT32_MAX && Nk * d * 2 < INT32_MAX && N * dv * 2 < INT32_MAX && Nk * dv * 2 < INT32_MAX;
}
struct BwdPad {
    bool on = false;
    int64_t Np = 0, Nkp = 0, Dp = 0, DVp = 0;
    size_t bytes = 0;
};
static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
static BwdPad pad_plan(int dtype, int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch) {
    BwdPad pl;
    if (dtype == FA_DTYPE_F32 || dtype == FA_DTYPE_F64 || d > kMaxHeadDim || dv > kMaxHeadDim ||
        shape_fast(dtype, N, Nk, d, dv))
        return pl;
    pl.Np = (N + 7) / 8 * 8;
    pl.Nkp = (Nk + 7) / 8 * 8;
    pl.Dp = head_dim_class(d);
    pl.DVp = head_dim_class(dv);
    if (!shape_fast(dtype, pl.Np, pl.Nkp, pl.Dp, pl.DVp) || pl.Np * batch > INT32_MAX / 2 ||
        pl.Nkp * batch > INT32_MAX / 2)
        return pl;
    pl.on = true;
    const size_t q = al256((size_t)(pl.Np * pl.Dp * batch) * 2), k = al256((size_t)(pl.Nkp * pl.Dp * batch) * 2);
    const size_t v = al256((size_t)(pl.Nkp * pl.DVp * batch) * 2), o = al256((size_t)(pl.Np * pl.DVp * batch) * 2);
    const size_t lm = al256((size_t)(pl.Np * batch) * 4);
    pl.bytes = 2 * q + 2 * k + 2 * v + 2 * o + 2 * lm;   // Q dQ, K dK, V dV, O dO, l m
    return pl;
}

// Single-pass plan (bwd_fused) on the shape the fast kernels run (padded or not):
// K = ceil(Nk/256) members per slab, T = ceil(N/64) slices, step offset 3 (needs
// 3K <= T); K <= CUs, one XCD per slab when K <= CUs/8 and the slab count is a
// multiple of 8 (a slab's members then run together: speed, not correctness, which
// needs no co-residency); auto only when the grid fills the chip once.  Workspace: the hand-off words (FusedFlags), then the two chains'
// running fp32 dQ sums (2 x 4·N·d bytes per slab).
struct FusedPlan {
    bool on = false;
    int nkb = 0, nqt = 0, xcd = 0;
    size_t flag_bytes = 0, bytes = 0;
};
static FusedPlan fused_plan(int dtype, int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch,
                            hipStream_t s = nullptr) {
    FusedPlan f;
    if (dtype == FA_DTYPE_F32 || dtype == FA_DTYPE_F64 || g_bwd_mode == 1 || g_bwd_force_generic || !shape_fast(dtype, N, Nk, d, dv)) return f;
    const int64_t K = (Nk + 255) / 256, T = (N + 63) / 64;
    const int cus = device_cus(s);
    if (cus < 8 || g_bwd_hoff * K > T || K > cus || batch * K > INT32_MAX / 2 || 2 * T * (d / 16) * 4096 >= INT32_MAX ||
        T >= (1 << 20))   // a slice index fits the 20 bits bwd_fused packs it in
        return f;
    const int xcd = (K <= cus / 8 && batch % 8 == 0 && g_bwd_xcd != 0) ? 1 : 0;
    if (g_bwd_mode == 0) {
        // auto: the grid fills the chip, and K divides the CUs a slab's members are dealt
        // over (one XCD's, or the chip's), so no slab waits part-resident behind another
        if (batch * K < cus || (xcd ? cus / 8 : cus) % K != 0) return f;
    }
    f.on = true;
    f.nkb = (int)K;
    f.nqt = (int)T;
    f.xcd = xcd;
    f.flag_bytes = al256((size_t)fused_flags(batch, T, K).words * 4);   // FusedFlags
    f.bytes = f.flag_bytes + al256((size_t)(2 * batch * T * (d / 16)) * 4096) + 256;   // two chains' running sums
    return f;
}

size_t dense_bwd_workspace(int dtype, int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch) {
    if (dtype == FA_DTYPE_F64) return kBwdHdrBytes + (size_t)(2 * N * batch * sizeof(double) + 256);   // nD, nlse in double
    const BwdPad pl = pad_plan(dtype, N, Nk, d, dv, batch);
    const int64_t rows = pl.on ? pl.Np : N;
    const FusedPlan fz = pl.on ? fused_plan(dtype, pl.Np, pl.Nkp, pl.Dp, pl.DVp, batch)
                               : fused_plan(dtype, N, Nk, d, dv, batch);
    return kBwdHdrBytes + (size_t)(2 * rows * batch * sizeof(float) + 256) + (pl.on ? pl.bytes + 256 : 0) + fz.bytes;
}

// dst (Np, Cp, B) <- src (N, C, B), zero-filled
template <class T>
__global__ __launch_bounds__(256) void bwd_pad(const T* __restrict__ src, T* __restrict__ dst, int N, int C,
                                               int Np, int Cp, int64_t total) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    const int n = (int)(e % Np);
    const int64_t bc = e / Np;
    const int c = (int)(bc % Cp);
    const int64_t b = bc / Cp;
    dst[e] = (n < N && c < C) ? src[(b * C + c) * N + n] : (T)0.0f;
}
// dst (N, C, B) <- src (Np, Cp, B)
template <class T>
__global__ __launch_bounds__(256) void bwd_unpad(const T* __restrict__ src, T* __restrict__ dst, int N, int C,
                                                 int Np, int Cp, int64_t total) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    const int n = (int)(e % N);
    const int64_t bc = e / N;
    const int c = (int)(bc % C);
    const int64_t b = bc / C;
    dst[e] = src[(b * Cp + c) * Np + n];
}
// l, m (N, 1, B) -> (Np, 1, B); padded queries get l = 1, m = 0
__global__ __launch_bounds__(256) void bwd_pad_lm(const float* __restrict__ l, const float* __restrict__ m,
                                                  float* __restrict__ lp, float* __restrict__ mp, int N, int Np,
                                                  int64_t total) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    const int n = (int)(e % Np);
    const int64_t b = e / Np;
    lp[e] = n < N ? l[b * N + n] : 1.0f;
    mp[e] = n < N ? m[b * N + n] : 0.0f;
}
template <class T>
static hipError_t pad_launch(const void* src, void* dst, int64_t N, int64_t C, int64_t Np, int64_t Cp, int64_t B,
                             hipStream_t s) {
    const int64_t total = Np * Cp * B;
    hipLaunchKernelGGL(bwd_pad<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, (const T*)src, (T*)dst,
                       (int)N, (int)C, (int)Np, (int)Cp, total);
    return hipGetLastError();
}
template <class T>
static hipError_t unpad_launch(const void* src, void* dst, int64_t N, int64_t C, int64_t Np, int64_t Cp, int64_t B,
                               hipStream_t s) {
    const int64_t total = N * C * B;
    hipLaunchKernelGGL(bwd_unpad<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, (const T*)src, (T*)dst,
                       (int)N, (int)C, (int)Np, (int)Cp, total);
    return hipGetLastError();
}

template <class T, class A = float>
static hipError_t launch_generic(const BwdParams& p, hipStream_t s) {
    const int64_t nq = ((int64_t)p.N + kGT - 1) / kGT * p.batch;
    const int64_t nk = ((int64_t)p.Nk + kGT - 1) / kGT * p.batch;
    const size_t rows = kGT * (2 * (p.d + 1) + 2 * (p.dv + 1));
    const size_t sm_dq = sizeof(A) * (rows + kGT * (kGT + 1));
    const size_t sm_kv = sizeof(A) * (rows + 2 * kGT * (kGT + 1));
    // > 64 KiB of dynamic LDS at d = dv = 128 (gfx950 has 160 KiB per CU)
    (void)hipFuncSetAttribute((const void*)bwd_generic_dq<T, A>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm_dq);
    (void)hipFuncSetAttribute((const void*)bwd_generic_dkdv<T, A>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm_kv);
    hipLaunchKernelGGL((bwd_generic_dq<T, A>), dim3((unsigned)nq), dim3(kGThreads), sm_dq, s, p);
    hipLaunchKernelGGL((bwd_generic_dkdv<T, A>), dim3((unsigned)nk), dim3(kGThreads), sm_kv, s, p);
    return hipGetLastError();
}

template <class T>
static hipError_t launch_typed(const BwdParams& p, hipStream_t s, bool fast) {
    const int64_t total = (int64_t)p.N * p.batch;
    bool vec = false;
    if constexpr (sizeof(T) == 2) {
        vec = p.N % 8 == 0 && ((uintptr_t)p.O & 15u) == 0 && ((uintptr_t)p.dO & 15u) == 0;
        if (vec) hipLaunchKernelGGL(bwd_prepass_v<T>, dim3((unsigned)((total / 8 + 255) / 256)), dim3(256), 0, s, p);
    }
    if (!vec) hipLaunchKernelGGL(bwd_prepass<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if constexpr (!std::is_same<T, float>::value) {
        if (fast) return launch_fast<T>(p, s);
    } else {
        if (fast) return launch_f32_mfma(p, s);
    }
    return launch_generic<T>(p, s);
}

static bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15u) == 0; }

// Single-pass state in the workspace at w: per-slice counters (zeroed here), then the
// running dQ sums.  The status word is hdr[1], which the pre-pass sets to hdr_err.
static hipError_t fused_setup(BwdParams& p, const FusedPlan& fz, char* w, hipStream_t s) {
    p.flags = (unsigned*)w;
    p.part = (float*)(w + fz.flag_bytes);
    p.nkb = fz.nkb; p.nqt = fz.nqt; p.xcd = fz.xcd;
    p.hdr_plan = 1;
    // mode 3 (tests): the timeout word starts set, so every poll gives up and the
    // guarded dQ pass must recompute dQ of every slab
    p.hdr_err = g_bwd_mode == 3 ? 1u : 0u;
    // L2-local hand-off: +6 % at d = dv = 64, -1 % at 128, where a slice's running
    // sums (32 KB) in flight over three steps fill most of the 4-MB L2 that also
    // serves the slab's Q / dO (profiles/r04_bwd_handoff_modes.log)
    p.l2local = g_bwd_l2local >= 0 ? g_bwd_l2local : (p.d <= 64 && p.dv <= 64 ? 1 : 0);
    p.hoff = g_bwd_hoff;
    p.stall_ticks = g_bwd_stall_us * 100;
    p.nodirect = g_bwd_nodirect;
#ifdef FA_BWD_ABL
    p.ablate = g_bwd_mode == 7 ? 8 : g_bwd_mode == 8 ? 16 : g_bwd_mode == 9 ? 32 : g_bwd_mode == 10 ? 64
             : g_bwd_mode == 11 ? 64 | 3 : g_bwd_mode >= 4 ? g_bwd_mode - 3 : 0;
#endif
    hipError_t e = hipMemsetAsync(w, 0, fz.flag_bytes, s);
    if (e == hipSuccess && g_bwd_mode == 3)
        e = hipMemsetD32Async((hipDeviceptr_t)(p.flags + fused_flags(p.batch, fz.nqt, fz.nkb).serr), 1u, (size_t)p.batch, s);
    return e;
}

int dense_bwd_handoff_status(const void* workspace, size_t workspace_bytes, hipStream_t s, int* status,
                             const char** why) {
    const uintptr_t ws0 = ((uintptr_t)workspace + 255) & ~(uintptr_t)255;
    if (!workspace || ws0 + 8 > (uintptr_t)workspace + workspace_bytes) {
        *why = "workspace missing or smaller than its header";
        return FA_ERR_INVALID_ARG;
    }
    unsigned h[2] = {0u, 0u};
    hipError_t e = hipMemcpyAsync(h, (const void*)ws0, sizeof(h), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    if ((h[0] & 0xFFFFFF00u) != kBwdHdrMagic) {
        *why = "workspace holds no fa_dense_bwd header (not the workspace of an fa_dense_bwd call)";
        return FA_ERR_INVALID_ARG;
    }
    *status = (h[0] & 0xFFu) == 1u ? (h[1] != 0u ? 1 : 0) : -1;
    return FA_OK;
}

int launch_dense_bwd(const DenseBwdArgs& a, hipStream_t s, const char** why) {
    if (a.d > kMaxHeadDim || a.dv > kMaxHeadDim) {
        *why = "head dimension exceeds the compiled maximum (128)";
        return FA_ERR_UNSUPPORTED;
    }
    if (a.N * a.d > INT32_MAX || a.Nk * a.d > INT32_MAX || a.N * a.dv > INT32_MAX ||
        a.Nk * a.dv > INT32_MAX || a.N * a.batch > INT32_MAX / 2 || a.Nk * a.batch > INT32_MAX / 2) {
        *why = "extent exceeds 2^31 elements";
        return FA_ERR_UNSUPPORTED;
    }
    BwdParams p;
    p.Q = a.Q; p.K = a.K; p.V = a.V; p.O = a.O; p.dO = a.dO; p.l = a.l; p.m = a.m;
    p.dQ = a.dQ; p.dK = a.dK; p.dV = a.dV;
    const uintptr_t ws0 = ((uintptr_t)a.workspace + 255) & ~(uintptr_t)255;
    p.hdr = (unsigned*)ws0;
    p.err = p.hdr + 1;
    const uintptr_t ws = ws0 + kBwdHdrBytes;
    p.nD = (float*)ws;
    p.nlse = p.nD + a.N * a.batch;
    p.N = (int)a.N; p.Nk = (int)a.Nk; p.d = (int)a.d; p.dv = (int)a.dv; p.batch = (int)a.batch;
    p.scale = a.scale;
    p.scale_log2 = a.scale * kLog2e;
    hipError_t e;
    if (a.dtype == FA_DTYPE_F64) {
        // Float64: row statistics recomputed in double (not from the float32 l, m),
        // then the SIMT passes in double
        if (a.workspace_bytes < dense_bwd_workspace(a.dtype, a.N, a.Nk, a.d, a.dv, a.batch)) {
            *why = "workspace smaller than fa_dense_bwd_workspace()";
            return FA_ERR_WORKSPACE;
        }
        double* nD = (double*)ws;
        double* nlse = nD + a.N * a.batch;
        // plan 0; word 3 (a chain-B tail left its slice to the combine) belongs to the
        // current call like word 0, so it is cleared wherever word 0 is written; word 2
        // (the sticky give-up count) is left alone
        if ((e = hipMemsetD32Async((hipDeviceptr_t)p.hdr, kBwdHdrMagic, 1, s)) != hipSuccess ||
            (e = hipMemsetD32Async((hipDeviceptr_t)(p.hdr + 3), 0, 1, s)) != hipSuccess) {
            *why = hipGetErrorString(e);
            return FA_ERR_HIP;
        }
        p.nD = (float*)nD;
        p.nlse = (float*)nlse;
        p.scale64 = a.scale64 > 0.0 ? a.scale64 : (double)a.scale;
        const int rc = launch_f64_bwd_stats(a, nD, nlse, s, why);
        if (rc != FA_OK) return rc;
        if ((e = launch_generic<double, double>(p, s)) != hipSuccess) {
            *why = hipGetErrorString(e);
            return FA_ERR_HIP;
        }
        return FA_OK;
    }
    const bool fast = !g_bwd_force_generic && shape_fast(a.dtype, a.N, a.Nk, a.d, a.dv) &&
                      aligned16(a.Q) && aligned16(a.K) && aligned16(a.V) && aligned16(a.dO);
    const BwdPad pl = pad_plan(a.dtype, a.N, a.Nk, a.d, a.dv, a.batch);
    if (!fast && pl.on && !g_bwd_force_generic) {
        // padded fast path: workspace = [nD | nlse] (Np rows) then the padded slabs
        const int64_t B = a.batch;
        char* w = (char*)(ws + al256((size_t)(2 * pl.Np * B) * sizeof(float)));
        auto take = [&](size_t bytes) { void* q = w; w += al256(bytes); return q; };
        void* Qp = take((size_t)(pl.Np * pl.Dp * B) * 2);
        void* dQp = take((size_t)(pl.Np * pl.Dp * B) * 2);
        void* Kp = take((size_t)(pl.Nkp * pl.Dp * B) * 2);
        void* dKp = take((size_t)(pl.Nkp * pl.Dp * B) * 2);
        void* Vp = take((size_t)(pl.Nkp * pl.DVp * B) * 2);
        void* dVp = take((size_t)(pl.Nkp * pl.DVp * B) * 2);
        void* Op = take((size_t)(pl.Np * pl.DVp * B) * 2);
        void* dOp = take((size_t)(pl.Np * pl.DVp * B) * 2);
        float* lp = (float*)take((size_t)(pl.Np * B) * 4);
        float* mp = (float*)take((size_t)(pl.Np * B) * 4);
        if ((size_t)(w - (char*)a.workspace) > a.workspace_bytes) {
            *why = "workspace smaller than fa_dense_bwd_workspace()";
            return FA_ERR_WORKSPACE;
        }
        const FusedPlan fz = fused_plan(a.dtype, pl.Np, pl.Nkp, pl.Dp, pl.DVp, B, s);
        if (fz.on && (size_t)(w - (char*)a.workspace) + fz.bytes <= a.workspace_bytes &&
            (e = fused_setup(p, fz, w, s)) != hipSuccess) {
            *why = hipGetErrorString(e);
            return FA_ERR_HIP;
        }
        const bool half = a.dtype == FA_DTYPE_F16;
        auto pad = [&](const void* src, void* dst, int64_t N, int64_t C, int64_t Np, int64_t Cp) {
            return half ? pad_launch<f16>(src, dst, N, C, Np, Cp, B, s) : pad_launch<bf16>(src, dst, N, C, Np, Cp, B, s);
        };
        auto unpad = [&](const void* src, void* dst, int64_t N, int64_t C, int64_t Np, int64_t Cp) {
            return half ? unpad_launch<f16>(src, dst, N, C, Np, Cp, B, s) : unpad_launch<bf16>(src, dst, N, C, Np, Cp, B, s);
        };
        const int64_t tlm = pl.Np * B;
        if ((e = pad(a.Q, Qp, a.N, a.d, pl.Np, pl.Dp)) != hipSuccess ||
            (e = pad(a.K, Kp, a.Nk, a.d, pl.Nkp, pl.Dp)) != hipSuccess ||
            (e = pad(a.V, Vp, a.Nk, a.dv, pl.Nkp, pl.DVp)) != hipSuccess ||
            (e = pad(a.O, Op, a.N, a.dv, pl.Np, pl.DVp)) != hipSuccess ||
            (e = pad(a.dO, dOp, a.N, a.dv, pl.Np, pl.DVp)) != hipSuccess) {
            *why = hipGetErrorString(e);
            return FA_ERR_HIP;
        }
        hipLaunchKernelGGL(bwd_pad_lm, dim3((unsigned)((tlm + 255) / 256)), dim3(256), 0, s, a.l, a.m, lp, mp,
                           (int)a.N, (int)pl.Np, tlm);
        BwdParams q = p;
        q.Q = Qp; q.K = Kp; q.V = Vp; q.O = Op; q.dO = dOp; q.l = lp; q.m = mp;
        q.dQ = dQp; q.dK = dKp; q.dV = dVp;
        q.nlse = q.nD + pl.Np * B;
        q.N = (int)pl.Np; q.Nk = (int)pl.Nkp; q.d = (int)pl.Dp; q.dv = (int)pl.DVp;
        e = half ? launch_typed<f16>(q, s, true) : launch_typed<bf16>(q, s, true);
        if (e == hipSuccess && (e = unpad(dQp, a.dQ, a.N, a.d, pl.Np, pl.Dp)) == hipSuccess &&
            (e = unpad(dKp, a.dK, a.Nk, a.d, pl.Nkp, pl.Dp)) == hipSuccess)
            e = unpad(dVp, a.dV, a.Nk, a.dv, pl.Nkp, pl.DVp);
        if (e != hipSuccess) {
            *why = hipGetErrorString(e);
            return FA_ERR_HIP;
        }
        return FA_OK;
    }
    if (fast) {
        const FusedPlan fz = fused_plan(a.dtype, a.N, a.Nk, a.d, a.dv, a.batch, s);
        char* w = (char*)ws + al256((size_t)(2 * a.N * a.batch) * sizeof(float));
        if (fz.on && (size_t)(w - (char*)a.workspace) + fz.bytes <= a.workspace_bytes &&
            (e = fused_setup(p, fz, w, s)) != hipSuccess) {
            *why = hipGetErrorString(e);
            return FA_ERR_HIP;
        }
    }
    switch (a.dtype) {
        case FA_DTYPE_BF16: e = launch_typed<bf16>(p, s, fast); break;
        case FA_DTYPE_F16: e = launch_typed<f16>(p, s, fast); break;
        case FA_DTYPE_F32:   // fp32 MFMA kernels (exact fp32 products)
            e = launch_typed<float>(p, s, !g_bwd_force_generic &&
                                              a.N * a.batch < INT32_MAX / 2 && a.Nk * a.batch < INT32_MAX / 2);
            break;
        default: *why = "unknown dtype"; return FA_ERR_INVALID_ARG;
    }
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    return FA_OK;
}

}  // namespace fa
