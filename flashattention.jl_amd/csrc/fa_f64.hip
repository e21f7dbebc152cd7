// fa_f64.hip — Float64 dense forward (and the backward's Float64 row statistics).
//
// Float64 is the element type of the reference's own test and of every timing it
// publishes (test/test.jl:12 `rand(T, …)` with T = Float64; logs/compare1.txt), so
// a Julia caller passing Array{Float64} keeps its precision here instead of being
// rejected.  gfx950's fp64 matrix rate is a small fraction of its bf16 rate and
// no attention workload on this GPU runs in fp64, so this is the parity path, not
// a performance path: LDS-tiled SIMT in double, the reference's blockwise
// algorithm (src/dense.jl:21-102) with the FA-2 deferred normalisation of the
// other kernels:
//
//  * one workgroup = 256 threads = QB = 64 queries of one slab (16 when 64 would
//    leave CUs idle: 4x the workgroups); Q stays in LDS as a [feature][QB] image
//    (coalesced loads along tokens);
//  * keys stream in tiles of 32 ([feature][32] images);
//  * thread (qi, g), g < NG = 256/QB, scores keys KPG·g .. KPG·g + KPG − 1 of the
//    tile for query qi, the row max and row sum go through an [NG][QB] LDS
//    exchange, and the same thread then owns output channels g, g + NG, … of query
//    qi (the O rescale needs no exchange);
//  * exp / log in double; τ is resolved in double (1/√d, src/dense.jl:43).
//
// l and m leave as float32 (the C ABI's type for every dtype).  The backward does
// not use them at Float64: STATS = true runs the same sweep without V and writes
// −(m + ln l)/τ in double into the backward's workspace (fa_bwd.hip).
#include <math.h>

#include "fa_common.h"
#include "fa_internal.h"
#include "../../include/fa_hip.h"

namespace fa {

struct F64Params {
    const double *Q, *K, *V;
    double* O;
    float *l, *m;
    double* nlse;   // STATS: −(m + ln l)/τ per query, raw dot-product units [batch][N]
    int N, Nk, d, dv, nqb;
    double scale;
};

constexpr int kQB64 = 64;    // queries per workgroup (QB = 16 for grids smaller than the chip)
constexpr int kKB64 = 32;    // keys per tile
constexpr int kTh64 = 256;

__device__ __forceinline__ double dmax(double a, double b) { return __builtin_elementwise_maximum(a, b); }

static size_t f64_lds_bytes(int d, int dv, bool stats, int QB) {
    return sizeof(double) * ((size_t)QB * d + (size_t)kKB64 * d + (stats ? 0 : (size_t)kKB64 * dv) +
                             (stats ? 0 : (size_t)QB * (kKB64 + 1)) + 2 * kTh64);
}

// QB queries per workgroup, NG = 256/QB thread groups per query: group g scores
// keys KPG·g .. KPG·g + KPG−1 of each tile and owns output channels g, g + NG, ….
template <bool STATS, int QB>
__global__ __launch_bounds__(kTh64) void dense_fwd_f64(F64Params p) {
    constexpr int NG = kTh64 / QB, KPG = kKB64 / NG, OPER = kMaxHeadDim / NG;
    static_assert(KPG >= 1 && QB * NG == kTh64, "geometry");
    extern __shared__ __attribute__((aligned(16))) double sm64[];
    const int d = p.d, dv = p.dv, N = p.N, Nk = p.Nk;
    double* const sQ = sm64;                                    // [d][QB]
    double* const sK = sQ + QB * d;                             // [d][32]
    double* const sV = sK + kKB64 * d;                          // [dv][32]
    double* const sP = sV + (STATS ? 0 : kKB64 * dv);           // [QB][33]
    double* const red = sP + (STATS ? 0 : QB * (kKB64 + 1));    // [2][NG][QB]: tile max, tile sum
    const int b = blockIdx.x / p.nqb, q0 = (blockIdx.x - b * p.nqb) * QB;
    const int tid = threadIdx.x, qi = tid % QB, g = tid / QB;
    const double* __restrict__ Qb = p.Q + (int64_t)b * N * d;
    const double* __restrict__ Kb = p.K + (int64_t)b * Nk * d;
    const double* __restrict__ Vb = STATS ? nullptr : p.V + (int64_t)b * Nk * dv;

    for (int i = tid; i < QB * d; i += kTh64) {
        const int f = i / QB, q = i % QB;
        sQ[i] = q0 + q < N ? Qb[(int64_t)f * N + q0 + q] : 0.0;
    }
    double o[OPER];
#pragma unroll
    for (int i = 0; i < OPER; ++i) o[i] = 0.0;
    double m_run = -__builtin_huge_val(), l_run = 0.0;

    for (int k0 = 0; k0 < Nk; k0 += kKB64) {
        __syncthreads();   // the previous tile's K / V / P readers are done
        for (int i = tid; i < kKB64 * d; i += kTh64) {
            const int f = i >> 5, k = i & 31;
            sK[i] = k0 + k < Nk ? Kb[(int64_t)f * Nk + k0 + k] : 0.0;
        }
        if (!STATS)
            for (int i = tid; i < kKB64 * dv; i += kTh64) {
                const int f = i >> 5, k = i & 31;
                sV[i] = k0 + k < Nk ? Vb[(int64_t)f * Nk + k0 + k] : 0.0;
            }
        __syncthreads();

        // scores of keys KPG·g .. KPG·g + KPG−1 for query qi (s = τ qᵀk, src/dense.jl:77)
        double s[KPG];
#pragma unroll
        for (int j = 0; j < KPG; ++j) s[j] = 0.0;
        for (int f = 0; f < d; ++f) {
            const double qv = sQ[f * QB + qi];
            const double* kr = sK + f * kKB64 + KPG * g;
#pragma unroll
            for (int j = 0; j < KPG; ++j) s[j] = fma(qv, kr[j], s[j]);
        }
        double mx = -__builtin_huge_val();
#pragma unroll
        for (int j = 0; j < KPG; ++j) {
            s[j] = k0 + KPG * g + j < Nk ? s[j] * p.scale : -__builtin_huge_val();
            mx = dmax(mx, s[j]);
        }
        red[g * QB + qi] = mx;
        __syncthreads();
        // online update (src/dense.jl:78-91): every thread of query qi holds the same m, l
        double tmax = red[qi];
#pragma unroll
        for (int gg = 1; gg < NG; ++gg) tmax = dmax(tmax, red[gg * QB + qi]);
        const double m_new = dmax(m_run, tmax);
        const double alpha = exp(m_run - m_new);
        double ps = 0.0;
#pragma unroll
        for (int j = 0; j < KPG; ++j) {
            const double pj = exp(s[j] - m_new);
            ps += pj;
            if (!STATS) sP[qi * (kKB64 + 1) + KPG * g + j] = pj;
        }
        red[kTh64 + g * QB + qi] = ps;
        __syncthreads();
        double lt = 0.0;
#pragma unroll
        for (int gg = 0; gg < NG; ++gg) lt += red[kTh64 + gg * QB + qi];
        l_run = l_run * alpha + lt;
        m_run = m_new;
        if (!STATS) {
            double pr[kKB64];
#pragma unroll
            for (int k = 0; k < kKB64; ++k) pr[k] = sP[qi * (kKB64 + 1) + k];
#pragma unroll
            for (int i = 0; i < OPER; ++i) {
                const int c = g + NG * i;
                if (c < dv) {
                    const double* vr = sV + c * kKB64;
                    double acc = o[i] * alpha;
#pragma unroll
                    for (int k = 0; k < kKB64; ++k) acc = fma(pr[k], vr[k], acc);
                    o[i] = acc;
                }
            }
        }
    }

    const int n = q0 + qi;
    if (n >= N) return;
    if (STATS) {
        if (g == 0) p.nlse[(int64_t)b * N + n] = -(m_run + log(l_run)) / p.scale;
        return;
    }
    const double inv = 1.0 / l_run;
    double* Ob = p.O + (int64_t)b * N * dv;
#pragma unroll
    for (int i = 0; i < OPER; ++i) {
        const int c = g + NG * i;
        if (c < dv) Ob[(int64_t)c * N + n] = o[i] * inv;
    }
    if (g == 0) {
        p.m[(int64_t)b * N + n] = (float)m_run;
        p.l[(int64_t)b * N + n] = (float)l_run;
    }
}

// −rowsum(dO ∘ O) in double, one thread per (b, n), coalesced along n.
__global__ __launch_bounds__(256) void bwd_rowdot_f64(const double* __restrict__ O, const double* __restrict__ dO,
                                                      double* __restrict__ nD, int N, int dv, int64_t total) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const int64_t b = idx / N, n = idx - b * N;
    const double* o = O + b * (int64_t)N * dv + n;
    const double* g = dO + b * (int64_t)N * dv + n;
    double acc = 0.0;
    for (int c = 0; c < dv; ++c) acc = fma(g[(int64_t)c * N], o[(int64_t)c * N], acc);
    nD[idx] = -acc;
}

static bool f64_fits(int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch, const char** why) {
    if (d > kMaxHeadDim || dv > kMaxHeadDim) {
        *why = "head dimension exceeds the compiled maximum (128)";
        return false;
    }
    if (N > INT32_MAX / 2 || Nk > INT32_MAX / 2 || (N + kQB64 - 1) / kQB64 * batch > INT32_MAX) {
        *why = "extent exceeds the 32-bit grid";
        return false;
    }
    return true;
}

template <bool STATS, int QB>
static hipError_t launch_f64_qb(F64Params p, int64_t batch, hipStream_t s) {
    p.nqb = (p.N + QB - 1) / QB;
    const size_t lds = f64_lds_bytes(p.d, p.dv, STATS, QB);
    (void)hipFuncSetAttribute((const void*)dense_fwd_f64<STATS, QB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    hipLaunchKernelGGL((dense_fwd_f64<STATS, QB>), dim3((unsigned)(p.nqb * batch)), dim3(kTh64), lds, s, p);
    return hipGetLastError();
}
// 64 queries per workgroup when that fills the chip, else 16 (4x the workgroups:
// the reference's own Float64 cases are single slabs of 256-16384 tokens)
template <bool STATS>
static hipError_t launch_f64_kernel(const F64Params& p, int64_t batch, hipStream_t s) {
    if ((int64_t)((p.N + kQB64 - 1) / kQB64) * batch >= 256) return launch_f64_qb<STATS, kQB64>(p, batch, s);
    return launch_f64_qb<STATS, 16>(p, batch, s);
}

int launch_dense_fwd_f64(const DenseArgs& a, hipStream_t s, const char** why) {
    if (!f64_fits(a.N, a.Nk, a.d, a.dv, a.batch, why)) return FA_ERR_UNSUPPORTED;
    F64Params p;
    p.Q = (const double*)a.Q; p.K = (const double*)a.K; p.V = (const double*)a.V; p.O = (double*)a.O;
    p.l = a.l; p.m = a.m; p.nlse = nullptr;
    p.N = (int)a.N; p.Nk = (int)a.Nk; p.d = (int)a.d; p.dv = (int)a.dv;
    p.nqb = (int)((a.N + kQB64 - 1) / kQB64);
    p.scale = a.scale64 > 0.0 ? a.scale64 : (double)a.scale;
    const hipError_t e = launch_f64_kernel<false>(p, a.batch, s);
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    return FA_OK;
}

int launch_f64_bwd_stats(const DenseBwdArgs& a, double* nD, double* nlse, hipStream_t s, const char** why) {
    if (!f64_fits(a.N, a.Nk, a.d, a.dv, a.batch, why)) return FA_ERR_UNSUPPORTED;
    F64Params p;
    p.Q = (const double*)a.Q; p.K = (const double*)a.K; p.V = nullptr; p.O = nullptr;
    p.l = nullptr; p.m = nullptr; p.nlse = nlse;
    p.N = (int)a.N; p.Nk = (int)a.Nk; p.d = (int)a.d; p.dv = (int)a.dv;
    p.nqb = (int)((a.N + kQB64 - 1) / kQB64);
    p.scale = a.scale64 > 0.0 ? a.scale64 : (double)a.scale;
    hipError_t e = launch_f64_kernel<true>(p, a.batch, s);
    if (e == hipSuccess) {
        const int64_t total = a.N * a.batch;
        hipLaunchKernelGGL(bwd_rowdot_f64, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                           (const double*)a.O, (const double*)a.dO, nD, (int)a.N, (int)a.dv, total);
        e = hipGetLastError();
    }
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    return FA_OK;
}

}  // namespace fa
