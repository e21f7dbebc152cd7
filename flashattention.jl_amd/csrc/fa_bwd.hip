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
#include <type_traits>

#include "fa_common.h"
#include "fa_internal.h"
#include "../../include/fa_hip.h"

namespace fa {

struct BwdParams {
    const void *Q, *K, *V, *O, *dO;
    const float *l, *m;
    void *dQ, *dK, *dV;
    float* Dv;     // workspace: rowsum(dO ∘ O)   [batch][N]
    float* lse2;   // workspace: (m + ln l)·log2e [batch][N]
    int N, Nk, d, dv, batch;
    float scale, scale_log2;
};

template <class T> __device__ __forceinline__ float to_f(T x) { return (float)x; }

// --------------------------------------------------------------------------
// 1. pre-pass (HBM-bound): one thread per (b, n), coalesced along n.
// --------------------------------------------------------------------------
template <class T>
__global__ __launch_bounds__(256) void bwd_prepass(BwdParams p) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t total = (int64_t)p.N * p.batch;
    if (idx >= total) return;
    const int64_t b = idx / p.N, n = idx - b * p.N;
    const T* O = (const T*)p.O + b * (int64_t)p.N * p.dv + n;
    const T* dO = (const T*)p.dO + b * (int64_t)p.N * p.dv + n;
    float acc = 0.0f;
    for (int c = 0; c < p.dv; ++c) acc = fmaf(to_f(dO[(int64_t)c * p.N]), to_f(O[(int64_t)c * p.N]), acc);
    p.Dv[idx] = acc;
    p.lse2[idx] = (p.m[idx] + logf(p.l[idx])) * kLog2e;
}

// --------------------------------------------------------------------------
// 2./3. generic SIMT path.  Tiles of 32 queries x 32 keys in LDS (fp32).
// --------------------------------------------------------------------------
constexpr int kGT = 32;          // tile edge
constexpr int kGThreads = 256;

// dQ: one block per (b, 32-query tile).
template <class T>
__global__ __launch_bounds__(kGThreads) void bwd_generic_dq(BwdParams p) {
    extern __shared__ __attribute__((aligned(16))) float gsm[];
    const int d = p.d, dv = p.dv, N = p.N, Nk = p.Nk;
    float* sQ = gsm;                     // [32][d]
    float* sdO = sQ + kGT * d;           // [32][dv]
    float* sK = sdO + kGT * dv;          // [32][d]
    float* sV = sK + kGT * d;            // [32][dv]
    float* sdS = sV + kGT * dv;          // [32 q][33]
    const int nqt = (N + kGT - 1) / kGT;
    const int b = blockIdx.x / nqt, q0 = (blockIdx.x % nqt) * kGT;
    const int tid = threadIdx.x;
    const T* Qb = (const T*)p.Q + (int64_t)b * N * d;
    const T* Kb = (const T*)p.K + (int64_t)b * Nk * d;
    const T* Vb = (const T*)p.V + (int64_t)b * Nk * dv;
    const T* dOb = (const T*)p.dO + (int64_t)b * N * dv;
    for (int i = tid; i < kGT * d; i += kGThreads) {
        const int q = i % kGT, f = i / kGT;
        sQ[q * d + f] = (q0 + q < N) ? to_f(Qb[(int64_t)f * N + q0 + q]) : 0.0f;
    }
    for (int i = tid; i < kGT * dv; i += kGThreads) {
        const int q = i % kGT, f = i / kGT;
        sdO[q * dv + f] = (q0 + q < N) ? to_f(dOb[(int64_t)f * N + q0 + q]) : 0.0f;
    }
    // each thread owns dQ entries (q, f) = (i % 32, i / 32) for i = tid + 256·t
    constexpr int kMaxPer = 128 * kGT / kGThreads;   // d <= 128
    float acc[kMaxPer];
#pragma unroll
    for (int t = 0; t < kMaxPer; ++t) acc[t] = 0.0f;
    const float* Dv = p.Dv + (int64_t)b * N;
    const float* L2 = p.lse2 + (int64_t)b * N;
    for (int k0 = 0; k0 < Nk; k0 += kGT) {
        __syncthreads();
        for (int i = tid; i < kGT * d; i += kGThreads) {
            const int k = i % kGT, f = i / kGT;
            sK[k * d + f] = (k0 + k < Nk) ? to_f(Kb[(int64_t)f * Nk + k0 + k]) : 0.0f;
        }
        for (int i = tid; i < kGT * dv; i += kGThreads) {
            const int k = i % kGT, f = i / kGT;
            sV[k * dv + f] = (k0 + k < Nk) ? to_f(Vb[(int64_t)f * Nk + k0 + k]) : 0.0f;
        }
        __syncthreads();
        for (int e = tid; e < kGT * kGT; e += kGThreads) {
            const int q = e / kGT, k = e % kGT;
            float ds = 0.0f;
            if (q0 + q < N && k0 + k < Nk) {
                float s = 0.0f, dp = 0.0f;
                for (int f = 0; f < d; ++f) s = fmaf(sQ[q * d + f], sK[k * d + f], s);
                for (int f = 0; f < dv; ++f) dp = fmaf(sdO[q * dv + f], sV[k * dv + f], dp);
                const float pr = exp2f(s * p.scale_log2 - L2[q0 + q]);
                ds = pr * (dp - Dv[q0 + q]);
            }
            sdS[q * (kGT + 1) + k] = ds;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < kMaxPer; ++t) {
            const int i = tid + kGThreads * t, q = i % kGT, f = i / kGT;
            if (f < d) {
                float a = acc[t];
                for (int k = 0; k < kGT; ++k) a = fmaf(sdS[q * (kGT + 1) + k], sK[k * d + f], a);
                acc[t] = a;
            }
        }
    }
    T* dQb = (T*)p.dQ + (int64_t)b * N * d;
#pragma unroll
    for (int t = 0; t < kMaxPer; ++t) {
        const int i = tid + kGThreads * t, q = i % kGT, f = i / kGT;
        if (f < d && q0 + q < N) dQb[(int64_t)f * N + q0 + q] = (T)(acc[t] * p.scale);
    }
}

// dK, dV: one block per (b, 32-key tile).
template <class T>
__global__ __launch_bounds__(kGThreads) void bwd_generic_dkdv(BwdParams p) {
    extern __shared__ __attribute__((aligned(16))) float gsm[];
    const int d = p.d, dv = p.dv, N = p.N, Nk = p.Nk;
    float* sK = gsm;                     // [32][d]
    float* sV = sK + kGT * d;            // [32][dv]
    float* sQ = sV + kGT * dv;           // [32][d]
    float* sdO = sQ + kGT * d;           // [32][dv]
    float* sP = sdO + kGT * dv;          // [32 q][33]
    float* sdS = sP + kGT * (kGT + 1);   // [32 q][33]
    const int nkt = (Nk + kGT - 1) / kGT;
    const int b = blockIdx.x / nkt, k0 = (blockIdx.x % nkt) * kGT;
    const int tid = threadIdx.x;
    const T* Qb = (const T*)p.Q + (int64_t)b * N * d;
    const T* Kb = (const T*)p.K + (int64_t)b * Nk * d;
    const T* Vb = (const T*)p.V + (int64_t)b * Nk * dv;
    const T* dOb = (const T*)p.dO + (int64_t)b * N * dv;
    for (int i = tid; i < kGT * d; i += kGThreads) {
        const int k = i % kGT, f = i / kGT;
        sK[k * d + f] = (k0 + k < Nk) ? to_f(Kb[(int64_t)f * Nk + k0 + k]) : 0.0f;
    }
    for (int i = tid; i < kGT * dv; i += kGThreads) {
        const int k = i % kGT, f = i / kGT;
        sV[k * dv + f] = (k0 + k < Nk) ? to_f(Vb[(int64_t)f * Nk + k0 + k]) : 0.0f;
    }
    constexpr int kMaxPer = 128 * kGT / kGThreads;
    float accK[kMaxPer], accV[kMaxPer];
#pragma unroll
    for (int t = 0; t < kMaxPer; ++t) { accK[t] = 0.0f; accV[t] = 0.0f; }
    const float* Dv = p.Dv + (int64_t)b * N;
    const float* L2 = p.lse2 + (int64_t)b * N;
    for (int q0 = 0; q0 < N; q0 += kGT) {
        __syncthreads();
        for (int i = tid; i < kGT * d; i += kGThreads) {
            const int q = i % kGT, f = i / kGT;
            sQ[q * d + f] = (q0 + q < N) ? to_f(Qb[(int64_t)f * N + q0 + q]) : 0.0f;
        }
        for (int i = tid; i < kGT * dv; i += kGThreads) {
            const int q = i % kGT, f = i / kGT;
            sdO[q * dv + f] = (q0 + q < N) ? to_f(dOb[(int64_t)f * N + q0 + q]) : 0.0f;
        }
        __syncthreads();
        for (int e = tid; e < kGT * kGT; e += kGThreads) {
            const int q = e / kGT, k = e % kGT;
            float pr = 0.0f, ds = 0.0f;
            if (q0 + q < N && k0 + k < Nk) {
                float s = 0.0f, dp = 0.0f;
                for (int f = 0; f < d; ++f) s = fmaf(sQ[q * d + f], sK[k * d + f], s);
                for (int f = 0; f < dv; ++f) dp = fmaf(sdO[q * dv + f], sV[k * dv + f], dp);
                pr = exp2f(s * p.scale_log2 - L2[q0 + q]);
                ds = pr * (dp - Dv[q0 + q]);
            }
            sP[q * (kGT + 1) + k] = pr;
            sdS[q * (kGT + 1) + k] = ds;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < kMaxPer; ++t) {
            const int i = tid + kGThreads * t, k = i % kGT, f = i / kGT;
            if (f < d) {
                float a = accK[t];
                for (int q = 0; q < kGT; ++q) a = fmaf(sdS[q * (kGT + 1) + k], sQ[q * d + f], a);
                accK[t] = a;
            }
            if (f < dv) {
                float a = accV[t];
                for (int q = 0; q < kGT; ++q) a = fmaf(sP[q * (kGT + 1) + k], sdO[q * dv + f], a);
                accV[t] = a;
            }
        }
    }
    T* dKb = (T*)p.dK + (int64_t)b * Nk * d;
    T* dVb = (T*)p.dV + (int64_t)b * Nk * dv;
#pragma unroll
    for (int t = 0; t < kMaxPer; ++t) {
        const int i = tid + kGThreads * t, k = i % kGT, f = i / kGT;
        if (k0 + k < Nk) {
            if (f < d) dKb[(int64_t)f * Nk + k0 + k] = (T)(accK[t] * p.scale);
            if (f < dv) dVb[(int64_t)f * Nk + k0 + k] = (T)accV[t];
        }
    }
}

// --------------------------------------------------------------------------
// launcher
// --------------------------------------------------------------------------
size_t dense_bwd_workspace(int, int64_t N, int64_t, int64_t, int64_t, int64_t batch) {
    return (size_t)(2 * N * batch * sizeof(float) + 256);
}

template <class T>
static hipError_t launch_generic(const BwdParams& p, hipStream_t s) {
    const int64_t nq = ((int64_t)p.N + kGT - 1) / kGT * p.batch;
    const int64_t nk = ((int64_t)p.Nk + kGT - 1) / kGT * p.batch;
    const size_t sm_dq = sizeof(float) * (kGT * (2 * p.d + 2 * p.dv) + kGT * (kGT + 1));
    const size_t sm_kv = sizeof(float) * (kGT * (2 * p.d + 2 * p.dv) + 2 * kGT * (kGT + 1));
    // > 64 KiB of dynamic LDS at d = dv = 128 (gfx950 has 160 KiB per CU)
    (void)hipFuncSetAttribute((const void*)bwd_generic_dq<T>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm_dq);
    (void)hipFuncSetAttribute((const void*)bwd_generic_dkdv<T>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm_kv);
    hipLaunchKernelGGL(bwd_generic_dq<T>, dim3((unsigned)nq), dim3(kGThreads), sm_dq, s, p);
    hipLaunchKernelGGL(bwd_generic_dkdv<T>, dim3((unsigned)nk), dim3(kGThreads), sm_kv, s, p);
    return hipGetLastError();
}

template <class T>
static hipError_t launch_typed(const BwdParams& p, hipStream_t s) {
    const int64_t total = (int64_t)p.N * p.batch;
    hipLaunchKernelGGL(bwd_prepass<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_generic<T>(p, s);
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
    const uintptr_t ws = ((uintptr_t)a.workspace + 255) & ~(uintptr_t)255;
    p.Dv = (float*)ws;
    p.lse2 = p.Dv + a.N * a.batch;
    p.N = (int)a.N; p.Nk = (int)a.Nk; p.d = (int)a.d; p.dv = (int)a.dv; p.batch = (int)a.batch;
    p.scale = a.scale;
    p.scale_log2 = a.scale * kLog2e;
    hipError_t e;
    switch (a.dtype) {
        case FA_DTYPE_BF16: e = launch_typed<bf16>(p, s); break;
        case FA_DTYPE_F16: e = launch_typed<f16>(p, s); break;
        case FA_DTYPE_F32: e = launch_typed<float>(p, s); break;
        default: *why = "unknown dtype"; return FA_ERR_INVALID_ARG;
    }
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    return FA_OK;
}

}  // namespace fa
