// fa_softmax.hip — standalone fused softmax for gfx950.
//
// Replaces fused_softmax!(P, S; dims) (reference src/fused_softmax.jl:1-41 —
// col_softmax! for dims = 1, row_softmax! for dims = 2; device versions
// src/cuda/fused_softmax.jl:11-314).  S, P: Julia column-major (M, N, batch);
// dims = 1 normalises each column S[:, j, b] (M contiguous elements), dims = 2
// each row S[i, :, b] (N elements at stride M).  P = exp(s − max s) / Σ exp(…),
// computed in fp32, stored in T.  P may alias S (fused_softmax!(S), :2).
//
// HBM-bound (≈ 5 FLOP per 2·esz bytes).  Kernels:
//  * sm_cols_reg: one 256-thread workgroup per column, the column held in
//    registers (≤ 8192 elements): one read, one write;
//  * sm_cols_part + sm_cols_norm: longer columns in 8192-element chunks —
//    per-chunk (max, Σexp) partials, then each chunk combines its column's
//    partials and writes (two reads, one write);
//  * sm_rows: dims = 2, one thread per row i (lanes over consecutive i, so every
//    access is coalesced across the wave), online (max, Σexp) over j, then a
//    second pass that writes; rows of ≤ 32 elements stay in registers.
#include <type_traits>

#include "fa_common.h"
#include "fa_internal.h"
#include "../../include/fa_hip.h"

namespace fa {

constexpr int kSmThreads = 256;
constexpr int kSmEPT = 32;                          // elements per thread in registers
constexpr int kSmChunk = kSmThreads * kSmEPT;       // 8192

template <class T> __device__ __forceinline__ float ld(const T* p, int64_t i) { return (float)p[i]; }

// (m, l) pair merge: l scaled to the common max; −inf maxima merge to −inf
__device__ __forceinline__ void ml_merge(float& m, float& l, float m2, float l2) {
    const float mn = fmaxf(m, m2);
    if (mn == kNegInf) { l = l + l2; m = mn; return; }
    l = l * __expf(m - mn) + l2 * __expf(m2 - mn);
    m = mn;
}

// workgroup-wide (m, l) reduction; every thread gets the result
__device__ __forceinline__ void block_ml(float& m, float& l) {
    __shared__ float sm[kSmThreads / 64], sl[kSmThreads / 64];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float m2 = __shfl_xor(m, o), l2 = __shfl_xor(l, o);
        ml_merge(m, l, m2, l2);
    }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) { sm[w] = m; sl[w] = l; }
    __syncthreads();
    m = sm[0]; l = sl[0];
#pragma unroll
    for (int i = 1; i < kSmThreads / 64; ++i) ml_merge(m, l, sm[i], sl[i]);
}

// dims = 1, column of M <= 8192 elements in registers; blockIdx.x = column (j + N·b)
template <class T>
__global__ __launch_bounds__(kSmThreads) void sm_cols_reg(const T* S, T* P, int M) {
    const int64_t base = (int64_t)blockIdx.x * M;
    float x[kSmEPT];
    float m = kNegInf;
#pragma unroll
    for (int e = 0; e < kSmEPT; ++e) {
        const int i = e * kSmThreads + threadIdx.x;
        x[e] = i < M ? ld(S, base + i) : kNegInf;
        m = fmaxf(m, x[e]);
    }
    float l = 0.f;
    if (m != kNegInf) {
#pragma unroll
        for (int e = 0; e < kSmEPT; ++e) l += __expf(x[e] - m);
    }
    block_ml(m, l);
    const float inv = 1.0f / l;
#pragma unroll
    for (int e = 0; e < kSmEPT; ++e) {
        const int i = e * kSmThreads + threadIdx.x;
        if (i < M) P[base + i] = (T)(__expf(x[e] - m) * inv);
    }
}

// dims = 1, long columns: partial (m, l) per 8192-element chunk
template <class T>
__global__ __launch_bounds__(kSmThreads) void sm_cols_part(const T* S, float2* part, int64_t M, int nchunk) {
    const int64_t col = blockIdx.x / nchunk;
    const int ch = blockIdx.x - (int)(col * nchunk);
    const int64_t base = col * M + (int64_t)ch * kSmChunk;
    const int64_t len = min((int64_t)kSmChunk, M - (int64_t)ch * kSmChunk);
    float m = kNegInf, l = 0.f;
    for (int64_t i = threadIdx.x; i < len; i += kSmThreads) {
        const float v = ld(S, base + i);
        ml_merge(m, l, v, 1.0f);
    }
    block_ml(m, l);
    if (threadIdx.x == 0) part[blockIdx.x] = make_float2(m, l);
}

template <class T>
__global__ __launch_bounds__(kSmThreads) void sm_cols_norm(const T* S, T* P, const float2* part, int64_t M, int nchunk) {
    const int64_t col = blockIdx.x / nchunk;
    const int ch = blockIdx.x - (int)(col * nchunk);
    float m = kNegInf, l = 0.f;
    for (int i = 0; i < nchunk; ++i) {
        const float2 q = part[col * nchunk + i];
        ml_merge(m, l, q.x, q.y);
    }
    const float inv = 1.0f / l;
    const int64_t base = col * M + (int64_t)ch * kSmChunk;
    const int64_t len = min((int64_t)kSmChunk, M - (int64_t)ch * kSmChunk);
    for (int64_t i = threadIdx.x; i < len; i += kSmThreads) P[base + i] = (T)(__expf(ld(S, base + i) - m) * inv);
}

// dims = 2: thread per row i of one batch slab; grid = (ceil(M / 256), batch)
template <class T, bool REG>
__global__ __launch_bounds__(kSmThreads) void sm_rows(const T* S, T* P, int64_t M, int N) {
    const int64_t i = (int64_t)blockIdx.x * kSmThreads + threadIdx.x;
    if (i >= M) return;
    const int64_t base = (int64_t)blockIdx.y * M * N + i;
    if constexpr (REG) {
        float x[32];
        float m = kNegInf;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            x[j] = j < N ? ld(S, base + (int64_t)j * M) : kNegInf;
            m = fmaxf(m, x[j]);
        }
        float l = 0.f;
#pragma unroll
        for (int j = 0; j < 32; ++j) l += j < N ? __expf(x[j] - m) : 0.f;
        const float inv = 1.0f / l;
#pragma unroll
        for (int j = 0; j < 32; ++j)
            if (j < N) P[base + (int64_t)j * M] = (T)(__expf(x[j] - m) * inv);
    } else {
        float m = kNegInf, l = 0.f;
        for (int j = 0; j < N; ++j) ml_merge(m, l, ld(S, base + (int64_t)j * M), 1.0f);
        const float inv = 1.0f / l;
        for (int j = 0; j < N; ++j) P[base + (int64_t)j * M] = (T)(__expf(ld(S, base + (int64_t)j * M) - m) * inv);
    }
}

size_t softmax_workspace(int64_t M, int64_t N, int64_t batch, int dims) {
    if (dims != 1 || M <= kSmChunk) return 0;
    const int64_t nchunk = (M + kSmChunk - 1) / kSmChunk;
    return (size_t)(nchunk * N * batch) * sizeof(float2) + 256;
}

template <class T>
static void launch_sm_typed(const SoftmaxArgs& a, hipStream_t s) {
    const T* S = (const T*)a.S;
    T* P = (T*)a.P;
    if (a.dims == 1) {
        const int64_t cols = a.N * a.batch;
        if (a.M <= kSmChunk) {
            hipLaunchKernelGGL((sm_cols_reg<T>), dim3((unsigned)cols), dim3(kSmThreads), 0, s, S, P, (int)a.M);
        } else {
            const int nchunk = (int)((a.M + kSmChunk - 1) / kSmChunk);
            float2* part = (float2*)a.workspace;
            const dim3 g((unsigned)(cols * nchunk));
            hipLaunchKernelGGL((sm_cols_part<T>), g, dim3(kSmThreads), 0, s, S, part, a.M, nchunk);
            hipLaunchKernelGGL((sm_cols_norm<T>), g, dim3(kSmThreads), 0, s, S, P, (const float2*)part, a.M, nchunk);
        }
    } else {
        const dim3 g((unsigned)((a.M + kSmThreads - 1) / kSmThreads), (unsigned)a.batch);
        if (a.N <= 32)
            hipLaunchKernelGGL((sm_rows<T, true>), g, dim3(kSmThreads), 0, s, S, P, a.M, (int)a.N);
        else
            hipLaunchKernelGGL((sm_rows<T, false>), g, dim3(kSmThreads), 0, s, S, P, a.M, (int)a.N);
    }
}

int launch_softmax(const SoftmaxArgs& a, hipStream_t s, const char** why) {
    if (a.N > INT32_MAX || a.batch > 65535 || (a.dims == 1 && a.N * a.batch * ((a.M + kSmChunk - 1) / kSmChunk) > UINT32_MAX) ||
        (a.dims == 2 && (a.M + kSmThreads - 1) / kSmThreads > UINT32_MAX)) {
        *why = "extent exceeds the launch grid";
        return FA_ERR_UNSUPPORTED;
    }
    switch (a.dtype) {
        case FA_DTYPE_BF16: launch_sm_typed<bf16>(a, s); break;
        case FA_DTYPE_F16: launch_sm_typed<f16>(a, s); break;
        case FA_DTYPE_F32: launch_sm_typed<float>(a, s); break;
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
