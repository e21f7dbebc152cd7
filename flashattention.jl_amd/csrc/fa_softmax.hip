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
//    second pass that writes; rows of ≤ 32 elements stay in registers;
//  * sm_cols_reg_v / sm_rows_v: the same with 16-byte accesses whenever M is a
//    multiple of 8 (bf16/fp16) or 4 (fp32) and S, P are 16-B aligned: a thread
//    owns that many consecutive elements of a column, resp. consecutive rows
//    (rows: the 4 waves of a workgroup split the columns and merge (max, Σexp)
//    through LDS, so there are ≥ 8 workgroups per 4096 rows).
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

// ---- 16-byte vectorised forms (M % VEC == 0, 16-B aligned S and P) ----
template <class T> struct SmVec { static constexpr int n = 16 / (int)sizeof(T); };

template <class T>
__device__ __forceinline__ void unpack16(const u32x4 raw, float* f) {
    if constexpr (sizeof(T) == 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            // copy the lane out first: __builtin_bit_cast of an ext-vector element
            // expression reads element 0 for every k (observed with hipcc, ROCm 7.2)
            const unsigned w = raw[k];
            f[k] = __builtin_bit_cast(float, w);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned w = raw[k];
            f[2 * k] = (float)__builtin_bit_cast(T, (unsigned short)(w & 0xFFFFu));
            f[2 * k + 1] = (float)__builtin_bit_cast(T, (unsigned short)(w >> 16));
        }
    }
}

template <class T>
__device__ __forceinline__ u32x4 pack16(const float* f) {
    u32x4 raw;
    if constexpr (sizeof(T) == 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) raw[k] = __builtin_bit_cast(unsigned, f[k]);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned lo = __builtin_bit_cast(unsigned short, (T)f[2 * k]);
            const unsigned hi = __builtin_bit_cast(unsigned short, (T)f[2 * k + 1]);
            raw[k] = lo | (hi << 16);
        }
    }
    return raw;
}

// dims = 1, column of M <= 8192 elements (M % VEC == 0) in registers as 16-B vectors
template <class T>
__global__ __launch_bounds__(kSmThreads) void sm_cols_reg_v(const T* S, T* P, int M) {
    constexpr int VEC = SmVec<T>::n, NV = kSmEPT / VEC;   // vectors per thread
    const int nvec = M / VEC;
    const u32x4* Sv = (const u32x4*)(S + (int64_t)blockIdx.x * M);
    u32x4* Pv = (u32x4*)(P + (int64_t)blockIdx.x * M);
    float x[NV][VEC];
    float m = kNegInf;
#pragma unroll
    for (int e = 0; e < NV; ++e) {
        const int v = e * kSmThreads + threadIdx.x;
        if (v < nvec) {
            unpack16<T>(Sv[v], x[e]);
        } else {
#pragma unroll
            for (int k = 0; k < VEC; ++k) x[e][k] = kNegInf;
        }
#pragma unroll
        for (int k = 0; k < VEC; ++k) m = fmaxf(m, x[e][k]);
    }
    float l = 0.f;
    if (m != kNegInf) {
#pragma unroll
        for (int e = 0; e < NV; ++e)
#pragma unroll
            for (int k = 0; k < VEC; ++k) l += __expf(x[e][k] - m);
    }
    block_ml(m, l);
    const float inv = 1.0f / l;
#pragma unroll
    for (int e = 0; e < NV; ++e) {
        const int v = e * kSmThreads + threadIdx.x;
        if (v < nvec) {
            float y[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) y[k] = __expf(x[e][k] - m) * inv;
            Pv[v] = pack16<T>(y);
        }
    }
}

// dims = 2 with 16-B accesses (M % VEC == 0): a workgroup owns 64·VEC consecutive
// rows (each lane VEC of them); its 4 waves split the N columns (j ≡ wave mod 4),
// merge their (max, Σexp) partials through LDS, then each writes its columns.
template <class T>
__global__ __launch_bounds__(kSmThreads) void sm_rows_v(const T* S, T* P, int64_t M, int N) {
    // Both passes stream the row block U columns at a time (U independent 16-B
    // loads in flight per lane).  Pass 1 merges each U-column chunk into the
    // running (m, l) with ONE rescale: chunk max (IEEE maximum: NaN propagates),
    // then l = l·e^(m−m') + Σ e^(f−m'); a chunk whose max is −inf changes nothing
    // (as ml_merge's guard), so leading −inf columns cannot poison l.
    constexpr int VEC = SmVec<T>::n, NWV = kSmThreads / 64, U = 8;
    __shared__ float pm[NWV][64 * VEC], pl[NWV][64 * VEC];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t i0 = ((int64_t)blockIdx.x * 64 + lane) * VEC;
    const bool act = i0 < M;
    const int64_t base = (int64_t)blockIdx.y * M * N + i0;
    float m[VEC], l[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) { m[k] = kNegInf; l[k] = 0.f; }
    if (act) {
        for (int j0 = wave; j0 < N; j0 += NWV * U) {
            u32x4 raw[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = j0 + NWV * u;
                raw[u] = j < N ? *(const u32x4*)(S + base + (int64_t)j * M) : u32x4{0u, 0u, 0u, 0u};
            }
            float f[U][VEC];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                unpack16<T>(raw[u], f[u]);
                if (j0 + NWV * u >= N)
#pragma unroll
                    for (int k = 0; k < VEC; ++k) f[u][k] = kNegInf;
            }
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                float cm = f[0][k];
#pragma unroll
                for (int u = 1; u < U; ++u) cm = vmax(cm, f[u][k]);
                const float mn = vmax(m[k], cm);
                float add = 0.0f;
#pragma unroll
                for (int u = 0; u < U; ++u) add += exp2_fast((f[u][k] - mn) * kLog2e);
                const bool skip = mn == kNegInf;
                l[k] = skip ? l[k] : fmaf(l[k], exp2_fast((m[k] - mn) * kLog2e), add);
                m[k] = skip ? m[k] : mn;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) { pm[wave][lane * VEC + k] = m[k]; pl[wave][lane * VEC + k] = l[k]; }
    __syncthreads();
    float mrow[VEC], inv[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        float mm = pm[0][lane * VEC + k], ll = pl[0][lane * VEC + k];
#pragma unroll
        for (int w = 1; w < NWV; ++w) ml_merge(mm, ll, pm[w][lane * VEC + k], pl[w][lane * VEC + k]);
        mrow[k] = mm;
        inv[k] = 1.0f / ll;
    }
    if (!act) return;
    for (int j0 = wave; j0 < N; j0 += NWV * U) {
        u32x4 raw[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = j0 + NWV * u;
            if (j < N) raw[u] = *(const u32x4*)(S + base + (int64_t)j * M);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = j0 + NWV * u;
            if (j < N) {
                float f[VEC];
                unpack16<T>(raw[u], f);
#pragma unroll
                for (int k = 0; k < VEC; ++k) f[k] = exp2_fast((f[k] - mrow[k]) * kLog2e) * inv[k];
                *(u32x4*)(P + base + (int64_t)j * M) = pack16<T>(f);
            }
        }
    }
}

size_t softmax_workspace(int64_t M, int64_t N, int64_t batch, int dims) {
    if (dims != 1 || M <= kSmChunk) return 0;
    const int64_t nchunk = (M + kSmChunk - 1) / kSmChunk;
    return (size_t)(nchunk * N * batch) * sizeof(float2) + 256;
}

// Float64 (the reference's test element type), computed in double.
// dims = 1: one wave per column, lanes stride the M contiguous elements (three sweeps).
__global__ __launch_bounds__(256) void sm_cols_f64(const double* __restrict__ S, double* __restrict__ P, int64_t M,
                                                   int64_t cols) {
    const int64_t col = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (col >= cols) return;
    const int lane = threadIdx.x & 63;
    const double* x = S + col * M;
    double* y = P + col * M;
    double m = -__builtin_huge_val(), l = 0.0;
    for (int64_t i = lane; i < M; i += 64) m = __builtin_elementwise_maximum(m, x[i]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = __builtin_elementwise_maximum(m, __shfl_xor(m, o));
    for (int64_t i = lane; i < M; i += 64) l += exp(x[i] - m);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) l += __shfl_xor(l, o);
    const double inv = 1.0 / l;
    for (int64_t i = lane; i < M; i += 64) y[i] = exp(x[i] - m) * inv;
}
// dims = 2: one thread per row (stride M), lanes on consecutive rows (coalesced).
__global__ __launch_bounds__(256) void sm_rows_f64(const double* __restrict__ S, double* __restrict__ P, int64_t M,
                                                   int N) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= M) return;
    const int64_t base = (int64_t)blockIdx.y * M * N + i;
    double m = -__builtin_huge_val(), l = 0.0;
    for (int j = 0; j < N; ++j) m = __builtin_elementwise_maximum(m, S[base + (int64_t)j * M]);
    for (int j = 0; j < N; ++j) l += exp(S[base + (int64_t)j * M] - m);
    const double inv = 1.0 / l;
    for (int j = 0; j < N; ++j) P[base + (int64_t)j * M] = exp(S[base + (int64_t)j * M] - m) * inv;
}

template <class T>
static void launch_sm_typed(const SoftmaxArgs& a, hipStream_t s) {
    const T* S = (const T*)a.S;
    T* P = (T*)a.P;
    constexpr int VEC = SmVec<T>::n;
    const bool vec = a.M % VEC == 0 && ((uintptr_t)a.S & 15u) == 0 && ((uintptr_t)a.P & 15u) == 0;
    if (a.dims == 1) {
        const int64_t cols = a.N * a.batch;
        if (a.M <= kSmChunk && vec) {
            hipLaunchKernelGGL((sm_cols_reg_v<T>), dim3((unsigned)cols), dim3(kSmThreads), 0, s, S, P, (int)a.M);
        } else if (a.M <= kSmChunk) {
            hipLaunchKernelGGL((sm_cols_reg<T>), dim3((unsigned)cols), dim3(kSmThreads), 0, s, S, P, (int)a.M);
        } else {
            const int nchunk = (int)((a.M + kSmChunk - 1) / kSmChunk);
            float2* part = (float2*)a.workspace;
            const dim3 g((unsigned)(cols * nchunk));
            hipLaunchKernelGGL((sm_cols_part<T>), g, dim3(kSmThreads), 0, s, S, part, a.M, nchunk);
            hipLaunchKernelGGL((sm_cols_norm<T>), g, dim3(kSmThreads), 0, s, S, P, (const float2*)part, a.M, nchunk);
        }
    } else if (vec && a.N > 32) {
        const dim3 g((unsigned)((a.M / VEC + 63) / 64), (unsigned)a.batch);
        hipLaunchKernelGGL((sm_rows_v<T>), g, dim3(kSmThreads), 0, s, S, P, a.M, (int)a.N);
    } else {
        const dim3 g((unsigned)((a.M + kSmThreads - 1) / kSmThreads), (unsigned)a.batch);
        if (a.N <= 32)
            hipLaunchKernelGGL((sm_rows<T, true>), g, dim3(kSmThreads), 0, s, S, P, a.M, (int)a.N);
        else
            hipLaunchKernelGGL((sm_rows<T, false>), g, dim3(kSmThreads), 0, s, S, P, a.M, (int)a.N);
    }
}

int launch_softmax(const SoftmaxArgs& a, hipStream_t s, const char** why) {
    // grid limits: x <= 2^31 - 1 blocks; dims = 2 puts the batch on grid.y (<= 65535)
    if (a.N > INT32_MAX || (a.dims == 1 && a.N * a.batch * ((a.M + kSmChunk - 1) / kSmChunk) > INT32_MAX) ||
        (a.dims == 2 && (a.batch > 65535 || (a.M + kSmThreads - 1) / kSmThreads > INT32_MAX))) {
        *why = "extent exceeds the launch grid";
        return FA_ERR_UNSUPPORTED;
    }
    switch (a.dtype) {
        case FA_DTYPE_BF16: launch_sm_typed<bf16>(a, s); break;
        case FA_DTYPE_F16: launch_sm_typed<f16>(a, s); break;
        case FA_DTYPE_F32: launch_sm_typed<float>(a, s); break;
        case FA_DTYPE_F64:
            if (a.dims == 1) {
                const int64_t cols = a.N * a.batch;
                hipLaunchKernelGGL(sm_cols_f64, dim3((unsigned)((cols + 3) / 4)), dim3(256), 0, s, (const double*)a.S,
                                   (double*)a.P, a.M, cols);
            } else {
                hipLaunchKernelGGL(sm_rows_f64, dim3((unsigned)((a.M + 255) / 256), (unsigned)a.batch), dim3(256), 0,
                                   s, (const double*)a.S, (double*)a.P, a.M, (int)a.N);
            }
            break;
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
