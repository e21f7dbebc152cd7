// fa_windowed.hip — windowed / block-local attention on gfx950.
//
// Replaces windowed_fa(q, k, v, ws; stride, pad) (reference
// src/windowed.jl:3-23; block_fa = stride ws, :1) and adds its backward
// (README.md:36-37 claims it, the reference has no code).
//
// Window geometry is NNlib.unfold / fold's (src/utils.jl:36-54): per spatial
// dim O_i = (S_i + 2 pad − ws) / stride + 1 windows, window token t =
// (t_1, t_2, t_3) first-dim-fastest, pixel x_i = o_i·stride − pad + t_i, zero
// padding outside the image (padded tokens are ordinary, UNMASKED keys with
// k = v = 0, exactly as in the reference).  y = fold(window outputs) ./
// coverage count, so uncovered pixels are 0/0 = NaN (Appendix A.7).
//
// Composed path (every dtype, any window size):
//   gather  : q, k, v → (T, d, L·B) window batches in the workspace;
//   dense   : fa_dense_fwd / fa_dense_bwd on the window batch (l, m land
//             directly in the caller's (T, 1, L, B) arrays: same layout);
//   fold    : deterministic per-pixel sum over covering windows (÷ count).
// The backward is the exact chain rule: dyw = window(dy ./ count), dense
// backward per window, fold (sum) of dqw / dkw / dvw.
#include "fa_common.h"
#include "fa_internal.h"
#include "../../include/fa_hip.h"

namespace fa {

struct WinDev {
    int nsp, ws, stride, pad, T, L, P;
    int S[3], O[3];
};

static WinDev to_dev(const WindowGeom& g) {
    WinDev w;
    w.nsp = g.nsp; w.ws = (int)g.ws; w.stride = (int)g.stride; w.pad = (int)g.pad;
    w.T = (int)g.T; w.L = (int)g.L; w.P = (int)g.P;
    for (int i = 0; i < 3; ++i) { w.S[i] = (int)g.S[i]; w.O[i] = (int)g.O[i]; }
    return w;
}

// pixel index of window w, token t (−1 = zero padding)
__device__ __forceinline__ int win_pixel(const WinDev& g, int w, int t) {
    int pix = 0, mul = 1;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i < g.nsp) {
            const int o = w % g.O[i];
            w /= g.O[i];
            const int ti = t % g.ws;
            t /= g.ws;
            const int x = o * g.stride - g.pad + ti;
            if (x < 0 || x >= g.S[i]) return -1;
            pix += x * mul;
            mul *= g.S[i];
        }
    }
    return pix;
}

// number of windows covering pixel pix (for the divisor)
__device__ __forceinline__ int win_count(const WinDev& g, int pix) {
    int cnt = 1;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i < g.nsp) {
            const int x = pix % g.S[i];
            pix /= g.S[i];
            const int num = x + g.pad - g.ws + 1;
            const int lo = num <= 0 ? 0 : (num + g.stride - 1) / g.stride;
            const int hi = min(g.O[i] - 1, (x + g.pad) / g.stride);
            cnt *= max(0, hi - lo + 1);
        }
    }
    return cnt;
}

// dst (T, C, L·B) ← window(src (S..., C, B)); DIVIDE scales by 1/coverage
template <class T, bool DIVIDE>
__global__ __launch_bounds__(256) void win_gather(const T* __restrict__ src, T* __restrict__ dst, int C,
                                                  int64_t total, WinDev g) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    const int t = (int)(e % g.T);
    int64_t rest = e / g.T;
    const int c = (int)(rest % C);
    rest /= C;
    const int w = (int)(rest % g.L);
    const int64_t b = rest / g.L;
    const int pix = win_pixel(g, w, t);
    float v = 0.0f;
    if (pix >= 0) {
        v = (float)src[(b * C + c) * (int64_t)g.P + pix];
        if constexpr (DIVIDE) v /= (float)win_count(g, pix);
    }
    dst[e] = (T)v;
}

// dst (S..., C, B) ← fold(src (T, C, L·B)) [÷ coverage count, NaN if 0]
template <class T, bool DIVIDE>
__global__ __launch_bounds__(256) void win_fold(const T* __restrict__ src, T* __restrict__ dst, int C,
                                                int64_t total, WinDev g) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    const int pix = (int)(e % g.P);
    const int64_t bc = e / g.P;             // b·C + c
    const int c = (int)(bc % C);
    const int64_t b = bc / C;
    int x[3] = {0, 0, 0}, lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
    int rem = pix;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i < g.nsp) {
            x[i] = rem % g.S[i];
            rem /= g.S[i];
            const int num = x[i] + g.pad - g.ws + 1;
            lo[i] = num <= 0 ? 0 : (num + g.stride - 1) / g.stride;
            hi[i] = min(g.O[i] - 1, (x[i] + g.pad) / g.stride);
        }
    }
    float acc = 0.0f;
    int cnt = 0;
    for (int o3 = lo[2]; o3 <= hi[2]; ++o3)
        for (int o2 = lo[1]; o2 <= hi[1]; ++o2)
            for (int o1 = lo[0]; o1 <= hi[0]; ++o1) {
                const int t1 = x[0] + g.pad - o1 * g.stride;
                const int t2 = g.nsp > 1 ? x[1] + g.pad - o2 * g.stride : 0;
                const int t3 = g.nsp > 2 ? x[2] + g.pad - o3 * g.stride : 0;
                const int w = o1 + g.O[0] * (o2 + g.O[1] * o3);
                const int t = t1 + g.ws * (t2 + g.ws * t3);
                acc += (float)src[t + (int64_t)g.T * (c + (int64_t)C * (w + (int64_t)g.L * b))];
                ++cnt;
            }
    if constexpr (DIVIDE) acc = acc / (float)cnt;   // 0/0 = NaN where uncovered (reference semantics)
    dst[e] = (T)acc;
}

static size_t esize(int dtype) { return dtype == FA_DTYPE_F32 ? 4 : 2; }
static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t windowed_fwd_workspace(int dtype, const WindowGeom& g, int64_t d, int64_t dv, int64_t batch) {
    const size_t tok = (size_t)(g.T * g.L * batch);
    return align256(tok * d * esize(dtype)) * 2 + align256(tok * dv * esize(dtype)) * 2 + 256;
}

size_t windowed_workspace(int dtype, const WindowGeom& g, int64_t d, int64_t dv, int64_t batch) {
    const size_t tok = (size_t)(g.T * g.L * batch);
    const size_t e = esize(dtype);
    return align256(tok * d * e) * 4 + align256(tok * dv * e) * 4 + align256(tok * 4) * 2 +
           align256(dense_bwd_workspace(dtype, g.T, g.T, d, dv, g.L * batch)) + 256;
}

template <class T>
static hipError_t gather(const void* src, void* dst, int C, int64_t batch, const WinDev& g, bool divide,
                         hipStream_t s) {
    const int64_t total = (int64_t)g.T * C * g.L * batch;
    const dim3 grid((unsigned)((total + 255) / 256));
    if (divide) hipLaunchKernelGGL((win_gather<T, true>), grid, dim3(256), 0, s, (const T*)src, (T*)dst, C, total, g);
    else hipLaunchKernelGGL((win_gather<T, false>), grid, dim3(256), 0, s, (const T*)src, (T*)dst, C, total, g);
    return hipGetLastError();
}
template <class T>
static hipError_t fold(const void* src, void* dst, int C, int64_t batch, const WinDev& g, bool divide,
                       hipStream_t s) {
    const int64_t total = (int64_t)g.P * C * batch;
    const dim3 grid((unsigned)((total + 255) / 256));
    if (divide) hipLaunchKernelGGL((win_fold<T, true>), grid, dim3(256), 0, s, (const T*)src, (T*)dst, C, total, g);
    else hipLaunchKernelGGL((win_fold<T, false>), grid, dim3(256), 0, s, (const T*)src, (T*)dst, C, total, g);
    return hipGetLastError();
}

static bool geom_fits(const WindowGeom& g, int64_t d, int64_t dv, int64_t batch) {
    return g.T * g.L * batch * (d > dv ? d : dv) < (int64_t)INT32_MAX * 2 && g.P * batch * (d > dv ? d : dv) < INT32_MAX * 2LL &&
           g.T * g.L < INT32_MAX && g.P < INT32_MAX;
}

template <class T>
static int windowed_fwd_typed(const WindowedArgs& a, hipStream_t s, const char** why) {
    const WinDev g = to_dev(a.g);
    const int64_t tok = a.g.T * a.g.L * a.batch;
    char* ws = (char*)(((uintptr_t)a.workspace + 255) & ~(uintptr_t)255);
    void* qw = ws;  ws += align256(tok * a.d * sizeof(T));
    void* kw = ws;  ws += align256(tok * a.d * sizeof(T));
    void* vw = ws;  ws += align256(tok * a.dv * sizeof(T));
    void* ow = ws;
    hipError_t e;
    if ((e = gather<T>(a.q, qw, (int)a.d, a.batch, g, false, s)) != hipSuccess ||
        (e = gather<T>(a.k, kw, (int)a.d, a.batch, g, false, s)) != hipSuccess ||
        (e = gather<T>(a.v, vw, (int)a.dv, a.batch, g, false, s)) != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    DenseArgs da{a.dtype, qw, kw, vw, ow, a.l, a.m, a.g.T, a.g.T, a.d, a.dv, a.g.L * a.batch, a.scale};
    const int rc = launch_dense_fwd(da, s, why);
    if (rc != FA_OK) return rc;
    if ((e = fold<T>(ow, a.y, (int)a.dv, a.batch, g, true, s)) != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    return FA_OK;
}

int launch_windowed_fwd(const WindowedArgs& a, hipStream_t s, const char** why) {
    if (a.d > kMaxHeadDim || a.dv > kMaxHeadDim) {
        *why = "head dimension exceeds the compiled maximum (128)";
        return FA_ERR_UNSUPPORTED;
    }
    if (!geom_fits(a.g, a.d, a.dv, a.batch)) {
        *why = "windowed problem too large for 32-bit window indexing";
        return FA_ERR_UNSUPPORTED;
    }
    switch (a.dtype) {
        case FA_DTYPE_BF16: return windowed_fwd_typed<bf16>(a, s, why);
        case FA_DTYPE_F16: return windowed_fwd_typed<f16>(a, s, why);
        case FA_DTYPE_F32: return windowed_fwd_typed<float>(a, s, why);
    }
    *why = "unknown dtype";
    return FA_ERR_INVALID_ARG;
}

template <class T>
static int windowed_bwd_typed(const WindowedBwdArgs& a, hipStream_t s, const char** why) {
    const WinDev g = to_dev(a.g);
    const int64_t tok = a.g.T * a.g.L * a.batch;
    const int64_t nb = a.g.L * a.batch;
    char* ws = (char*)(((uintptr_t)a.workspace + 255) & ~(uintptr_t)255);
    auto take = [&](size_t bytes) { void* p = ws; ws += align256(bytes); return p; };
    void* qw = take(tok * a.d * sizeof(T));
    void* kw = take(tok * a.d * sizeof(T));
    void* vw = take(tok * a.dv * sizeof(T));
    void* ow = take(tok * a.dv * sizeof(T));
    void* dyw = take(tok * a.dv * sizeof(T));
    void* dqw = take(tok * a.d * sizeof(T));
    void* dkw = take(tok * a.d * sizeof(T));
    void* dvw = take(tok * a.dv * sizeof(T));
    float* lw = (float*)take(tok * 4);
    float* mw = (float*)take(tok * 4);
    const size_t dws = dense_bwd_workspace(a.dtype, a.g.T, a.g.T, a.d, a.dv, nb);
    void* dwork = take(dws);
    hipError_t e;
    if ((e = gather<T>(a.q, qw, (int)a.d, a.batch, g, false, s)) != hipSuccess ||
        (e = gather<T>(a.k, kw, (int)a.d, a.batch, g, false, s)) != hipSuccess ||
        (e = gather<T>(a.v, vw, (int)a.dv, a.batch, g, false, s)) != hipSuccess ||
        (e = gather<T>(a.dy, dyw, (int)a.dv, a.batch, g, true, s)) != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    // per-window outputs O_w (the backward's D = rowsum(dO_w ∘ O_w) needs them)
    DenseArgs da{a.dtype, qw, kw, vw, ow, lw, mw, a.g.T, a.g.T, a.d, a.dv, nb, a.scale};
    int rc = launch_dense_fwd(da, s, why);
    if (rc != FA_OK) return rc;
    DenseBwdArgs ba{a.dtype, qw, kw, vw, ow, dyw, a.l, a.m, dqw, dkw, dvw, a.g.T, a.g.T, a.d, a.dv, nb,
                    a.scale, dwork, dws};
    rc = launch_dense_bwd(ba, s, why);
    if (rc != FA_OK) return rc;
    if ((e = fold<T>(dqw, a.dq, (int)a.d, a.batch, g, false, s)) != hipSuccess ||
        (e = fold<T>(dkw, a.dk, (int)a.d, a.batch, g, false, s)) != hipSuccess ||
        (e = fold<T>(dvw, a.dv_, (int)a.dv, a.batch, g, false, s)) != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    return FA_OK;
}

int launch_windowed_bwd(const WindowedBwdArgs& a, hipStream_t s, const char** why) {
    if (a.d > kMaxHeadDim || a.dv > kMaxHeadDim) {
        *why = "head dimension exceeds the compiled maximum (128)";
        return FA_ERR_UNSUPPORTED;
    }
    if (!geom_fits(a.g, a.d, a.dv, a.batch)) {
        *why = "windowed problem too large for 32-bit window indexing";
        return FA_ERR_UNSUPPORTED;
    }
    switch (a.dtype) {
        case FA_DTYPE_BF16: return windowed_bwd_typed<bf16>(a, s, why);
        case FA_DTYPE_F16: return windowed_bwd_typed<f16>(a, s, why);
        case FA_DTYPE_F32: return windowed_bwd_typed<float>(a, s, why);
    }
    *why = "unknown dtype";
    return FA_ERR_INVALID_ARG;
}

}  // namespace fa
