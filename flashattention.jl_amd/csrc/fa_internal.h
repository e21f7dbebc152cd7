// fa_internal.h — host-side launcher interface between api.cpp (argument
// validation, C ABI) and the kernel translation units.  Not installed.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace fa {

struct DenseArgs {
    int dtype;                 // fa_dtype
    const void *Q, *K, *V;
    void* O;
    float *l, *m;
    int64_t N, Nk, d, dv, batch;
    float scale;               // already resolved (> 0)
    void* workspace = nullptr; // optional: padded K / V copies for ragged Nk (fa_dense_fwd_workspace)
    size_t workspace_bytes = 0;
    double scale64 = 0.0;      // Float64 kernels: τ resolved in double (0: use scale)
};

struct DenseBwdArgs {
    int dtype;
    const void *Q, *K, *V, *O, *dO;
    const float *l, *m;
    void *dQ, *dK, *dV;
    int64_t N, Nk, d, dv, batch;
    float scale;
    void* workspace;
    size_t workspace_bytes;
    double scale64 = 0.0;      // Float64 kernels: τ resolved in double (0: use scale)
};

struct WindowGeom {
    int nsp;                   // spatial rank 1..3
    int64_t S[3];              // spatial extents (first = fastest)
    int64_t O[3];              // windows per dim
    int64_t ws, stride, pad;
    int64_t T;                 // ws^nsp tokens per window
    int64_t L;                 // windows per image
    int64_t P;                 // pixels per image
};

struct WindowedArgs {
    int dtype;
    const void *q, *k, *v;
    void* y;
    float *l, *m;
    WindowGeom g;
    int64_t d, dv, batch;
    float scale;
    void* workspace;
    size_t workspace_bytes;
    double scale64 = 0.0;
};

struct WindowedBwdArgs {
    int dtype;
    const void *q, *k, *v, *y, *dy;
    const float *l, *m;
    void *dq, *dk, *dv_;
    WindowGeom g;
    int64_t d, dv, batch;
    float scale;
    void* workspace;
    size_t workspace_bytes;
    double scale64 = 0.0;
};

struct CircArgs {
    int dtype;
    const void *Q, *K, *V;
    void* O;
    float *l, *m;
    int64_t N, d, dv, batch, W;
    float scale;
    double scale64 = 0.0;      // Float64 kernel: τ resolved in double (0: use scale)
};

struct SoftmaxArgs {
    int dtype;
    const void* S;
    void* P;
    int64_t M, N, batch;
    int dims;                  // 1: over M (contiguous), 2: over N (stride M)
    void* workspace;
    size_t workspace_bytes;
};

// Each returns a hipError_t-like code through *err and a fa_status.
int launch_dense_fwd(const DenseArgs& a, hipStream_t s, const char** why);
size_t dense_fwd_workspace(int dtype, int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch);
size_t dense_bwd_workspace(int dtype, int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch);
int launch_dense_bwd(const DenseBwdArgs& a, hipStream_t s, const char** why);
int dense_bwd_handoff_status(const void* workspace, size_t workspace_bytes, hipStream_t s, int* status,
                             const char** why);
// Float64 (fa_f64.hip): the forward, and the backward's row statistics in double
// (nD = −rowsum(dO ∘ O), nlse = −(m + ln l)/τ recomputed from Q, K; [batch][N] each)
int launch_dense_fwd_f64(const DenseArgs& a, hipStream_t s, const char** why);
int launch_f64_bwd_stats(const DenseBwdArgs& a, double* nD, double* nlse, hipStream_t s, const char** why);
// element size of a fa_dtype (0: unknown)
// CUs of the device the work runs on: the stream's device (the current device for
// the NULL stream, and for fa_dense_bwd_workspace, which takes no stream); 0 on error.
inline int device_cus(hipStream_t s) {
    int dev = 0, cus = 0;
    if (s != nullptr) {
        if (hipStreamGetDevice(s, &dev) != hipSuccess) return 0;
    } else if (hipGetDevice(&dev) != hipSuccess) {
        return 0;
    }
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    return cus;
}

inline size_t dtype_size(int dtype) { return dtype == 0 ? 4 : dtype == 1 || dtype == 2 ? 2 : dtype == 3 ? 8 : 0; }
size_t windowed_workspace(int dtype, const WindowGeom& g, int64_t d, int64_t dv, int64_t batch);
size_t windowed_fwd_workspace(int dtype, const WindowGeom& g, int64_t d, int64_t dv, int64_t batch);
int launch_windowed_fwd(const WindowedArgs& a, hipStream_t s, const char** why);
int launch_windowed_bwd(const WindowedBwdArgs& a, hipStream_t s, const char** why);
int launch_circulant_fwd(const CircArgs& a, hipStream_t s, const char** why);
// window (unfold) / unwindow (fold, sum over overlaps) of one tensor (S..., C, B) <-> (T, C, L, B)
int launch_window(int dtype, const void* src, void* dst, const WindowGeom& g, int64_t C, int64_t batch,
                  bool unwindow, hipStream_t s, const char** why);
size_t softmax_workspace(int64_t M, int64_t N, int64_t batch, int dims);
int launch_softmax(const SoftmaxArgs& a, hipStream_t s, const char** why);

// Padded head-dim class a kernel is compiled for: 32, 64 or 128 (0 = none).
inline int head_dim_class(int64_t d) {
    if (d <= 32) return 32;
    if (d <= 64) return 64;
    if (d <= 128) return 128;
    return 0;
}

constexpr int kMaxHeadDim = 128;

// Debug / benchmark knobs (fa_debug_set_*; not part of include/fa_hip.h and not
// ABI state).  They are THREAD-LOCAL: a knob set on one host thread changes only
// the kernels that thread launches, so concurrent callers on other threads stay
// on the default paths and the public entry points remain stateless for them.
extern thread_local int g_fwd_variant;        // forward kernel variant
extern thread_local int g_fwd_last_path;      // 30 when the last fast forward launch ran fa_fwd_p4
extern thread_local float g_fwd_rescale_log2; // forward fast kernels: lazy-rescale threshold (log2 units)
extern thread_local int g_bwd_force_generic;  // backward: force the generic SIMT path
extern thread_local int g_bwd_mode;           // backward MFMA path: 0 auto, 1 split passes, 2 single pass
extern thread_local int g_bwd_l2local;        // single pass: running sums handed over in the XCD's L2
extern thread_local int g_bwd_hoff;           // single pass: step offset between consecutive members
extern thread_local int g_bwd_stall_us;       // single pass: no-progress bound of a poll (us)
extern thread_local int g_bwd_nodirect;       // single pass (tests): chain-B tails never add A's total themselves
extern thread_local int g_bwd_xcd;            // single pass: one XCD per slab where eligible (-1 auto, 0 never)
extern thread_local int g_win_force_composed; // windowed: forced path (composed / fused variants)
extern thread_local int g_win_bwd_grid;       // windowed: strip backward workgroups (0: one per CU)
extern thread_local int g_circ_force_generic; // circulant: forced kernel

}  // namespace fa
