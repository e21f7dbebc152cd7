// api.cpp — the extern "C" boundary declared in include/fa_hip.h.
//
// Validates arguments the way the reference's Julia methods would fail
// (DimensionMismatch → FA_ERR_INVALID_ARG), resolves the default scale
// τ = 1/√d (src/dense.jl:43), and dispatches to the kernel launchers.  No
// process-global state: the error string and the fa_debug_set_* knobs are
// thread-local (the knobs are test/benchmark hooks, not ABI); never allocates,
// synchronises or aborts.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <string>

#include "../../include/fa_hip.h"
#include "fa_internal.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fn, const char* msg) {
    g_last_error = std::string(fn) + ": " + msg;
    return code;
}

int ok() {
    g_last_error.clear();
    return FA_OK;
}

bool valid_dtype(int dt) {
    return dt == FA_DTYPE_F32 || dt == FA_DTYPE_BF16 || dt == FA_DTYPE_F16 || dt == FA_DTYPE_F64;
}

float resolve_scale(float scale, int64_t d) {
    if (!(scale > 0.0f) || !std::isfinite(scale)) return (float)(1.0 / std::sqrt((double)d));
    return scale;
}
// τ for the Float64 kernels: the default 1/√d in double (src/dense.jl:43), else the
// caller's float scale widened.
double resolve_scale64(float scale, int64_t d) {
    if (!(scale > 0.0f) || !std::isfinite(scale)) return 1.0 / std::sqrt((double)d);
    return (double)scale;
}

// Empty inputs, as dense_fa! (src/dense.jl:21-102) treats them: N = 0 or batch = 0
// runs no tile (nothing to write); Nk = 0 leaves the initial O = 0, l = 0,
// m = −Inf (:58-60).  Returns true when the call is complete.
bool dense_fwd_empty(int dtype, void* O, float* l, float* m, int64_t N, int64_t Nk, int64_t dv, int64_t batch,
                     hipStream_t s, int* rc) {
    *rc = FA_OK;
    if (N == 0 || batch == 0) return true;
    if (Nk != 0) return false;
    const size_t esz = fa::dtype_size(dtype);
    if (!O || !l || !m) { *rc = FA_ERR_INVALID_ARG; return true; }
    if (hipMemsetAsync(O, 0, (size_t)(N * dv * batch) * esz, s) != hipSuccess ||
        hipMemsetAsync(l, 0, (size_t)(N * batch) * 4, s) != hipSuccess ||
        hipMemsetD32Async((hipDeviceptr_t)m, 0xFF800000u, (size_t)(N * batch), s) != hipSuccess)
        *rc = FA_ERR_HIP;
    return true;
}

// Window geometry of NNlib.unfold(x, (ws…, d, 1); stride, pad) (src/utils.jl:40).
int make_geom(fa::WindowGeom& g, int nspatial, const int64_t* spatial, int64_t ws, int64_t stride,
              int64_t pad, const char** why) {
    if (nspatial < 1 || nspatial > 3 || !spatial) { *why = "nspatial must be 1, 2 or 3"; return FA_ERR_INVALID_ARG; }
    if (ws < 1) { *why = "window size must be >= 1"; return FA_ERR_INVALID_ARG; }
    if (stride < 1) { *why = "stride must be >= 1"; return FA_ERR_INVALID_ARG; }
    if (pad < 0) pad = (ws - 1) / 2;
    g.nsp = nspatial;
    g.ws = ws;
    g.stride = stride;
    g.pad = pad;
    g.T = 1;
    g.L = 1;
    g.P = 1;
    for (int i = 0; i < 3; ++i) { g.S[i] = 1; g.O[i] = 1; }
    for (int i = 0; i < nspatial; ++i) {
        if (spatial[i] < 1) { *why = "spatial extents must be >= 1"; return FA_ERR_INVALID_ARG; }
        const int64_t span = spatial[i] + 2 * pad - ws;
        if (span < 0) { *why = "window larger than the padded input"; return FA_ERR_INVALID_ARG; }
        g.S[i] = spatial[i];
        g.O[i] = span / stride + 1;
        g.T *= ws;
        g.L *= g.O[i];
        g.P *= spatial[i];
    }
    return FA_OK;
}

}  // namespace

extern "C" {

const char* fa_last_error(void) { return g_last_error.c_str(); }

int fa_abi_version(void) { return FA_HIP_ABI_VERSION; }

int fa_max_head_dim(void) { return fa::kMaxHeadDim; }

// Not part of the public header: selects the forward kernel variant for A/B
// benchmarking: 0 = auto (per head-dim class), 5 / 7 = 8 waves x {1, 2} query
// blocks per wave on 32x32x16 MFMA; 20 = the default geometries with per-element Q
// gathers and O stores; 30 = the one-wave-per-SIMD persistent kernel (fa_fwd_p4.hip)
// where its shape rules allow.  (The measured-and-rejected 4-wave, 16x16x32 and
// 4-waves-per-SIMD geometries were removed in round 4, the persistent 8-wave d <= 64
// kernel, a measured tie, in round 6; git history keeps them.)
int fa_debug_set_fwd_variant(int v) {
    const int old = fa::g_fwd_variant;
    if (v == 0 || v == 5 || v == 7 || v == 20 || v == 30) fa::g_fwd_variant = v;
    return old;
}

// Not part of the public header: 30 when the calling thread's last forward ran the
// one-wave-per-SIMD kernel (fa_fwd_p4.hip), 0 otherwise (tests, bench labels).
int fa_debug_fwd_last_path(void) { return fa::g_fwd_last_path; }

// Not part of the public header: lazy-rescale threshold of the bf16/f16 forward
// kernels in log2 units (default 8; 0 = rescale on every max increase, the
// textbook order).  Accuracy tests only; returns the previous value.
float fa_debug_set_rescale_threshold(float t) {
    const float old = fa::g_fwd_rescale_log2;
    if (t >= 0.0f && t <= 16.0f) fa::g_fwd_rescale_log2 = t;
    return old;
}

// Not part of the public header: 1 forces the generic (SIMT) backward.
int fa_debug_set_bwd_generic(int v) {
    const int old = fa::g_bwd_force_generic;
    fa::g_bwd_force_generic = v != 0;
    return old;
}

// Not part of the public header: backward MFMA path (0 auto, 1 the dK/dV + dQ
// passes, 2 the single pass wherever its shape conditions hold, 3 as 2 with the
// hand-off's timeout word preset, which exercises the dQ fallback pass).  Builds with
// -DFA_BWD_ABL also accept the timing-only ablations of the single pass, which compute
// a WRONG dQ: 4, 5, 6 no waits, no running-sum traffic, neither; 7, 8 no running-sum
// loads / stores; 9 no dS image writes; 10 no next-slice Q/dO DMA; 11 = 10 + 6.  Any other value is rejected (returns -1, the
// mode is unchanged).
int fa_debug_set_bwd_mode(int v) {
    const int old = fa::g_bwd_mode;
#ifdef FA_BWD_ABL
    constexpr int kMaxMode = 11;
#else
    constexpr int kMaxMode = 3;
#endif
    if (v < 0 || v > kMaxMode) return -1;
    fa::g_bwd_mode = v;
    return old;
}

// Not part of the public header: the single-pass backward hands its running dQ sums
// over in the XCD's L2 when all of a slab's members run on one XCD (plain stores instead
// of sc1 write-through): -1 auto (d, dv <= 64), 0 never, 1 always; returns the previous
// value (-2 for an invalid argument).
int fa_debug_set_bwd_l2local(int v) {
    const int old = fa::g_bwd_l2local;
    if (v < -1 || v > 1) return -2;
    fa::g_bwd_l2local = v;
    return old;
}

// Not part of the public header: the single-pass backward's slab placement: -1 auto (a
// slab's members on one XCD when they fit), 0 members dealt over the whole chip;
// returns the previous value (-2 for an invalid argument).
int fa_debug_set_bwd_xcd(int v) {
    const int old = fa::g_bwd_xcd;
    if (v < -1 || v > 0) return -2;
    fa::g_bwd_xcd = v;
    return old;
}

// Not part of the public header: the single-pass backward's step offset between
// consecutive members of a slice's chain (1..4, default 3); returns the previous value
// (-2 for an invalid argument).
int fa_debug_set_bwd_hoff(int v) {
    const int old = fa::g_bwd_hoff;
    if (v < 1 || v > 4) return -2;
    fa::g_bwd_hoff = v;
    return old;
}

// Not part of the public header: the single-pass backward's no-progress bound in
// microseconds (a poll gives up when the launch published nothing for this long;
// 10..10000000, default 100000); returns the previous value (-2 for an invalid argument).
int fa_debug_set_bwd_stall_us(int v) {
    const int old = fa::g_bwd_stall_us;
    if (v < 10 || v > 10000000) return -2;
    fa::g_bwd_stall_us = v;
    return old;
}

// Not part of the public header (tests): 1 makes every chain-B tail of the single-pass
// backward store its total and leave dQ = A + B of the wrapped slices to the guarded dQ
// pass's combine (the path a co-tenant can force), 0 the default; returns the previous
// value (-2 for an invalid argument).
int fa_debug_set_bwd_nodirect(int v) {
    const int old = fa::g_bwd_nodirect;
    if (v < 0 || v > 1) return -2;
    fa::g_bwd_nodirect = v;
    return old;
}

// Not part of the public header: circulant kernel override (1 one-wave-per-query,
// 2 LDS-tiled SIMT; 0 auto).
int fa_debug_set_circ_generic(int v) {
    const int old = fa::g_circ_force_generic;
    fa::g_circ_force_generic = (v == 1 || v == 2) ? v : 0;
    return old;
}

// Not part of the public header: windowed forward path override (1 composed,
// 2 register-gather fused, 3 one-window row-shift (ws <= 7) / row-scatter, 4 four-window
// row-scatter, 5 one-window row-scatter, 6 two-window row-shift (the auto choice at ws <= 7),
// 10 eight-window strip (stride == ws), 12 three-window row-shift, where eligible; 13: the
// per-window backward with two windows per workgroup; 0 auto).  Modes 7-9 (rejected
// experimental kernels) were removed; they now select the auto path.
int fa_debug_set_win_composed(int v) {
    const int old = fa::g_win_force_composed;
    fa::g_win_force_composed = ((v >= 1 && v <= 6) || v == 10 || v == 12 || v == 13) ? v : 0;
    return old;
}

// Not part of the public header: workgroups of the persistent strip backward (0 = one per
// CU, the default; 1..4096 caps the grid).  Benchmark knob; returns the previous value.
int fa_debug_set_win_bwd_grid(int v) {
    const int old = fa::g_win_bwd_grid;
    if (v >= 0 && v <= 4096) fa::g_win_bwd_grid = v;
    return old;
}

size_t fa_dense_fwd_workspace(int dtype, int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch) {
    if (!valid_dtype(dtype) || N < 1 || Nk < 1 || d < 1 || dv < 1 || batch < 1) return 0;
    return fa::dense_fwd_workspace(dtype, N, Nk, d, dv, batch);
}

int fa_dense_fwd_ws(int dtype, const void* Q, const void* K, const void* V, void* O, float* l, float* m,
                    int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch, float scale,
                    void* workspace, size_t workspace_bytes, void* hip_stream) {
    static const char* fn = "fa_dense_fwd_ws";
    if (!valid_dtype(dtype)) return fail(FA_ERR_INVALID_ARG, fn, "unknown dtype");
    if (N < 0 || Nk < 0 || d < 1 || dv < 1 || batch < 0)
        return fail(FA_ERR_INVALID_ARG, fn, "DimensionMismatch: N, Nk, batch must be >= 0 and d, dv >= 1");
    int erc;
    if (dense_fwd_empty(dtype, O, l, m, N, Nk, dv, batch, (hipStream_t)hip_stream, &erc))
        return erc == FA_OK ? ok() : fail(erc, fn, erc == FA_ERR_HIP ? "hipMemsetAsync failed" : "null pointer");
    if (!Q || !K || !V || !O || !l || !m) return fail(FA_ERR_INVALID_ARG, fn, "null pointer");
    const size_t need = fa::dense_fwd_workspace(dtype, N, Nk, d, dv, batch);
    if (need > 0 && (!workspace || workspace_bytes < need))
        return fail(FA_ERR_WORKSPACE, fn, "workspace missing or smaller than fa_dense_fwd_workspace()");
    fa::DenseArgs a{dtype, Q, K, V, O, l, m, N, Nk, d, dv, batch, resolve_scale(scale, d)};
    a.scale64 = resolve_scale64(scale, d);
    a.workspace = workspace;
    a.workspace_bytes = workspace_bytes;
    const char* why = "";
    const int rc = fa::launch_dense_fwd(a, (hipStream_t)hip_stream, &why);
    return rc == FA_OK ? ok() : fail(rc, fn, why);
}

int fa_dense_fwd(int dtype, const void* Q, const void* K, const void* V, void* O, float* l, float* m,
                 int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch, float scale,
                 void* hip_stream) {
    static const char* fn = "fa_dense_fwd";
    if (!valid_dtype(dtype)) return fail(FA_ERR_INVALID_ARG, fn, "unknown dtype");
    if (N < 0 || Nk < 0 || d < 1 || dv < 1 || batch < 0)
        return fail(FA_ERR_INVALID_ARG, fn, "DimensionMismatch: N, Nk, batch must be >= 0 and d, dv >= 1");
    int erc;
    if (dense_fwd_empty(dtype, O, l, m, N, Nk, dv, batch, (hipStream_t)hip_stream, &erc))
        return erc == FA_OK ? ok() : fail(erc, fn, erc == FA_ERR_HIP ? "hipMemsetAsync failed" : "null pointer");
    if (!Q || !K || !V || !O || !l || !m) return fail(FA_ERR_INVALID_ARG, fn, "null pointer");
    fa::DenseArgs a{dtype, Q, K, V, O, l, m, N, Nk, d, dv, batch, resolve_scale(scale, d)};
    a.scale64 = resolve_scale64(scale, d);
    const char* why = "";
    const int rc = fa::launch_dense_fwd(a, (hipStream_t)hip_stream, &why);
    return rc == FA_OK ? ok() : fail(rc, fn, why);
}

size_t fa_dense_bwd_workspace(int dtype, int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch) {
    if (!valid_dtype(dtype) || N < 1 || Nk < 1 || d < 1 || dv < 1 || batch < 1) return 0;
    return fa::dense_bwd_workspace(dtype, N, Nk, d, dv, batch);
}

int fa_dense_bwd(int dtype, const void* Q, const void* K, const void* V, const void* O, const void* dO,
                 const float* l, const float* m, void* dQ, void* dK, void* dV, int64_t N, int64_t Nk,
                 int64_t d, int64_t dv, int64_t batch, float scale, void* workspace,
                 size_t workspace_bytes, void* hip_stream) {
    static const char* fn = "fa_dense_bwd";
    if (!valid_dtype(dtype)) return fail(FA_ERR_INVALID_ARG, fn, "unknown dtype");
    if (N < 0 || Nk < 0 || d < 1 || dv < 1 || batch < 0)
        return fail(FA_ERR_INVALID_ARG, fn, "DimensionMismatch: N, Nk, batch must be >= 0 and d, dv >= 1");
    if (N == 0 || Nk == 0 || batch == 0) {   // empty sums: every gradient element is 0
        const size_t esz = fa::dtype_size(dtype);
        const hipStream_t s = (hipStream_t)hip_stream;
        const size_t nq = (size_t)(N * d * batch), nk = (size_t)(Nk * d * batch), nv = (size_t)(Nk * dv * batch);
        if ((nq && !dQ) || (nk && (!dK || !dV))) return fail(FA_ERR_INVALID_ARG, fn, "null pointer");
        if ((nq && hipMemsetAsync(dQ, 0, nq * esz, s) != hipSuccess) ||
            (nk && hipMemsetAsync(dK, 0, nk * esz, s) != hipSuccess) ||
            (nv && hipMemsetAsync(dV, 0, nv * esz, s) != hipSuccess))
            return fail(FA_ERR_HIP, fn, "hipMemsetAsync failed");
        return ok();
    }
    if (!Q || !K || !V || !O || !dO || !l || !m || !dQ || !dK || !dV)
        return fail(FA_ERR_INVALID_ARG, fn, "null pointer");
    const size_t need = fa::dense_bwd_workspace(dtype, N, Nk, d, dv, batch);
    if (need > 0 && (!workspace || workspace_bytes < need))
        return fail(FA_ERR_WORKSPACE, fn, "workspace missing or smaller than fa_dense_bwd_workspace()");
    fa::DenseBwdArgs a{dtype, Q, K, V, O, dO, l, m, dQ, dK, dV, N, Nk, d, dv, batch,
                       resolve_scale(scale, d), workspace, workspace_bytes};
    a.scale64 = resolve_scale64(scale, d);
    const char* why = "";
    const int rc = fa::launch_dense_bwd(a, (hipStream_t)hip_stream, &why);
    return rc == FA_OK ? ok() : fail(rc, fn, why);
}

int fa_dense_bwd_handoff_status(const void* workspace, size_t workspace_bytes, void* hip_stream, int* status) {
    static const char* fn = "fa_dense_bwd_handoff_status";
    if (!status) return fail(FA_ERR_INVALID_ARG, fn, "null status pointer");
    const char* why = "";
    const int rc = fa::dense_bwd_handoff_status(workspace, workspace_bytes, (hipStream_t)hip_stream, status, &why);
    return rc == FA_OK ? ok() : fail(rc, fn, why);
}

size_t fa_windowed_workspace(int dtype, int nspatial, const int64_t* spatial, int64_t d, int64_t dv,
                             int64_t batch, int64_t ws, int64_t stride, int64_t pad) {
    fa::WindowGeom g;
    const char* why = "";
    if (!valid_dtype(dtype) || d < 1 || dv < 1 || batch < 1) return 0;
    if (make_geom(g, nspatial, spatial, ws, stride, pad, &why) != FA_OK) return 0;
    return fa::windowed_workspace(dtype, g, d, dv, batch);
}

size_t fa_windowed_fwd_workspace(int dtype, int nspatial, const int64_t* spatial, int64_t d, int64_t dv,
                                 int64_t batch, int64_t ws, int64_t stride, int64_t pad) {
    fa::WindowGeom g;
    const char* why = "";
    if (!valid_dtype(dtype) || d < 1 || dv < 1 || batch < 1) return 0;
    if (make_geom(g, nspatial, spatial, ws, stride, pad, &why) != FA_OK) return 0;
    return fa::windowed_fwd_workspace(dtype, g, d, dv, batch);
}

int fa_windowed_fwd(int dtype, const void* q, const void* k, const void* v, void* y, float* l, float* m,
                    int nspatial, const int64_t* spatial, int64_t d, int64_t dv, int64_t batch,
                    int64_t ws, int64_t stride, int64_t pad, float scale, void* workspace,
                    size_t workspace_bytes, void* hip_stream) {
    static const char* fn = "fa_windowed_fwd";
    if (!valid_dtype(dtype)) return fail(FA_ERR_INVALID_ARG, fn, "unknown dtype");
    if (d < 1 || dv < 1 || batch < 0)
        return fail(FA_ERR_INVALID_ARG, fn, "DimensionMismatch: d, dv must be >= 1, batch >= 0");
    fa::WindowedArgs a{};
    const char* why = "";
    int rc = make_geom(a.g, nspatial, spatial, ws, stride, pad, &why);
    if (rc != FA_OK) return fail(rc, fn, why);
    if (batch == 0) return ok();   // no image: windowed_fa on an empty batch computes nothing
    if (!q || !k || !v || !y || !l || !m) return fail(FA_ERR_INVALID_ARG, fn, "null pointer");
    a.dtype = dtype; a.q = q; a.k = k; a.v = v; a.y = y; a.l = l; a.m = m;
    a.d = d; a.dv = dv; a.batch = batch;
    a.scale = resolve_scale(scale, d);
    a.scale64 = resolve_scale64(scale, d);
    const size_t need = fa::windowed_fwd_workspace(dtype, a.g, d, dv, batch);
    if (need > 0 && (!workspace || workspace_bytes < need))
        return fail(FA_ERR_WORKSPACE, fn, "workspace missing or smaller than fa_windowed_fwd_workspace()");
    a.workspace = workspace;
    a.workspace_bytes = workspace_bytes;
    rc = fa::launch_windowed_fwd(a, (hipStream_t)hip_stream, &why);
    return rc == FA_OK ? ok() : fail(rc, fn, why);
}

static int window_common(const char* fn, int dtype, const void* src, void* dst, int nspatial,
                         const int64_t* spatial, int64_t C, int64_t batch, int64_t ws, int64_t stride,
                         int64_t pad, bool unwindow, void* hip_stream) {
    if (!valid_dtype(dtype)) return fail(FA_ERR_INVALID_ARG, fn, "unknown dtype");
    if (C < 1 || batch < 0) return fail(FA_ERR_INVALID_ARG, fn, "DimensionMismatch: C must be >= 1, batch >= 0");
    fa::WindowGeom g{};
    const char* why = "";
    int rc = make_geom(g, nspatial, spatial, ws, stride, pad, &why);
    if (rc != FA_OK) return fail(rc, fn, why);
    if (batch == 0) return ok();   // empty batch: nothing to move
    if (!src || !dst) return fail(FA_ERR_INVALID_ARG, fn, "null pointer");
    rc = fa::launch_window(dtype, src, dst, g, C, batch, unwindow, (hipStream_t)hip_stream, &why);
    return rc == FA_OK ? ok() : fail(rc, fn, why);
}

int fa_window(int dtype, const void* x, void* xw, int nspatial, const int64_t* spatial, int64_t C,
              int64_t batch, int64_t ws, int64_t stride, int64_t pad, void* hip_stream) {
    return window_common("fa_window", dtype, x, xw, nspatial, spatial, C, batch, ws, stride, pad, false,
                         hip_stream);
}

int fa_unwindow(int dtype, const void* xw, void* x, int nspatial, const int64_t* spatial, int64_t C,
                int64_t batch, int64_t ws, int64_t stride, int64_t pad, void* hip_stream) {
    return window_common("fa_unwindow", dtype, xw, x, nspatial, spatial, C, batch, ws, stride, pad, true,
                         hip_stream);
}

int fa_windowed_bwd(int dtype, const void* q, const void* k, const void* v, const void* y, const void* dy,
                    const float* l, const float* m, void* dq, void* dk, void* dv_, int nspatial,
                    const int64_t* spatial, int64_t d, int64_t dv, int64_t batch, int64_t ws,
                    int64_t stride, int64_t pad, float scale, void* workspace, size_t workspace_bytes,
                    void* hip_stream) {
    static const char* fn = "fa_windowed_bwd";
    if (!valid_dtype(dtype)) return fail(FA_ERR_INVALID_ARG, fn, "unknown dtype");
    if (d < 1 || dv < 1 || batch < 0)
        return fail(FA_ERR_INVALID_ARG, fn, "DimensionMismatch: d, dv must be >= 1, batch >= 0");
    fa::WindowedBwdArgs a{};
    const char* why = "";
    int rc = make_geom(a.g, nspatial, spatial, ws, stride, pad, &why);
    if (rc != FA_OK) return fail(rc, fn, why);
    if (batch == 0) return ok();   // no image, no gradient element
    if (!q || !k || !v || !y || !dy || !l || !m || !dq || !dk || !dv_)
        return fail(FA_ERR_INVALID_ARG, fn, "null pointer");
    const size_t need = fa::windowed_workspace(dtype, a.g, d, dv, batch);
    if (need > 0 && (!workspace || workspace_bytes < need))
        return fail(FA_ERR_WORKSPACE, fn, "workspace missing or smaller than fa_windowed_workspace()");
    a.dtype = dtype; a.q = q; a.k = k; a.v = v; a.y = y; a.dy = dy; a.l = l; a.m = m;
    a.dq = dq; a.dk = dk; a.dv_ = dv_;
    a.d = d; a.dv = dv; a.batch = batch;
    a.scale = resolve_scale(scale, d);
    a.scale64 = resolve_scale64(scale, d);
    a.workspace = workspace;
    a.workspace_bytes = workspace_bytes;
    rc = fa::launch_windowed_bwd(a, (hipStream_t)hip_stream, &why);
    return rc == FA_OK ? ok() : fail(rc, fn, why);
}

int fa_circulant_fwd(int dtype, const void* Q, const void* K, const void* V, void* O, float* l, float* m,
                     int64_t N, int64_t d, int64_t dv, int64_t batch, int64_t W, float scale,
                     void* hip_stream) {
    static const char* fn = "fa_circulant_fwd";
    if (!valid_dtype(dtype)) return fail(FA_ERR_INVALID_ARG, fn, "unknown dtype");
    if (N < 0 || d < 1 || dv < 1 || batch < 0)
        return fail(FA_ERR_INVALID_ARG, fn, "DimensionMismatch: d, dv must be >= 1, N, batch >= 0");
    if (W < 1) return fail(FA_ERR_INVALID_ARG, fn, "DimensionMismatch: window size W must be >= 1");
    if (N == 0 || batch == 0) return ok();   // circulant_fa! loops over no row / slab
    if (!Q || !K || !V || !O || !l || !m) return fail(FA_ERR_INVALID_ARG, fn, "null pointer");
    fa::CircArgs a{dtype, Q, K, V, O, l, m, N, d, dv, batch, W, resolve_scale(scale, d)};
    a.scale64 = resolve_scale64(scale, d);
    const char* why = "";
    const int rc = fa::launch_circulant_fwd(a, (hipStream_t)hip_stream, &why);
    return rc == FA_OK ? ok() : fail(rc, fn, why);
}

size_t fa_softmax_workspace(int64_t M, int64_t N, int64_t batch, int dims) {
    if (M < 1 || N < 1 || batch < 1 || (dims != 1 && dims != 2)) return 0;
    return fa::softmax_workspace(M, N, batch, dims);
}

int fa_softmax(int dtype, const void* S, void* P, int64_t M, int64_t N, int64_t batch, int dims,
               void* workspace, size_t workspace_bytes, void* hip_stream) {
    static const char* fn = "fa_softmax";
    if (!valid_dtype(dtype)) return fail(FA_ERR_INVALID_ARG, fn, "unknown dtype");
    if (dims != 1 && dims != 2) return fail(FA_ERR_INVALID_ARG, fn, "only softmax in dims 1 or 2 supported");
    if (M < 1 || N < 1 || batch < 0)
        return fail(FA_ERR_INVALID_ARG, fn, "DimensionMismatch: M, N must be >= 1, batch >= 0");
    if (batch == 0) return ok();   // no matrix to normalise
    if (!S || !P) return fail(FA_ERR_INVALID_ARG, fn, "null pointer");
    const size_t need = fa::softmax_workspace(M, N, batch, dims);
    if (need > 0 && (!workspace || workspace_bytes < need))
        return fail(FA_ERR_WORKSPACE, fn, "workspace missing or smaller than fa_softmax_workspace()");
    fa::SoftmaxArgs a{dtype, S, P, M, N, batch, dims, workspace, workspace_bytes};
    const char* why = "";
    const int rc = fa::launch_softmax(a, (hipStream_t)hip_stream, &why);
    return rc == FA_OK ? ok() : fail(rc, fn, why);
}

}  // extern "C"
