/*
 * fa_hip.h — C ABI of the MI355X (gfx950) flash-attention library.
 *
 * Drop-in boundary for the hot path of nikopj/FlashAttention.jl
 * (reference mounted read-only at /root/reference; citations are path:line
 * inside it).  The Julia host code binds these symbols with `ccall`
 * (INTEGRATION.md); the Python ctypes mirror in flashattention.jl_amd/fa_hip
 * binds the very same symbols, so parity evidence transfers.
 *
 * Layout contract (all entry points): the reference's Julia column-major
 * layout with contiguous batch.  A 3-D array X of Julia shape (N, d, B) sits
 * at element offset  n + N*k + N*d*b  (src/dense.jl:6-8 flattens spatial dims
 * into N).  l and m are (N, 1, B): offset n + N*b.  There is no separate head
 * dimension: (batch, heads) of the benchmark configs are one batch of B*H
 * (SURVEY.md §8a).
 *
 * Every pointer is a DEVICE pointer owned by the caller.  Inputs are read
 * only; outputs are fully written (the callee initialises, as
 * src/dense.jl:58-60 does).  `hip_stream` is a hipStream_t (NULL = default
 * stream).  Calls are asynchronous on that stream, stateless, and safe from
 * concurrent host threads on distinct streams.  No call allocates device
 * memory, synchronises, or aborts: each returns FA_OK (0) or a nonzero
 * fa_status, with a thread-local message in fa_last_error().  A workspace
 * belongs to one call at a time: calls that may run concurrently (distinct
 * streams) need distinct workspaces (the backward kernels keep hand-off
 * counters and strip counters in theirs).  A workspace may start at any
 * address: the *_workspace() sizes include 256 bytes of slack, and every entry
 * point rounds the addresses of its counters and staging buffers up to 256 B
 * inside it.
 */
#ifndef FA_HIP_H
#define FA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FA_HIP_ABI_VERSION 1

/* Element type of Q, K, V, O (and dO, dQ, dK, dV).  l, m are always float32
 * (documented deviation: the reference keeps them in T, src/dense.jl:12-13).
 * FA_DTYPE_F64 is the element type of the reference's own tests and timings
 * (test/test.jl:12, logs/compare1.txt): dense forward / backward, the windowed
 * forward / backward, window / unwindow, circulant and softmax accept it; it runs
 * fp64 SIMT parity kernels, and its backward recomputes the row statistics in
 * double instead of reading the float32 l, m. */
typedef enum fa_dtype {
    FA_DTYPE_F32  = 0,
    FA_DTYPE_BF16 = 1,
    FA_DTYPE_F16  = 2,
    FA_DTYPE_F64  = 3
} fa_dtype;

typedef enum fa_status {
    FA_OK                = 0,
    FA_ERR_INVALID_ARG   = 1, /* bad pointer / size / dtype (reference: DimensionMismatch) */
    FA_ERR_UNSUPPORTED   = 2, /* valid but unsupported (e.g. head dim > fa_max_head_dim()) */
    FA_ERR_HIP           = 3, /* HIP launch / runtime error */
    FA_ERR_WORKSPACE     = 4  /* workspace missing or too small */
} fa_status;

/* Dense forward.  Replaces the body of
 *   dense_fa!(O, l, m, Q, K, V)          src/dense.jl:21-102
 * (and, with caller-side allocation, dense_fa(q, k, v), src/dense.jl:1-19).
 *   Q (N, d, B), K (Nk, d, B), V (Nk, dv, B)  ->  O (N, dv, B),
 *   l (N, 1, B) = sum_j exp(s_ij - m_i),  m (N, 1, B) = max_j s_ij,
 *   s = scale * Q K^T  (natural-log units, as src/dense.jl:78-91).
 * scale <= 0 selects the reference's tau = 1/sqrt(d) (src/dense.jl:43).
 * The reference requires Nk == N and dv == d (Appendix A.1); both are lifted.
 * Empty inputs behave as dense_fa! does with empty arrays: N == 0 or B == 0 is a
 * no-op (no pointer is dereferenced); Nk == 0 writes O = 0, l = 0, m = -Inf, the
 * initial state of src/dense.jl:58-60.  d, dv must be >= 1. */
int fa_dense_fwd(int dtype,
                 const void* Q, const void* K, const void* V,
                 void* O, float* l, float* m,
                 int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch,
                 float scale, void* hip_stream);

/* fa_dense_fwd with a caller-owned workspace (same contract otherwise).  For
 * bf16 / fp16 with Nk % 8 != 0 the workspace holds zero-padded K / V copies of
 * row stride roundup(Nk, 8), so the ragged shape runs the fast MFMA kernels
 * instead of the generic one (3.6-6x).  workspace may be NULL
 * when fa_dense_fwd_workspace() returns 0. */
int fa_dense_fwd_ws(int dtype,
                    const void* Q, const void* K, const void* V,
                    void* O, float* l, float* m,
                    int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch,
                    float scale, void* workspace, size_t workspace_bytes,
                    void* hip_stream);

/* Workspace bytes fa_dense_fwd_ws needs for these sizes (0 is a valid answer). */
size_t fa_dense_fwd_workspace(int dtype, int64_t N, int64_t Nk, int64_t d,
                              int64_t dv, int64_t batch);

/* Workspace bytes fa_dense_bwd needs for these sizes (0 is a valid answer):
 * a 256-B header (fa_dense_bwd_handoff_status), 8·N·batch bytes of row
 * statistics; for bf16 / fp16 shapes outside the MFMA kernels' set, zero-padded
 * copies; and when the single-pass kernel applies (grids that
 * fill the chip), per-slice counters plus the running fp32 dQ sums of the two
 * chains per slice, 2·4·N·d·batch bytes (17.2 GB for configs[4]'s 1024 slabs of
 * (16384, 128)).  A
 * smaller workspace that still holds the first parts (the size this function
 * returns under fa_debug_set_bwd_mode(1)) runs the two-pass form instead.  The
 * answer depends on the current device's CU count. */
size_t fa_dense_bwd_workspace(int dtype, int64_t N, int64_t Nk, int64_t d,
                              int64_t dv, int64_t batch);

/* Dense backward.  Replaces dense_fa_backward(Q, K, V, O, dO, l, m)
 * (src/dense.jl:104-167; executable spec OneDFastBack,
 * src_cpp/FlashAttention.cpp:194-252):
 *   P = exp(s - m)/l, dV = P^T dO, dP = dO V^T, D = rowsum(dO .* O),
 *   dS = P .* (dP - D), dQ = scale dS K, dK = scale dS^T Q.
 * l, m are the forward's outputs.  dQ, dK, dV are fully written, without
 * atomics.  dK and dV are bitwise reproducible.  dQ is bitwise reproducible
 * whenever the single pass's ordered dQ hand-off completes (it sums each query
 * slice over the key blocks in a fixed order).  Every hand-off wait is on a
 * workgroup dispatched earlier in the same launch, so no co-residency is needed:
 * other streams or processes sharing the GPU slow the call down but do not make it
 * give up.  A wait gives up only as a safety net, when neither the launch's arrival
 * count nor any member of the waiting slab has made progress for
 * FA_BWD_HANDOFF_STALL_US microseconds (100 ms); dQ of that slab is then recomputed
 * by a separate pass that sums in a different order: same values within rounding,
 * not the same bits, and slower.  fa_dense_bwd_handoff_status reports whether any
 * slab did. */
#define FA_BWD_HANDOFF_STALL_US 100000
int fa_dense_bwd(int dtype,
                 const void* Q, const void* K, const void* V,
                 const void* O, const void* dO,
                 const float* l, const float* m,
                 void* dQ, void* dK, void* dV,
                 int64_t N, int64_t Nk, int64_t d, int64_t dv, int64_t batch,
                 float scale, void* workspace, size_t workspace_bytes,
                 void* hip_stream);

/* Diagnostic for the call that last used `workspace` in fa_dense_bwd: reads the
 * workspace header (synchronises hip_stream, so call it after that backward on the
 * same stream).  *status = -1: that call ran the two-pass form (no hand-off),
 * 0: single pass, every dQ hand-off completed, 1: single pass, some slab's hand-off
 * gave up and its dQ was recomputed (see fa_dense_bwd).  FA_ERR_INVALID_ARG if the workspace
 * holds no fa_dense_bwd header. */
int fa_dense_bwd_handoff_status(const void* workspace, size_t workspace_bytes,
                                void* hip_stream, int* status);

/* Windowed forward.  Replaces windowed_fa(q, k, v, ws; stride, pad)
 * (src/windowed.jl:3-23; block_fa = stride ws, src/windowed.jl:1), fusing
 * window (src/utils.jl:36-44) -> dense_fa -> unwindow / divisor
 * (src/utils.jl:46-54, src/windowed.jl:16-19) into one pass.
 *   q, k: (S_1, ..., S_k, d, B);  v: (S_1, ..., S_k, dv, B)
 *   y:    (S_1, ..., S_k, dv, B)  (pixels no window covers are NaN, as in
 *                                  the reference, Appendix A.7)
 *   l, m: (ws^k, 1, L, B) window layout (src/windowed.jl:20-21),
 *         L = prod_i ((S_i + 2 pad - ws) / stride + 1).
 * nspatial = k in 1..3; pad < 0 selects the reference default (ws-1)/2.
 * B == 0 (an empty batch) is a no-op after the geometry is validated; the
 * same holds for fa_window, fa_unwindow and fa_windowed_bwd. */
int fa_windowed_fwd(int dtype,
                    const void* q, const void* k, const void* v,
                    void* y, float* l, float* m,
                    int nspatial, const int64_t* spatial,
                    int64_t d, int64_t dv, int64_t batch,
                    int64_t ws, int64_t stride, int64_t pad,
                    float scale, void* workspace, size_t workspace_bytes,
                    void* hip_stream);

/* Workspace bytes fa_windowed_fwd needs (0 is a valid answer: the fused
 * single-pass kernel needs none; large windows / fp32 use a composed
 * gather -> dense -> fold path that stages windows in the workspace). */
size_t fa_windowed_fwd_workspace(int dtype, int nspatial, const int64_t* spatial,
                                 int64_t d, int64_t dv, int64_t batch,
                                 int64_t ws, int64_t stride, int64_t pad);

/* window(x, ws; stride, pad) — reference src/utils.jl:36-45 (NNlib.unfold):
 * x (S_1..S_k, C, batch) -> xw (ws^k, C, L, batch), zero padding outside the
 * image, window token order first-spatial-dim fastest.  xw fully written. */
int fa_window(int dtype, const void* x, void* xw,
              int nspatial, const int64_t* spatial, int64_t C, int64_t batch,
              int64_t ws, int64_t stride, int64_t pad, void* hip_stream);

/* unwindow(xw, size(x), ws; stride, pad) — reference src/utils.jl:47-54
 * (NNlib.fold): xw (ws^k, C, L, batch) -> x (S_1..S_k, C, batch), the SUM over
 * overlapping windows (0 where no window covers a pixel).  Deterministic (one
 * thread per output pixel, fixed window order).  x fully written. */
int fa_unwindow(int dtype, const void* xw, void* x,
                int nspatial, const int64_t* spatial, int64_t C, int64_t batch,
                int64_t ws, int64_t stride, int64_t pad, void* hip_stream);

/* Workspace bytes fa_windowed_bwd needs. */
size_t fa_windowed_workspace(int dtype, int nspatial, const int64_t* spatial,
                             int64_t d, int64_t dv, int64_t batch,
                             int64_t ws, int64_t stride, int64_t pad);

/* Windowed backward (README.md:36-37 claims it, no code
 * exists in the reference): the exact chain rule of windowed_fa.
 * y, l, m are fa_windowed_fwd's outputs; dq, dk, dv fully written. */
int fa_windowed_bwd(int dtype,
                    const void* q, const void* k, const void* v,
                    const void* y, const void* dy,
                    const float* l, const float* m,
                    void* dq, void* dk, void* dv_,
                    int nspatial, const int64_t* spatial,
                    int64_t d, int64_t dv, int64_t batch,
                    int64_t ws, int64_t stride, int64_t pad,
                    float scale, void* workspace, size_t workspace_bytes,
                    void* hip_stream);

/* Circulant (periodic banded) attention, replaces
 *   circulant_fa!(O, l, m, Q, K, V, W)   reference src/circulant.jl:9-118
 * (naive form circulant_dpa! src/naive/circulant.jl:8-36).  Query i attends
 * the W band entries (i - p + t) mod N, t = 0..W-1, p = (W-1)/2 — the keys
 * cartesian_circulant enumerates (src/utils.jl:6-17); W > N repeats keys.
 * Q, K: (N, d, batch); V: (N, dv, batch); O: (N, dv, batch); l, m: (N, 1, batch)
 * float32 with the dense_fa! meaning.  Any W >= 1 (the reference's own
 * benchmark uses even W, bench/compare.jl:98).  N == 0 or batch == 0 is a
 * no-op (the reference's row and batch loops run zero times). */
int fa_circulant_fwd(int dtype, const void* Q, const void* K, const void* V,
                     void* O, float* l, float* m,
                     int64_t N, int64_t d, int64_t dv, int64_t batch, int64_t W,
                     float scale, void* hip_stream);

/* Standalone fused softmax, replaces
 *   fused_softmax!(P, S; dims)   reference src/fused_softmax.jl:1-41
 * (device versions src/cuda/fused_softmax.jl:11-314).  S, P: (M, N, batch)
 * column-major, same dtype; dims = 1 normalises each column S[:, j, b]
 * (M contiguous elements), dims = 2 each row S[i, :, b].  P may equal S
 * (in place, fused_softmax!(S)).  A vector is (M, 1, 1) with dims = 1.
 * Computed in fp32; an all -Inf or NaN-containing vector gives NaN, as the
 * reference's arithmetic does.  batch == 0 is a no-op; M or N == 0 is
 * rejected (a reduction over an empty dimension). */
size_t fa_softmax_workspace(int64_t M, int64_t N, int64_t batch, int dims);
int fa_softmax(int dtype, const void* S, void* P, int64_t M, int64_t N, int64_t batch, int dims,
               void* workspace, size_t workspace_bytes, void* hip_stream);

/* Thread-local description of the last error on this host thread ("" if none). */
const char* fa_last_error(void);

/* FA_HIP_ABI_VERSION of the loaded library. */
int fa_abi_version(void);

/* Largest d (and dv) the kernels accept. */
int fa_max_head_dim(void);

#ifdef __cplusplus
}
#endif

#endif /* FA_HIP_H */
