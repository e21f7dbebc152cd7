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
#include <type_traits>

#include "fa_common.h"
#include "fa_internal.h"
#include "../../include/fa_hip.h"

// Phase-timestamp hook for latency studies (tools/exp/win_stamp.hip defines it);
// compiled out of the product library.
#ifndef FA_STAMP
#define FA_STAMP(k)
#endif
#ifndef FA_BSTAMP   // the persistent strip backward's per-strip hook: 0 start, 1 + j load j landed,
                    // 9 + c dV chunk c, 11 + c dK chunk c, 13 + c dQ chunk c stored, 15 end
#define FA_BSTAMP(k)
#endif
// Timing-only ablations of win_rows1s (tools/exp/win_ablate.hip; 0 in the product):
// 1 = no y stores, 2 = every row load from one address; of win_strip
// (tools/exp/strip_stamp.py): 4 = no y strip-image writes, 8 = no y global stores,
// 16 = no 2-B stores of the chunks shared with a neighbour strip; of win_bwd_strip
// (tools/exp/bwd_strip_stamp.py): 32 = no gradient stores, 64 = no gradient image writes
#ifndef FA_WIN_ABL
#define FA_WIN_ABL 0
#endif

// FA_WIN_PART: this file is compiled twice (Makefile): 1 = the forward entry points (with
// the scheduler's register-pressure trackers: the strip forward -1.5 % at configs[2]
// B = 32), 2 = the backward's (without: its strip kernel +0.6 % with them); 0 (a direct
// include, e.g. the stamp harnesses) = both.  Kernels are templates, so each part emits
// the ones its entry points instantiate.
#ifndef FA_WIN_PART
#define FA_WIN_PART 0
#endif

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
    typedef typename std::conditional<sizeof(T) == 8, double, float>::type A;   // Float64 stays double
    A v = (A)0;
    if (pix >= 0) {
        v = (A)src[(b * C + c) * (int64_t)g.P + pix];
        if constexpr (DIVIDE) v /= (A)win_count(g, pix);
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
    typedef typename std::conditional<sizeof(T) == 8, double, float>::type A;   // Float64 stays double
    A acc = (A)0;
    int cnt = 0;
    for (int o3 = lo[2]; o3 <= hi[2]; ++o3)
        for (int o2 = lo[1]; o2 <= hi[1]; ++o2)
            for (int o1 = lo[0]; o1 <= hi[0]; ++o1) {
                const int t1 = x[0] + g.pad - o1 * g.stride;
                const int t2 = g.nsp > 1 ? x[1] + g.pad - o2 * g.stride : 0;
                const int t3 = g.nsp > 2 ? x[2] + g.pad - o3 * g.stride : 0;
                const int w = o1 + g.O[0] * (o2 + g.O[1] * o3);
                const int t = t1 + g.ws * (t2 + g.ws * t3);
                acc += (A)src[t + (int64_t)g.T * (c + (int64_t)C * (w + (int64_t)g.L * b))];
                ++cnt;
            }
    if constexpr (DIVIDE) acc = acc / (A)cnt;   // 0/0 = NaN where uncovered (reference semantics)
    dst[e] = (T)acc;
}


// --------------------------------------------------------------------------
// Fused single-pass windowed forward (bf16 / fp16, T <= 64 tokens per window,
// d, dv <= 64): one wave per window, 4 windows per workgroup.
//
// The window's pixel indices go to a 64-entry LDS table; Q, K and V are then
// gathered straight from the image into MFMA fragment registers with buffer
// loads (the zero-padding pixels read as 0 through an out-of-range offset), so
// no window batch is ever materialised in HBM.  Scores are the transposed
// tile Sᵀ = K·Qᵀ (keys on accumulator rows, natural key order), softmax is
// exact per window (all keys in registers: max over 2 key blocks + one
// permlane swap), and Oᵀ = Vᵀ·Pᵀ takes P straight from the accumulator.
// Query blocks of 32 are processed one after the other to bound registers.
// Output: stride >= ws (no overlap) stores y directly (each covered pixel has
// exactly one owner window; uncovered pixels are NaN-filled separately), else
// the window outputs go to the workspace and win_fold sums / divides.
// --------------------------------------------------------------------------
template <class T, int D, int DV, int NKB, bool DIRECT>
__global__ __launch_bounds__(256, 2) void win_fused(const T* __restrict__ q, const T* __restrict__ k,
                                                    const T* __restrict__ v, T* __restrict__ out,
                                                    float* __restrict__ lo, float* __restrict__ mo,
                                                    WinDev g, int d, int dv, int batch, float scale,
                                                    float scale_log2) {
    typedef typename Frag8<T>::type F8;
    __shared__ int ptab[4][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
    const int64_t wid = (int64_t)blockIdx.x * 4 + wave;       // global window id (w + L·b)
    const bool live = wid < (int64_t)g.L * batch;
    const int w = live ? (int)(wid % g.L) : 0;
    const int b = live ? (int)(wid / g.L) : 0;
    ptab[wave][lane] = (live && lane < g.T) ? win_pixel(g, w, lane) : -1;
    __syncthreads();
    const int* tab = ptab[wave];
    constexpr unsigned kOOB = 0x7FFFFFF0u;                      // past any slab: buffer load → 0
    const auto qrs = __builtin_amdgcn_make_buffer_rsrc((void*)(q + (int64_t)b * d * g.P), (short)0, d * g.P * 2, 0x00020000);
    const auto krs = __builtin_amdgcn_make_buffer_rsrc((void*)(k + (int64_t)b * d * g.P), (short)0, d * g.P * 2, 0x00020000);
    const auto vrs = __builtin_amdgcn_make_buffer_rsrc((void*)(v + (int64_t)b * dv * g.P), (short)0, dv * g.P * 2, 0x00020000);
    auto off = [&](int f, int pix) -> unsigned { return pix < 0 ? kOOB : (unsigned)((f * g.P + pix) * 2); };
    auto ld = [&](__amdgpu_buffer_rsrc_t rs, unsigned o) -> T {
        return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b16(rs, o, 0, 0));
    };

    // K: A operand of Sᵀ (row = key kb·32 + r), V: A operand of Oᵀ (row = feature)
    F8 kf[NKB][D / 16], vf[DV / 32][NKB][2];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
        const int pk = tab[kb * 32 + r];
#pragma unroll
        for (int s = 0; s < D / 16; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e) kf[kb][s][e] = ld(krs, off(16 * s + 8 * h + e, pk));
    }
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            // B-operand k order of the accumulator: element j of half h ↔ row 16s + 8(j>>2) + 4h + (j&3)
            int pv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) pv[j] = tab[kb * 32 + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3)];
#pragma unroll
            for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                for (int j = 0; j < 8; ++j) vf[cb][kb][s][j] = ld(vrs, off(cb * 32 + r, pv[j]));
        }

    const int T_ = g.T;
#pragma unroll
    for (int qb = 0; qb < NKB; ++qb) {
        const int tq = qb * 32 + r;                 // this lane's query token
        const int pq = tab[tq];
        F8 qf[D / 16];
#pragma unroll
        for (int s = 0; s < D / 16; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e) qf[s][e] = ld(qrs, off(16 * s + 8 * h + e, pq));
        f32x16 sa[NKB];
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
#pragma unroll
            for (int x = 0; x < 16; ++x) sa[kb][x] = 0.0f;
#pragma unroll
            for (int s = 0; s < D / 16; ++s) sa[kb] = mfma32x32x16(kf[kb][s], qf[s], sa[kb]);
#pragma unroll
            for (int x = 0; x < 16; ++x)
                if (kb * 32 + acc_row(x, h) >= T_) sa[kb][x] = kNegInf;   // tokens past the window
        }
        float pm[4] = {kNegInf, kNegInf, kNegInf, kNegInf};
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x) pm[x & 3] = vmax(pm[x & 3], sa[kb][x]);
        const float mt = swap_halves_max(vmax(vmax(pm[0], pm[1]), vmax(pm[2], pm[3])));
        const float mc = mt * scale_log2;
        float ps[4] = {0.f, 0.f, 0.f, 0.f};
        F8 pf[NKB][2];
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const float pr = exp2_fast(fmaf(sa[kb][x], scale_log2, -mc));
                ps[x & 3] += pr;
                pf[kb][x >> 3][x & 7] = (T)pr;
            }
        const float lt = swap_halves_sum((ps[0] + ps[1]) + (ps[2] + ps[3]));
        const float inv = 1.0f / lt;
        f32x16 oa[DV / 32];
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb) {
#pragma unroll
            for (int x = 0; x < 16; ++x) oa[cb][x] = 0.0f;
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int s = 0; s < 2; ++s) oa[cb] = mfma32x32x16(vf[cb][kb][s], pf[kb][s], oa[cb]);
        }
        if (live && tq < T_) {
            if (h == 0) {
                const int64_t li = tq + (int64_t)T_ * wid;
                mo[li] = mt * scale;
                lo[li] = lt;
            }
            if constexpr (DIRECT) {
                if (pq >= 0) {
                    T* yb = out + (int64_t)b * dv * g.P + pq;
#pragma unroll
                    for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                        for (int x = 0; x < 16; ++x) {
                            const int cc = cb * 32 + acc_row(x, h);
                            if (cc < dv) yb[(int64_t)cc * g.P] = (T)(oa[cb][x] * inv);
                        }
                }
            } else {
                T* ob = out + (int64_t)T_ * dv * wid + tq;      // (T, dv, L·B) window batch
#pragma unroll
                for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                    for (int x = 0; x < 16; ++x) {
                        const int cc = cb * 32 + acc_row(x, h);
                        if (cc < dv) ob[(int64_t)cc * T_] = (T)(oa[cb][x] * inv);
                    }
            }
        }
    }
}

// NaN for pixels no window covers (reference 0/0, Appendix A.7); DIRECT mode only
template <class T>
__global__ __launch_bounds__(256) void win_nan_uncovered(T* __restrict__ y, int dv, int64_t total, WinDev g) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    const int pix = (int)(e % g.P);
    if (win_count(g, pix) == 0) y[e] = (T)__builtin_nanf("");
}

static bool fully_covered(const WindowGeom& g) {
    for (int i = 0; i < g.nsp; ++i) {
        if (g.stride > g.ws) return false;                                  // gaps between windows
        if (-g.pad > 0) return false;
        if ((g.O[i] - 1) * g.stride - g.pad + g.ws - 1 < g.S[i] - 1) return false;   // uncovered tail
    }
    return true;
}

// --------------------------------------------------------------------------
// Row-staged single-pass windowed forward (2-D, stride >= ws, ws <= 8,
// bf16/fp16, d, dv <= 64, image width % 8 == 0).  The register-gather kernel
// above is texture-addresser bound (2-byte gathers across 64 feature planes:
// profiles/r01_windowed_ta_counters.txt).  Here a workgroup owns 4 adjacent
// windows of one window row; lanes load IMAGE-ALIGNED 16-byte chunks along
// x (never straddling a row, no shifts, no negative offsets) and scatter the
// pixels into per-window token slots in LDS (slot = 8·ty + tx, the dense
// forward's swizzled [feature][slot] images).  Features stream in chunks (16
// for q, k — Sᵀ accumulates in registers across chunks; 32 for v), so the LDS
// footprint is one chunk.  Out-of-image pixels and padding slots stay zero
// (zero-filled image): the reference's zero padding.
// --------------------------------------------------------------------------
template <class T, int D, int DV>
__global__ __launch_bounds__(256, 2) void win_rows(const T* __restrict__ q, const T* __restrict__ k,
                                                   const T* __restrict__ v, T* __restrict__ out,
                                                   float* __restrict__ lo, float* __restrict__ mo,
                                                   WinDev g, int d, int dv, int batch, int ngx,
                                                   float scale, float scale_log2) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int NWIN = 4, NTH = 256;
    constexpr int FQ = D < 32 ? D : 32, FV = 32;              // feature chunk: q/k, v
    constexpr int KROW = 128, VROW = 144;
    constexpr int QKIMG = FQ * KROW;                           // one window, one tensor, one q/k chunk
    constexpr int VIMG = FV * VROW;
    constexpr int REGION = (2 * NWIN * QKIMG > NWIN * VIMG) ? 2 * NWIN * QKIMG : NWIN * VIMG;
    __shared__ __attribute__((aligned(16))) char smem[REGION];
    auto kswz = [](int f) { return ((f >> 1) & 1) << 1; };

    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int W_ = g.S[0], H_ = g.S[1], P_ = g.P, ws = g.ws, st = g.stride;
    int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int gx = bid % ngx; bid /= ngx;
    const int wy = bid % g.O[1];
    const int b = bid / g.O[1];
    const int wx0 = gx * NWIN;
    const int nwin = min(NWIN, g.O[0] - wx0);
    const int xs = wx0 * st - g.pad;                           // x of window 0, token 0
    const int xe = (wx0 + nwin - 1) * st - g.pad + ws;         // one past the last window's pixels
    const int y0 = wy * st - g.pad;
    const int c_lo = max(xs, 0) >> 3, c_hi = (min(xe, W_) + 7) >> 3;   // image-aligned 8-pixel chunks
    const int ncx = c_hi - c_lo;
    const int ylo = max(y0, 0), yhi = min(y0 + ws, H_);
    const int nrow = max(yhi - ylo, 0);

    // zero the staging region, then scatter nf features (from feature f0) of
    // tensor src into image base + wl·imgbytes with the given row layout
    auto zero_region = [&]() {
        for (int o = tid * 16; o < REGION; o += NTH * 16) *(u32x4*)(smem + o) = u32x4{0u, 0u, 0u, 0u};
    };
    auto stage = [&](const T* src, int C, int f0, int nf, int base, int imgbytes, bool vlayout) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(src + (int64_t)b * C * P_), (short)0, C * P_ * 2, 0x00020000);
        const int items = nf * nrow * ncx;
        for (int it = tid; it < items; it += NTH) {
            const int cx = it % ncx;
            const int rest = it / ncx;
            const int yy = rest % nrow, fl = rest / nrow;
            const int f = f0 + fl, y = ylo + yy, x8 = (c_lo + cx) * 8;
            u32x4 val = u32x4{0u, 0u, 0u, 0u};
            if (f < C) val = __builtin_amdgcn_raw_buffer_load_b128(rs, (f * P_ + y * W_ + x8) * 2, 0, 0);
            const int ty = y - y0;
            // (window, token column) of the chunk's first pixel; consecutive pixels
            // then advance incrementally (tx < 0: left of window 0)
            const int rel = x8 - xs;
            int wl = rel >= 0 ? rel / st : 0;
            int tx = rel >= 0 ? rel - wl * st : rel;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                if (tx >= 0 && tx < ws && wl < nwin) {
                    const unsigned wd = val[e >> 1];
                    const unsigned short px = (unsigned short)((e & 1) ? (wd >> 16) : (wd & 0xFFFFu));
                    const int slot = ty * 8 + tx;
                    const int o = vlayout ? fl * VROW + slot * 2
                                          : fl * KROW + (((slot >> 4) ^ kswz(fl)) * 32) + (slot & 15) * 2;
                    *(unsigned short*)(smem + base + wl * imgbytes + o) = px;
                }
                if (++tx == st) { tx = 0; ++wl; }
            }
        }
    };

    const int g4 = lane >> 4, kh = g4 & 1, qq = (lane & 15) >> 2, pp = lane & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
    f32x16 sa[2][2];                                           // [key block][query block]
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
            for (int x = 0; x < 16; ++x) sa[kb][qb][x] = 0.0f;

    // ---- Sᵀ = K·Qᵀ over feature chunks.  Every chunk writes the same slot
    //      positions (pixel validity does not depend on the feature), so the
    //      padding slots stay zero after one zero-fill per layout. ----
    zero_region();
    __syncthreads();
    for (int f0 = 0; f0 < D; f0 += FQ) {
        stage(q, d, f0, FQ, 0, QKIMG, false);
        stage(k, d, f0, FQ, NWIN * QKIMG, QKIMG, false);
        __syncthreads();
        if (wave < nwin) {
            const char* qimg = smem + wave * QKIMG;
            const char* kimg = smem + NWIN * QKIMG + wave * QKIMG;
#pragma unroll
            for (int s16 = 0; s16 < FQ / 16; ++s16) {          // 16-feature k-steps of the chunk
                F8 kf[2], qf[2];
#pragma unroll
                for (int blk = 0; blk < 2; ++blk) {
                    const int o = (16 * s16 + 8 * h + qq) * KROW + (((blk * 2 + kh) ^ kswz(qq)) * 32);
                    kf[blk] = __builtin_shufflevector(__builtin_bit_cast(F4, ds_read_tr16(kimg + o + 8 * sig)),
                                                      __builtin_bit_cast(F4, ds_read_tr16(kimg + o + 8 * sig + 4 * KROW)), 0, 1, 2, 3, 4, 5, 6, 7);
                    qf[blk] = __builtin_shufflevector(__builtin_bit_cast(F4, ds_read_tr16(qimg + o + 8 * pp)),
                                                      __builtin_bit_cast(F4, ds_read_tr16(qimg + o + 8 * pp + 4 * KROW)), 0, 1, 2, 3, 4, 5, 6, 7);
                }
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int qb = 0; qb < 2; ++qb) sa[kb][qb] = mfma32x32x16(kf[kb], qf[qb], sa[kb][qb]);
            }
        }
        __syncthreads();
    }

    // ---- exact softmax per query (keys: the window's ws x ws real slots) ----
    F8 pf[2][2][2];                                            // [query block][key block][half]
    float mt[2], lt[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int kt = kb * 32 + (x & 3) + 4 * ((x >> 2) & 1) + 8 * h + 16 * (x >> 3);
                if ((kt & 7) >= ws || (kt >> 3) >= ws) sa[kb][qb][x] = kNegInf;
            }
        float pm[4] = {sa[0][qb][0], sa[0][qb][1], sa[0][qb][2], sa[0][qb][3]};
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int x = (kb == 0 ? 4 : 0); x < 16; ++x) pm[x & 3] = vmax(pm[x & 3], sa[kb][qb][x]);
        mt[qb] = swap_halves_max(vmax(vmax(pm[0], pm[1]), vmax(pm[2], pm[3])));
        const float mc = mt[qb] * scale_log2;
        float ps[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const float pr = exp2_fast(fmaf(sa[kb][qb][x], scale_log2, -mc));
                ps[x & 3] += pr;
                pf[qb][kb][x >> 3][x & 7] = (T)pr;
            }
        lt[qb] = swap_halves_sum((ps[0] + ps[1]) + (ps[2] + ps[3]));
    }

    // ---- Oᵀ = Vᵀ·Pᵀ over feature chunks of 32, stored straight to the pixels ----
    const int wx = wx0 + wave;
    const int64_t wid = (int64_t)(wx + g.O[0] * wy) + (int64_t)g.L * b;
    zero_region();                                             // v layout (last barrier of the q/k loop passed)
    __syncthreads();
    for (int c0 = 0; c0 < DV; c0 += FV) {
        stage(v, dv, c0, FV, 0, VIMG, true);
        __syncthreads();
        if (wave < nwin) {
            const char* vimg = smem + wave * VIMG + r * VROW + 16 * h;
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) {
                f32x16 oa;
#pragma unroll
                for (int x = 0; x < 16; ++x) oa[x] = 0.0f;
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2)
                        oa = mfma32x32x16(*(const F8*)(vimg + (kb * 32 + 16 * s2) * 2), pf[qb][kb][s2], oa);
                const int qslot = qb * 32 + r, qtx = qslot & 7, qty = qslot >> 3;
                const int px = wx * st - g.pad + qtx, py = y0 + qty;
                if (qtx < ws && qty < ws && px >= 0 && px < W_ && py >= 0 && py < H_) {
                    const float inv = 1.0f / lt[qb];
                    T* yb = out + (int64_t)b * dv * P_ + (int64_t)py * W_ + px;
#pragma unroll
                    for (int x = 0; x < 16; ++x) {
                        const int cc = c0 + acc_row(x, h);
                        if (cc < dv) yb[(int64_t)cc * P_] = (T)(oa[x] * inv);
                    }
                }
            }
        }
        __syncthreads();
    }
    if (wave < nwin && h == 0) {
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            const int qslot = qb * 32 + r, qtx = qslot & 7, qty = qslot >> 3;
            if (qtx < ws && qty < ws) {
                const int64_t li = qty * ws + qtx + (int64_t)g.T * wid;
                mo[li] = mt[qb] * scale;
                lo[li] = lt[qb];
            }
        }
    }
}

// --------------------------------------------------------------------------
// Row-staged kernel, one window per workgroup (small launches: B = 1 of
// configs[2] has 324 windows, so four windows per workgroup would leave most
// CUs idle).  q, k and v are staged in ONE phase: every thread issues all its
// image-aligned 16-B row loads before it scatters any of them (items decoded
// with fixed strides — 2 chunks per row, 8 rows per feature — so out-of-window
// items read an out-of-range offset, i.e. 0, and are skipped at the scatter),
// so the workgroup pays one HBM round trip instead of one per item.  The 4
// waves split the window: wave w computes query block (w & 1) and the 32-wide
// v feature chunk (w >> 1).
// --------------------------------------------------------------------------
template <class T, int D, int DV>
__global__ __launch_bounds__(256) void win_rows1(const T* __restrict__ q, const T* __restrict__ k,
                                                 const T* __restrict__ v, T* __restrict__ out,
                                                 float* __restrict__ lo, float* __restrict__ mo,
                                                 WinDev g, int d, int dv, float scale, float scale_log2) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int NTH = 256, KROW = 128, VROW = 144;
    constexpr int QIMG = D * KROW, VIMG = DV * VROW, REGION = 2 * QIMG + VIMG;
    constexpr int NBQ = D * 16 / NTH, NBV = DV * 16 / NTH;    // items per thread: feature x 8 rows x 2 chunks
    static_assert(D * 16 % NTH == 0 && DV * 16 % NTH == 0, "item split");
    __shared__ __attribute__((aligned(16))) char smem[REGION];
    auto kswz = [](int f) { return ((f >> 1) & 1) << 1; };

    FA_STAMP(0);
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int W_ = g.S[0], H_ = g.S[1], P_ = g.P, ws = g.ws, st = g.stride;
    const int bid = blockIdx.x;
    const int wx = bid % g.O[0], wy = (bid / g.O[0]) % g.O[1], b = bid / (g.O[0] * g.O[1]);
    const int xs = wx * st - g.pad, y0 = wy * st - g.pad;
    const int c_lo = max(xs, 0) >> 3;
    const int ncx = max(((min(xs + ws, W_) + 7) >> 3) - c_lo, 0);
    const int ylo = max(y0, 0), nrow = max(min(y0 + ws, H_) - ylo, 0);

    // item it -> (feature fl = it >> 4, row yy = (it >> 1) & 7, chunk cx = it & 1)
    auto item_off = [&](int it, int C) {
        const int cx = it & 1, yy = (it >> 1) & 7, fl = it >> 4;
        const bool ok = cx < ncx && yy < nrow && fl < C;
        return ok ? (fl * P_ + (ylo + yy) * W_ + (c_lo + cx) * 8) * 2 : 0x7FFFFFF0;
    };
    const auto qrs = slab_rsrc(q + (int64_t)b * d * P_, (uint32_t)(d * P_ * 2));
    const auto krs = slab_rsrc(k + (int64_t)b * d * P_, (uint32_t)(d * P_ * 2));
    const auto vrs = slab_rsrc(v + (int64_t)b * dv * P_, (uint32_t)(dv * P_ * 2));
    u32x4 rq[NBQ], rk[NBQ], rv[NBV];
#pragma unroll
    for (int j = 0; j < NBQ; ++j) {
        const int o = item_off(tid + NTH * j, d);
        rq[j] = __builtin_amdgcn_raw_buffer_load_b128(qrs, o, 0, 0);
        rk[j] = __builtin_amdgcn_raw_buffer_load_b128(krs, o, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NBV; ++j) rv[j] = __builtin_amdgcn_raw_buffer_load_b128(vrs, item_off(tid + NTH * j, dv), 0, 0);

    for (int o = tid * 16; o < REGION; o += NTH * 16) *(u32x4*)(smem + o) = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();
    FA_STAMP(1);
    auto scatter = [&](const u32x4& val, int it, int C, char* base, bool vlayout) {
        const int cx = it & 1, yy = (it >> 1) & 7, fl = it >> 4;
        if (!(cx < ncx && yy < nrow && fl < C)) return;
        const int ty = ylo + yy - y0;
        int tx = (c_lo + cx) * 8 - xs;
#pragma unroll
        for (int e = 0; e < 8; ++e, ++tx) {
            if (tx >= 0 && tx < ws) {
                const unsigned wd = val[e >> 1];
                const unsigned short px = (unsigned short)((e & 1) ? (wd >> 16) : (wd & 0xFFFFu));
                const int slot = ty * 8 + tx;
                const int o = vlayout ? fl * VROW + slot * 2 : fl * KROW + (((slot >> 4) ^ kswz(fl)) * 32) + (slot & 15) * 2;
                *(unsigned short*)(base + o) = px;
            }
        }
    };
#pragma unroll
    for (int j = 0; j < NBQ; ++j) {
        scatter(rq[j], tid + NTH * j, d, smem, false);
        scatter(rk[j], tid + NTH * j, d, smem + QIMG, false);
    }
#pragma unroll
    for (int j = 0; j < NBV; ++j) scatter(rv[j], tid + NTH * j, dv, smem + 2 * QIMG, true);
    __syncthreads();
    FA_STAMP(2);

    // ---- Sᵀ = K·Qᵀ for this wave's query block ----
    const int qb = wave & 1, vc = wave >> 1;
    const int g4 = lane >> 4, kh = g4 & 1, qq = (lane & 15) >> 2, pp = lane & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
    f32x16 sa[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int x = 0; x < 16; ++x) sa[kb][x] = 0.0f;
#pragma unroll
    for (int s16 = 0; s16 < D / 16; ++s16) {
        const int orow = (16 * s16 + 8 * h + qq) * KROW;
        F8 kf[2];
#pragma unroll
        for (int blk = 0; blk < 2; ++blk) {
            const char* a = smem + QIMG + orow + (((blk * 2 + kh) ^ kswz(qq)) * 32) + 8 * sig;
            kf[blk] = __builtin_shufflevector(__builtin_bit_cast(F4, ds_read_tr16(a)),
                                              __builtin_bit_cast(F4, ds_read_tr16(a + 4 * KROW)), 0, 1, 2, 3, 4, 5, 6, 7);
        }
        const char* a = smem + orow + (((qb * 2 + kh) ^ kswz(qq)) * 32) + 8 * pp;
        const F8 qf = __builtin_shufflevector(__builtin_bit_cast(F4, ds_read_tr16(a)),
                                              __builtin_bit_cast(F4, ds_read_tr16(a + 4 * KROW)), 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) sa[kb] = mfma32x32x16(kf[kb], qf, sa[kb]);
    }

    FA_STAMP(3);
    // ---- exact softmax per query (keys: the window's ws x ws real slots) ----
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int x = 0; x < 16; ++x) {
            const int kt = kb * 32 + (x & 3) + 4 * ((x >> 2) & 1) + 8 * h + 16 * (x >> 3);
            if ((kt & 7) >= ws || (kt >> 3) >= ws) sa[kb][x] = kNegInf;
        }
    const float mt = swap_halves_max(lane_max<2>(sa));
    const float mc = mt * scale_log2;
    float ps[4] = {0.f, 0.f, 0.f, 0.f};
    F8 pf[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int x = 0; x < 16; ++x) {
            const float pr = exp2_fast(fmaf(sa[kb][x], scale_log2, -mc));
            ps[x & 3] += pr;
            pf[kb][x >> 3][x & 7] = (T)pr;
        }
    const float lt = swap_halves_sum((ps[0] + ps[1]) + (ps[2] + ps[3]));

    FA_STAMP(4);
    // ---- Oᵀ = Vᵀ·Pᵀ for this wave's 32-feature chunk, stored straight to the pixels ----
    const int qslot = qb * 32 + r, qtx = qslot & 7, qty = qslot >> 3;
    if (vc < DV / 32) {
        const char* vimg = smem + 2 * QIMG + (vc * 32 + r) * VROW + 16 * h;
        f32x16 oa;
#pragma unroll
        for (int x = 0; x < 16; ++x) oa[x] = 0.0f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) oa = mfma32x32x16(*(const F8*)(vimg + (kb * 32 + 16 * s2) * 2), pf[kb][s2], oa);
        const int px = xs + qtx, py = y0 + qty;
        if (qtx < ws && qty < ws && px >= 0 && px < W_ && py >= 0 && py < H_) {
            const float inv = 1.0f / lt;
            T* yb = out + (int64_t)b * dv * P_ + (int64_t)py * W_ + px;
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int cc = vc * 32 + acc_row(x, h);
                if (cc < dv) yb[(int64_t)cc * P_] = (T)(oa[x] * inv);
            }
        }
    }
    if (vc == 0 && h == 0 && qtx < ws && qty < ws) {
        const int64_t wid = (int64_t)(wx + g.O[0] * wy) + (int64_t)g.L * b;
        const int64_t li = qty * ws + qtx + (int64_t)g.T * wid;
        mo[li] = mt * scale;
        lo[li] = lt;
    }
    FA_STAMP(5);
}

// --------------------------------------------------------------------------
// Row-SHIFT staging, ws <= 7 (the default row-staged kernel for ws <= 7 at
// every launch size; two windows per workgroup, below).  A window row of <= 7 pixels always
// fits in the 8 pixels that start at the dword-aligned pixel
//   a = clamp(xs & ~1, 0, W - 8),
// so every (feature, window row) item is ONE 16-B buffer load, a wave-uniform
// shift by sh = xs - a pixels (dword selects + v_alignbyte), a uniform mask
// (slot < ws, pixel inside the image) and ONE ds_write_b128 into the dense
// kernel's LDS layouts: 6 loads and 6 LDS writes per thread, no zero-fill and
// no 2-byte scatter (the scatter kernel above spent ~30 % of its time there,
// tools/exp/win_stamp.py).  Items cover all 8 slot rows and all D features,
// so padding slots are written as zeros.  Workgroups are dealt to XCDs in
// contiguous window runs (xcd_remap), so horizontally adjacent windows, which
// share cache lines, hit one XCD's L2: configs[2] B=1 12.2 -> 6.8 us.  Two
// windows per workgroup (their loads coalesce, below) took B=32 97 -> 83 us.
// --------------------------------------------------------------------------
__device__ __forceinline__ unsigned pick_dword(const u32x4& in, int idx) {
    unsigned r = 0u;
    r = idx == 0 ? in[0] : r;
    r = idx == 1 ? in[1] : r;
    r = idx == 2 ? in[2] : r;
    r = idx == 3 ? in[3] : r;
    return r;
}
// out pixel t = in pixel (t + sh) (0 outside 0..7), sh in (-8, 8) wave-uniform,
// then AND-ed with the per-slot mask.  Interior windows (ax = xs rounded down to even)
// shift by 0 or 1 pixel: one v_alignbyte per dword (round 5; the runtime dword picks of
// the general case are kept for windows at the image's left and right edges).
__device__ __forceinline__ u32x4 shift_row(const u32x4& in, int sh, const unsigned (&mask)[4]) {
    const int s2 = sh >> 1;              // floor(sh / 2)
    u32x4 o;
    if (s2 == 0) {
        const unsigned ab = (sh & 1) ? 2u : 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = __builtin_amdgcn_alignbyte(j < 3 ? in[j + 1] : 0u, in[j], ab) & mask[j];
    } else if (sh & 1) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            o[j] = __builtin_amdgcn_alignbyte(pick_dword(in, j + s2 + 1), pick_dword(in, j + s2), 2u) & mask[j];
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = pick_dword(in, j + s2) & mask[j];
    }
    return o;
}

// Workgroup barrier that orders LDS only (s_waitcnt lgkmcnt(0); s_barrier):
// outstanding global loads are not waited for.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);   // gfx9 encoding: vmcnt 63, expcnt 7, lgkmcnt 0
    __builtin_amdgcn_s_barrier();
}

// LDS accesses hidden from the compiler (inline asm).  hipcc makes every LDS access
// it can see wait for ALL outstanding LDS-DMA (s_waitcnt vmcnt(0)): it cannot tell
// the DMA's destination buffer from the one being read, so a multi-buffer DMA
// pipeline would drain at every step.  An asm read's result is NOT ready until
// lds_wait(); pass it through lds_fence() after that wait, before any use.
__device__ __forceinline__ uint32_t lds_off(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ s16x4 lds_tr16(const void* p) {
    s16x4 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(lds_off(p)) : "memory");
    return r;
}
__device__ __forceinline__ u32x4 lds_b128(const void* p) {
    u32x4 r;
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(lds_off(p)) : "memory");
    return r;
}
__device__ __forceinline__ u32x2 lds_b64(const void* p) {
    u32x2 r;
    asm volatile("ds_read_b64 %0, %1" : "=v"(r) : "v"(lds_off(p)) : "memory");
    return r;
}
__device__ __forceinline__ float lds_b32(const void* p) {
    float r;
    asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(lds_off(p)) : "memory");
    return r;
}
__device__ __forceinline__ void lds_w16(void* p, unsigned v) {
    asm volatile("ds_write_b16 %0, %1" : : "v"(lds_off(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void lds_w32u(void* p, unsigned v) {
    asm volatile("ds_write_b32 %0, %1" : : "v"(lds_off(p)), "v"(v) : "memory");
}
// Returning agent-scope atomic add, hidden from the compiler's waitcnt model (the
// caller counts it in its vmcnt bookkeeping and fences the result after the wait).
__device__ __forceinline__ unsigned atomic_add_ret(unsigned* p, unsigned v) {
    unsigned r;
    asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(r) : "v"(p), "v"(v) : "memory");
    return r;
}

template <class X>
__device__ __forceinline__ void lds_fence(X& x) { asm volatile("" : "+v"(x)); }

// Per-lane variant of shift_row (windows of one workgroup differ in shift; -8 < sh < 8,
// so the dword shift s2 = floor(sh / 2) is in [-4, 3]): three bit-select levels (1, 2, 4
// dwords) over the zero-extended row, with lane masks, then the odd pixel by
// v_alignbyte with the lane's byte shift.  (Written as selects of array elements, the
// compiler turned the levels into indexed scratch accesses.)
__device__ __forceinline__ u32x4 shift_row_lane(const u32x4& in, int sh, const unsigned (&mask)[4]) {
    const int u = (sh >> 1) + 4;                     // 0 .. 7: e[j] = ext[j + u] = in[j + s2]
    const unsigned m1 = 0u - (unsigned)(u & 1), m2 = 0u - (unsigned)((u >> 1) & 1), m4 = 0u - (unsigned)((u >> 2) & 1);
    auto bfi = [](unsigned m, unsigned x, unsigned y) { return (x & m) | (y & ~m); };
    unsigned ext[13];
#pragma unroll
    for (int i = 0; i < 13; ++i) ext[i] = (i >= 4 && i < 8) ? in[i - 4] : 0u;
    unsigned a1[12], a2[10], e[5];
#pragma unroll
    for (int i = 0; i < 12; ++i) a1[i] = bfi(m1, ext[i + 1], ext[i]);
#pragma unroll
    for (int i = 0; i < 10; ++i) a2[i] = bfi(m2, a1[i + 2], a1[i]);
#pragma unroll
    for (int j = 0; j < 5; ++j) e[j] = bfi(m4, a2[j + 4], a2[j]);
    const unsigned ab = (sh & 1) ? 2u : 0u;
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = __builtin_amdgcn_alignbyte(e[j + 1], e[j], ab) & mask[j];
    return o;
}

// NWIN horizontally adjacent windows per workgroup (4 waves each).  Staging items
// interleave the windows on adjacent lanes, so the NWIN 16-B row loads of one
// (feature, row) — 14 B apart at stride 7 — fall in the same cache line and
// coalesce in the texture path (NWIN = 1: the wave-uniform shift above).
template <class T, int D, int DV, int NWIN>
__global__ __launch_bounds__(256 * NWIN) void win_rows1s(const T* __restrict__ q, const T* __restrict__ k,
                                                         const T* __restrict__ v, T* __restrict__ out,
                                                         float* __restrict__ lo, float* __restrict__ mo,
                                                         WinDev g, int d, int dv, int64_t nwin_total,
                                                         float scale, float scale_log2) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int NTH = 256 * NWIN, KROW = 128, VROW = 144;
    constexpr int QIMG = D * KROW, VIMG = DV * VROW, REGION = 2 * QIMG + VIMG;
    constexpr int NIQ = D * 8 / 256, NIV = DV * 8 / 256;    // items per thread: window x feature x 8 slot rows
    static_assert(D * 8 % 256 == 0 && DV * 8 % 256 == 0, "item split");
    __shared__ __attribute__((aligned(16))) char smem[NWIN * REGION];
    auto kswz = [](int f) { return ((f >> 1) & 1) << 1; };

    FA_STAMP(0);
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int W_ = g.S[0], H_ = g.S[1], P_ = g.P, ws = g.ws, st = g.stride;
    const int64_t wid0 = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * NWIN;
    const int nperimg = g.O[0] * g.O[1];
    struct Win { int wx, wy, b, xs, y0, ax; bool ok; };
    auto win_of = [&](int wl) {
        Win w;
        const int id = (int)wid0 + wl;   // 32-bit: the host keeps L·B < 2^31 on this path
        w.ok = id < (int)nwin_total;
        const int idc = w.ok ? id : 0;
        w.b = idc / nperimg;
        const int rem = idc - w.b * nperimg;
        w.wy = rem / g.O[0];
        w.wx = rem - w.wy * g.O[0];
        w.xs = w.wx * st - g.pad;
        w.y0 = w.wy * st - g.pad;
        w.ax = min(max(w.xs & ~1, 0), W_ - 8);
        return w;
    };

    // item it -> (window it % NWIN, feature f = (it / NWIN) >> 3, slot row yy = (it / NWIN) & 7)
    // descriptors over the workgroup's first image and the next one (a window
    // pair may straddle images); item offsets are relative to image b0
    const int b0 = win_of(0).b;
    const int nimg = min(NWIN == 1 ? 1 : 2, (int)nwin_total / nperimg - b0);
    // every item of a lane belongs to the same window (NTH is a multiple of NWIN)
    const int wl_me = NWIN == 1 ? 0 : (int)(tid % NWIN);
    const Win wme = win_of(wl_me);
    auto item_off = [&](int it, int C) {
        const Win& w = wme;
        const int rest = NWIN == 1 ? it : it / NWIN, yy = rest & 7, f = rest >> 3, y = w.y0 + yy;
        const bool ok = w.ok && yy < ws && y >= 0 && y < H_ && f < C;
        if (FA_WIN_ABL & 2) return 0;
        return ok ? (((w.b - b0) * C + f) * P_ + y * W_ + w.ax) * 2 : 0x7FFFFFF0;
    };
    const auto qrs = slab_rsrc(q + (int64_t)b0 * d * P_, (uint32_t)(nimg * d * P_ * 2));
    const auto krs = slab_rsrc(k + (int64_t)b0 * d * P_, (uint32_t)(nimg * d * P_ * 2));
    const auto vrs = slab_rsrc(v + (int64_t)b0 * dv * P_, (uint32_t)(nimg * dv * P_ * 2));
    u32x4 rq[NIQ], rk[NIQ], rv[NIV];
#pragma unroll
    for (int j = 0; j < NIQ; ++j) {
        const int o = item_off(tid + NTH * j, d);
        rq[j] = __builtin_amdgcn_raw_buffer_load_b128(qrs, o, 0, 0);
        rk[j] = __builtin_amdgcn_raw_buffer_load_b128(krs, o, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NIV; ++j) rv[j] = __builtin_amdgcn_raw_buffer_load_b128(vrs, item_off(tid + NTH * j, dv), 0, 0);

    // staging of one item: shift into slots, mask (slot < ws, pixel inside the image).
    // A lane's window, masks and shift are computed once.  Round 5: when no lane of the wave
    // shifts by 2 pixels or more (every window away from the image's left and right
    // edges: ax = xs rounded down to even, so the shift is 0 or 1), the shift is one
    // v_alignbyte per dword with the lane's byte shift instead of five runtime dword
    // picks (the staging was ~400 VALU, 163 of them v_cndmask, per lane before the barrier).
    unsigned mask_me[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int t0 = 2 * j, t1 = 2 * j + 1;
        const bool v0 = t0 < ws && wme.xs + t0 >= 0 && wme.xs + t0 < W_;
        const bool v1 = t1 < ws && wme.xs + t1 >= 0 && wme.xs + t1 < W_;
        mask_me[j] = (v0 ? 0x0000FFFFu : 0u) | (v1 ? 0xFFFF0000u : 0u);
    }
    const int sh_me = wme.xs - wme.ax;
    const bool near_shift = NWIN > 1 && __builtin_amdgcn_ballot_w64((sh_me >> 1) != 0) == 0;
    const unsigned ab_me = (sh_me & 1) ? 2u : 0u;
    auto stage = [&](auto fast, const u32x4& val, int it, char* img, bool vlayout) {
        const int rest = NWIN == 1 ? it : it / NWIN, yy = rest & 7, f = rest >> 3;
        u32x4 o;
        if constexpr (NWIN == 1) {
            o = shift_row(val, sh_me, mask_me);
        } else if constexpr (decltype(fast)::value) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                o[j] = __builtin_amdgcn_alignbyte(j < 3 ? val[j + 1] : 0u, val[j], ab_me) & mask_me[j];
        } else {
            o = shift_row_lane(val, sh_me, mask_me);
        }
        char* base = smem + wl_me * REGION + (img - smem);
        const int off = vlayout ? f * VROW + yy * 16 : f * KROW + (((yy >> 1) ^ kswz(f)) * 32) + (yy & 1) * 16;
        *(u32x4*)(base + off) = o;
    };
    // V staged before the one barrier too (round 5): its loads were issued with Q's and
    // K's, and staging it after the softmax put a second barrier and the staging on the
    // path to the stores
    auto stage_all = [&](auto fast) {
#pragma unroll
        for (int j = 0; j < NIQ; ++j) {
            stage(fast, rq[j], tid + NTH * j, smem, false);
            stage(fast, rk[j], tid + NTH * j, smem + QIMG, false);
        }
#pragma unroll
        for (int j = 0; j < NIV; ++j) stage(fast, rv[j], tid + NTH * j, smem + 2 * QIMG, true);
    };
    if (near_shift) stage_all(std::true_type{});
    else stage_all(std::false_type{});
    lds_barrier();
    FA_STAMP(2);

    // ---- this wave's window, query block and v chunk ----
    const int wl = wave >> 2;
    const Win w = win_of(wl);
    char* const wsm = smem + wl * REGION;
    const int qb = wave & 1, vc = (wave >> 1) & 1;
    const int g4 = lane >> 4, kh = g4 & 1, qq = (lane & 15) >> 2, pp = lane & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
    f32x16 sa[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int x = 0; x < 16; ++x) sa[kb][x] = 0.0f;
#pragma unroll
    for (int s16 = 0; s16 < D / 16; ++s16) {
        const int orow = (16 * s16 + 8 * h + qq) * KROW;
        F8 kf[2];
#pragma unroll
        for (int blk = 0; blk < 2; ++blk) {
            const char* a = wsm + QIMG + orow + (((blk * 2 + kh) ^ kswz(qq)) * 32) + 8 * sig;
            kf[blk] = __builtin_shufflevector(__builtin_bit_cast(F4, ds_read_tr16(a)),
                                              __builtin_bit_cast(F4, ds_read_tr16(a + 4 * KROW)), 0, 1, 2, 3, 4, 5, 6, 7);
        }
        const char* a = wsm + orow + (((qb * 2 + kh) ^ kswz(qq)) * 32) + 8 * pp;
        const F8 qf = __builtin_shufflevector(__builtin_bit_cast(F4, ds_read_tr16(a)),
                                              __builtin_bit_cast(F4, ds_read_tr16(a + 4 * KROW)), 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) sa[kb] = mfma32x32x16(kf[kb], qf, sa[kb]);
    }
    FA_STAMP(3);

    // ---- exact softmax per query (keys: the window's ws x ws real slots) ----
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int x = 0; x < 16; ++x) {
            const int kt = kb * 32 + (x & 3) + 4 * ((x >> 2) & 1) + 8 * h + 16 * (x >> 3);
            if ((kt & 7) >= ws || (kt >> 3) >= ws) sa[kb][x] = kNegInf;
        }
    const float mt = swap_halves_max(lane_max<2>(sa));
    const float mc = mt * scale_log2;
    float ps[4];
    F8 pf[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int x = 0; x < 16; ++x) {
            const float pr = exp2_fast(fmaf(sa[kb][x], scale_log2, -mc));
            if (kb == 0 && x < 4) ps[x] = pr; else ps[x & 3] += pr;
            pf[kb][x >> 3][x & 7] = (T)pr;
        }
    const float lt = swap_halves_sum((ps[0] + ps[1]) + (ps[2] + ps[3]));
    FA_STAMP(4);

    // ---- Oᵀ = Vᵀ·Pᵀ for this wave's 32-feature chunk, stored straight to the pixels ----
    const int qslot = qb * 32 + r, qtx = qslot & 7, qty = qslot >> 3;
#pragma unroll
    for (int cv = vc; cv < DV / 32 && w.ok; cv += 2) {   // DV = 128: chunks vc and vc + 2
        const char* vimg = wsm + 2 * QIMG + (cv * 32 + r) * VROW + 16 * h;
        f32x16 oa;
#pragma unroll
        for (int x = 0; x < 16; ++x) oa[x] = 0.0f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) oa = mfma32x32x16(*(const F8*)(vimg + (kb * 32 + 16 * s2) * 2), pf[kb][s2], oa);
        const int px = w.xs + qtx, py = w.y0 + qty;
        if (qtx < ws && qty < ws && px >= 0 && px < W_ && py >= 0 && py < H_) {
            const float inv = 1.0f / lt;
            T* yb = out + (int64_t)w.b * dv * P_ + (int64_t)py * W_ + px;
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int cc = cv * 32 + acc_row(x, h);
                if (cc < dv && (!(FA_WIN_ABL & 1) || oa[x] == 1234.5f)) yb[(int64_t)cc * P_] = (T)(oa[x] * inv);
            }
        }
    }
    if (vc == 0 && h == 0 && qtx < ws && qty < ws && w.ok) {
        const int64_t wid = (int64_t)(w.wx + g.O[0] * w.wy) + (int64_t)g.L * w.b;
        const int64_t li = qty * ws + qtx + (int64_t)g.T * wid;
        mo[li] = mt * scale;
        lo[li] = lt;
    }
    FA_STAMP(5);
}

// --------------------------------------------------------------------------
// Strip kernel: NS = 8 horizontally adjacent windows of one window row per
// workgroup, one window per wave (bf16/f16, 2-D, stride == ws <= 7, d, dv <= 64,
// width % 8 == 0, q, k, v, y 16-B aligned; the default for large launches).
//
// Why: the per-window kernels move q, k, v and y in 14-B window-row segments, so
// every load / store instruction touches ~64 cache lines that ~9 windows of other
// workgroups share: ~14 M L2 requests of ~20 B per configs[2] B = 32 call
// (r02_windowed_fwd_pmc.txt), which sets their pace, not HBM.  Here the eight
// windows' rows sit side by side in every DMA instruction (8 lanes x 16 B per
// cache line) and y leaves as whole 16-B chunks of the strip's 56 contiguous
// pixels.  The first strip holds k0 <= 8 windows, k0 chosen so that every strip
// boundary falls on a 16-B chunk boundary (k0 * ws = pad mod 8, solvable for odd
// ws): then no chunk is shared with a neighbour strip.  When no k0 aligns them
// (even ws), the two strip ends are 2-B stores.
//
// Channels are streamed so the eight windows fit in LDS:
//   * two 32-KB buffers (64 KB: two workgroups per CU) take the image loads in
//     turn, each issued as soon as its buffer is free: Q / K chunks of 16 features
//     ([16 f][8 slot rows][8 windows] x 16 B, 16 KB each), then the two 32-feature
//     V chunks ([32 f][8][8] x 16 B), which land under the last QKᵀ steps;
//     Sᵀ = K·Qᵀ accumulates over the chunks (one 16-deep MFMA step per chunk,
//     64 x 64 slots per window, 2 x 2 blocks);
//   * y: per V chunk, each wave writes its window's normalised O into a strip
//     image [32 f][8 rows][64 px] over that V chunk, then the workgroup stores it
//     row by row.
// Slots are ROTATED: slot (yy, sx) of window w holds pixel
// (ax_w + sx, y0 + yy), ax_w = clamp(xs_w & ~1, 0, W - 8); padding columns enter
// the softmax analytically (npad zero keys), padding rows load as zeros.
// LDS-DMA writes lane-linearly, so the swizzles are applied through each lane's
// choice of (window, slot row):
//   Q / K: window position w ^ (f & 7) ^ ((c >> 1) & 1) << 2  (ds_read_b64_tr_b16: f & 4 is fixed per
//          instruction, so this is the conflict-free (f & 3, c) pattern; the 16-B row reads of the
//          strip backward's register stash, 16 features at a time, then meet 2-way conflicts, not 4);
//   V    : slot-row position c ^ ((f >> 3) & 1), window position w ^ (f & 7)  (ds_read_b128, conflict-free).
// --------------------------------------------------------------------------
constexpr int kStripW = 8;                          // windows per strip workgroup
// Strip image [f][8 rows][64 px] (1 KB per feature): byte offset of pixel px.  The
// 16-B chunk index is XORed with (row & 3, f >> 2).  A 2-B write instruction of a
// wave covers, per 32-lane group, 4 slot rows x one window's 8 consecutive pixels of
// one feature; writes bank on 32 dwords (MI355X_MICROARCH §LDS), so the 128-B rows
// all start on bank 0 and only the XOR separates them: with row & 3 the 4 rows take
// 4 different 16-B chunks, and when a window's 8 pixels straddle two chunks (c, c + 1)
// the XOR swaps them so the rows' dwords stay complementary — conflict-free.  (Round 3
// used row >> 1: rows 2k and 2k + 1 met on the same banks, ~1.9 conflict cycles per
// write, profiles/r04_win_bwd_strip_lds_conflicts.txt.)  The 16-B chunk reads of the
// stores (ds_read_b128, 16-lane groups, 64 banks) stay conflict-free: an XOR below 4
// keeps each chunk in its half of the row.
typedef float f32x2 __attribute__((ext_vector_type(2)));
// two fp32 -> a packed pair of T (v_cvt_pk_*), and back
template <class T>
__device__ __forceinline__ unsigned pk2(f32x2 v) {
    typedef T T2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, T2));
}
template <class T>
__device__ __forceinline__ f32x2 unpk2(unsigned u) {
    typedef T T2 __attribute__((ext_vector_type(2)));
    return __builtin_convertvector(__builtin_bit_cast(T2, u), f32x2);
}
__device__ __forceinline__ int simg_swz(int f, int row) { return (row & 3) | (((f >> 2) & 1) << 2); }
__device__ __forceinline__ int simg_pos(int f, int row, int px) {
    return f * 1024 + row * 128 + (((px >> 3) ^ simg_swz(f, row)) << 4) + (px & 7) * 2;
}
__device__ __forceinline__ int sqk_swz(int f, int c) { return (f & 7) ^ (((c >> 1) & 1) << 2); }
__device__ __forceinline__ int sqk_pos(int f, int c, int w) {   // byte offset in a Q / K chunk image
    return f * 1024 + c * 128 + ((w ^ sqk_swz(f, c)) << 4);
}
__device__ __forceinline__ int sv_pos(int f, int c, int w) {    // byte offset in a V chunk image
    return f * 1024 + ((c ^ ((f >> 3) & 1)) << 7) + ((w ^ (f & 7)) << 4);
}

template <class T, int D, int DV>
__global__ __launch_bounds__(512, 2) void win_strip(const T* __restrict__ q, const T* __restrict__ k,
                                                    const T* __restrict__ v, T* __restrict__ out,
                                                    float* __restrict__ lo, float* __restrict__ mo, WinDev g, int d,
                                                    int dv, int nsx, int k0, int nwg, float scale, float scale_log2) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    static_assert(D % 16 == 0 && D <= 64 && DV % 32 == 0 && DV <= 64, "head dims");
    constexpr int NQC = D / 16, NVC = DV / 32;       // Q/K chunks of 16 features, V chunks of 32
    constexpr int NLD = NQC + NVC;                   // image loads, alternating between the two buffers
    constexpr int BUF = 32768;
    // two separate LDS objects (not one array): the compiler's LDS-DMA wait tracking tells
    // them apart, so a read of one buffer does not wait for the DMA into the other
    __shared__ __attribute__((aligned(16))) char sbuf0[BUF], sbuf1[BUF];   // 64 KB: two workgroups per CU
    auto bufp = [&](int i) __attribute__((always_inline)) { return (i & 1) ? sbuf1 : sbuf0; };

    FA_STAMP(0);
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int W_ = g.S[0], H_ = g.S[1], P_ = g.P, ws = g.ws, st = g.stride, nwx = g.O[0];
    const int lid = xcd_remap(blockIdx.x, nwg);
    const int sxi = lid % nsx, t0 = lid / nsx, wy = t0 % g.O[1], b = t0 / g.O[1];
    const int wx0 = sxi == 0 ? 0 : k0 + (sxi - 1) * kStripW, y0 = wy * st - g.pad;
    const int nvalid = min(sxi == 0 ? k0 : kStripW, nwx - wx0);
    auto ax_of = [&](int w) { return min(max(((wx0 + w) * st - g.pad) & ~1, 0), W_ - 8); };
    const auto qrs = slab_rsrc(q + (int64_t)b * d * P_, (uint32_t)(d * P_ * 2));
    const auto krs = slab_rsrc(k + (int64_t)b * d * P_, (uint32_t)(d * P_ * 2));
    const auto vrs = slab_rsrc(v + (int64_t)b * dv * P_, (uint32_t)(dv * P_ * 2));

    // one DMA instruction = one feature row f of an image: lane -> (slot row, window).
    // (buffer descriptors are passed, not captured: a lambda capturing one made
    // hipcc's host pass drop the kernel's launch stub, with no diagnostic)
    auto dma_qk = [&](__amdgpu_buffer_rsrc_t rs, char* img, int fl, int fg) {
        const int pc = lane >> 3, pw = lane & 7;
        const int w = pw ^ sqk_swz(fl, pc), y = y0 + pc;
        const bool ok = w < nvalid && pc < ws && y >= 0 && y < H_ && fg < d;
        const int off = ok ? (fg * P_ + y * W_ + ax_of(w)) * 2 : 0x7FFFFFF0;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(img + fl * 1024), 16,
                                                 off, 0, 0, 0);
    };
    auto dma_v = [&](__amdgpu_buffer_rsrc_t rs, char* img, int fl, int fg) {
        const int c = (lane >> 3) ^ ((fl >> 3) & 1), w = (lane & 7) ^ (fl & 7), y = y0 + c;
        const bool ok = w < nvalid && c < ws && y >= 0 && y < H_ && fg < dv;
        const int off = ok ? (fg * P_ + y * W_ + ax_of(w)) * 2 : 0x7FFFFFF0;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(img + fl * 1024), 16,
                                                 off, 0, 0, 0);
    };
    // image load i (QK chunk i, then V chunk i - NQC) into buffer i & 1: 32 DMA
    // instructions (one feature row each), 4 per wave
    auto issue = [&](__amdgpu_buffer_rsrc_t qr, __amdgpu_buffer_rsrc_t kr, __amdgpu_buffer_rsrc_t vr, int i) {
        char* buf = bufp(i);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int rr = j * 8 + wave;                  // 0..31
            if (i < NQC) {
                if (rr < 16) dma_qk(qr, buf, rr, i * 16 + rr);
                else dma_qk(kr, buf + 16384, rr - 16, i * 16 + rr - 16);
            } else {
                dma_v(vr, buf, rr, (i - NQC) * 32 + rr);
            }
        }
    };
    issue(qrs, krs, vrs, 0);
    issue(qrs, krs, vrs, 1);

    // ---- this wave's window ----
    const int wl = wave;
    const bool wok = wl < nvalid;
    const int wx = wx0 + wl, xs = wx * st - g.pad, ax = ax_of(wl);
    const int c0 = xs - ax, c1 = c0 + ws;
    const int ncols = min(c1, 8) - max(c0, 0);
    const float npad = (float)((ws - ncols) * ws);       // padding-column tokens (zero keys)
    const int g4 = lane >> 4, kh = g4 & 1, qq = (lane & 15) >> 2, pp = lane & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;

    f32x16 sa[2][2];                                     // [key block][query block]
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
            for (int x = 0; x < 16; ++x) sa[kb][qb][x] = 0.0f;

    // Load cc is consumed at step cc; load cc + 1 is always the one issued after it,
    // so this wave waits with 4 DMA instructions in flight, then an LDS-only barrier
    // (a __syncthreads fence would drain those too) makes every wave's part visible.
#pragma unroll
    for (int cc = 0; cc < NQC; ++cc) {
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        lds_barrier();
        if (cc == 0) FA_STAMP(1);
        const char* buf = bufp(cc);
        // tr-read rows 8h + qq (+4): chunk-local features; slot rows 4blk + 2kh + (sig >> 1) / qb*4 + 2kh + (pp >> 1)
        // (asm reads: the next buffer's DMA stays in flight)
        s16x4 rk[2][2], rq[2][2];
#pragma unroll
        for (int blk = 0; blk < 2; ++blk) {
            const char* a = buf + 16384 + sqk_pos(8 * h + qq, 4 * blk + 2 * kh + (sig >> 1), wl) + (sig & 1) * 8;
            rk[blk][0] = lds_tr16(a);
            rk[blk][1] = lds_tr16(buf + 16384 + sqk_pos(8 * h + qq + 4, 4 * blk + 2 * kh + (sig >> 1), wl) + (sig & 1) * 8);
            const char* aq = buf + sqk_pos(8 * h + qq, 4 * blk + 2 * kh + (pp >> 1), wl) + (pp & 1) * 8;
            rq[blk][0] = lds_tr16(aq);
            rq[blk][1] = lds_tr16(buf + sqk_pos(8 * h + qq + 4, 4 * blk + 2 * kh + (pp >> 1), wl) + (pp & 1) * 8);
        }
        lds_wait();
        F8 kf[2], qf[2];
#pragma unroll
        for (int blk = 0; blk < 2; ++blk) {
#pragma unroll
            for (int i = 0; i < 2; ++i) { lds_fence(rk[blk][i]); lds_fence(rq[blk][i]); }
            kf[blk] = __builtin_shufflevector(__builtin_bit_cast(F4, rk[blk][0]), __builtin_bit_cast(F4, rk[blk][1]),
                                              0, 1, 2, 3, 4, 5, 6, 7);
            qf[blk] = __builtin_shufflevector(__builtin_bit_cast(F4, rq[blk][0]), __builtin_bit_cast(F4, rq[blk][1]),
                                              0, 1, 2, 3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) sa[kb][qb] = mfma32x32x16(kf[kb], qf[qb], sa[kb][qb]);
        if (cc + 2 < NLD) {
            lds_barrier();                                // every wave is done with this buffer
            issue(qrs, krs, vrs, cc + 2);
        }
    }

    FA_STAMP(2);
    // ---- exact softmax per query over the window's real keys (+ npad zero keys) ----
    F8 pf[2][2][2];                                      // [query block][key block][16-key half]
    float mt[2], lt[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int kt = kb * 32 + (x & 3) + 4 * ((x >> 2) & 1) + 8 * h + 16 * (x >> 3);
                const int sx = kt & 7;
                if ((kt >> 3) >= ws || sx < c0 || sx >= c1) sa[kb][qb][x] = kNegInf;
            }
        f32x16 two[2] = {sa[0][qb], sa[1][qb]};
        float m = swap_halves_max(lane_max<2>(two));
        if (npad > 0.0f) m = vmax(m, 0.0f);
        const float mc = m * scale_log2;
        float ps[4];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const float pr = exp2_fast(fmaf(sa[kb][qb][x], scale_log2, -mc));
                if (kb == 0 && x < 4) ps[x] = pr; else ps[x & 3] += pr;
                pf[qb][kb][x >> 3][x & 7] = (T)pr;
            }
        float l = swap_halves_sum((ps[0] + ps[1]) + (ps[2] + ps[3]));
        if (npad > 0.0f) l = fmaf(npad, exp2_fast(-mc), l);
        mt[qb] = m;
        lt[qb] = l;
    }
    // l, m (window layout) and the padding-column query tokens
    if (wok) {
        const int64_t wbase = (int64_t)g.T * ((int64_t)(wx + nwx * wy) + (int64_t)g.L * b);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            const int qs = qb * 32 + r, qtx = qs & 7, qty = qs >> 3;
            if (h == 0 && qtx >= c0 && qtx < c1 && qty < ws) {
                const int64_t li = wbase + qty * ws + (qtx - c0);
                mo[li] = mt[qb] * scale;
                lo[li] = lt[qb];
            }
        }
        if (lane < g.T) {                                 // padding-column query tokens (q = 0): every score is 0
            const int px = xs + lane % ws;
            if (px < 0 || px >= W_) {
                mo[wbase + lane] = 0.0f;
                lo[wbase + lane] = (float)g.T;
            }
        }
    }
    // this wave's V DMA (and the l, m stores).  The builtin, not asm: hipcc then knows no
    // LDS-DMA is pending, and adds no vmcnt(0) of its own before the epilogue's LDS
    // accesses (which made chunk 1's image reads wait for chunk 0's y stores).
    __builtin_amdgcn_s_waitcnt(0x0F70);
    lds_barrier();                                       // every wave's V landed
    FA_STAMP(3);

    // ---- per 32-feature chunk: Oᵀ = Vᵀ·Pᵀ, then (over the V image) the strip image
    //      [32 f][8 rows][64 px] of normalised O, then 16-B stores of the strip's pixels ----
    const int xs0 = wx0 * st - g.pad, X0 = xs0 & ~7;     // strip start, its 16-B aligned base
    const int xlo = max(xs0, 0), xhi = min(xs0 + nvalid * ws, W_);
    const auto ors = slab_rsrc(out + (int64_t)b * dv * P_, (uint32_t)(dv * P_ * 2));
    unsigned vm[4];                                      // key-slot mask of a V fragment (one slot row)
#pragma unroll
    for (int j = 0; j < 4; ++j)
        vm[j] = ((2 * j >= c0 && 2 * j < c1) ? 0x0000FFFFu : 0u) | ((2 * j + 1 >= c0 && 2 * j + 1 < c1) ? 0xFFFF0000u : 0u);
#pragma unroll
    for (int vc = 0; vc < NVC; ++vc) {
        char* img = bufp(NQC + vc);
        f32x16 oa[2];
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
            for (int x = 0; x < 16; ++x) oa[qb][x] = 0.0f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                u32x4 vr = *(const u32x4*)(img + sv_pos(r, kb * 4 + s2 * 2 + h, wl));
#pragma unroll
                for (int j = 0; j < 4; ++j) vr[j] &= vm[j];
#pragma unroll
                for (int qb = 0; qb < 2; ++qb) oa[qb] = mfma32x32x16(__builtin_bit_cast(F8, vr), pf[qb][kb][s2], oa[qb]);
            }
        lds_barrier();                                   // every wave has read this V chunk
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            const int qs = qb * 32 + r, qtx = qs & 7, qty = qs >> 3;
            const float inv = 1.0f / lt[qb];
            if (wok && qtx >= c0 && qtx < c1 && qty < ws && !(FA_WIN_ABL & 4)) {
                const int px = ax + qtx - X0;
#pragma unroll
                for (int x = 0; x < 16; ++x)
                    *(T*)(img + simg_pos(acc_row(x, h), qty, px)) = (T)(oa[qb][x] * inv);
            }
        }
        lds_barrier();
        constexpr int NU = 32 * 8 * 8;                   // (feature, row, 16-B chunk) units: a wave covers
#pragma unroll                                           // 8 rows x 8 chunks of one feature
        for (int it = 0; it < NU / 512; ++it) {
            const int u = it * 512 + tid, f = u >> 6, row = (u >> 3) & 7, j = u & 7;
            const int y = y0 + row, fg = vc * 32 + f, x0 = X0 + 8 * j;
            if (row >= ws || y < 0 || y >= H_ || fg >= dv || x0 + 8 <= xlo || x0 >= xhi || (FA_WIN_ABL & 8)) continue;
            const int go = ((fg * P_ + y * W_ + x0) * 2);
            const char* src = img + f * 1024 + row * 128 + ((j ^ simg_swz(f, row)) << 4);
            if (x0 >= xlo && x0 + 8 <= xhi) {
                __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4*)src, ors, go, 0, 0);
            } else if (!(FA_WIN_ABL & 16)) {             // a chunk shared with the neighbour strip
                for (int e = 0; e < 8; ++e)
                    if (x0 + e >= xlo && x0 + e < xhi)
                        __builtin_amdgcn_raw_buffer_store_b16(*(const unsigned short*)(src + 2 * e), ors, go + 2 * e, 0, 0);
            }
        }
        if (vc == 0) FA_STAMP(4);
    }
    FA_STAMP(5);
}

// --------------------------------------------------------------------------
// Fused windowed BACKWARD, one window per workgroup (bf16/f16, 2-D, stride >= ws,
// ws <= 7, d, dv <= 64): the exact chain rule of windowed_fa for non-overlapping
// windows, where every covered pixel belongs to exactly one window, so
// dyw = window(dy ./ count) is dy itself and the fold is a direct store.
// Replaces, for these shapes, the composed gather -> dense backward -> fold
// path (T = 49 tokens is not a multiple of 8, so that path runs the SIMT
// backward: 20 ms at B = 32).
//
//   staging  : q, k, v, dy rows by the row-shift loads of the forward kernel into
//              [feature][slot] images (128-B swizzled rows).  y is not read (round 5:
//              a fifth of the loads, on CUs that run two windows at B = 1).
//   phase 1  : wave (qb, kb) computes the 32x32 blocks S = Q Kᵀ and dP = dO Vᵀ
//              (queries on accumulator rows, keys on lanes) with −lse/τ as S's
//              initial accumulator, P = exp2(c·S'), and D = rowsum(P ∘ dP) (= rowsum
//              (dy ∘ y)): each wave's 32-key partial by DPP / permlane16 sums within
//              its lane halves, the two key halves' partials added through LDS; then
//              dS = P ∘ (dP − D), and P, dS (bf16) go into [key][query] images (144-B rows).
//   phase 2  : 12 blocks over the 4 waves: dVᵀ = dOᵀ P, dKᵀ = τ Qᵀ dS (row
//              reads), dQᵀ = τ Kᵀ dSᵀ (dSᵀ by transposed reads of the [key][query]
//              image); each lane stores one slot's features straight to its pixel.
// Padding slots (tx or ty >= ws): keys masked (P = dS = 0), queries have lse = +inf.
// --------------------------------------------------------------------------
template <class T, int D, int DV, int NWIN>
__global__ __launch_bounds__(256 * NWIN) void win_bwd_rows(const T* __restrict__ q, const T* __restrict__ k,
                                                    const T* __restrict__ v, const T* __restrict__ y,
                                                    const T* __restrict__ dy, const float* __restrict__ lw,
                                                    const float* __restrict__ mw, T* __restrict__ dq,
                                                    T* __restrict__ dk, T* __restrict__ dvo, WinDev g, int d,
                                                    int dv, int nwin_total, float scale, float scale_log2) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int NTH = 256 * NWIN, KROW = 128, PROW = 144;
    constexpr int QIMG = D * KROW, VIMG = DV * KROW, PIMG = 64 * PROW;
    constexpr int OQ = 0, OK_ = QIMG, OV = 2 * QIMG, ODO = 2 * QIMG + VIMG, OP = 2 * QIMG + 2 * VIMG,
                  ODS = OP + PIMG, OLSE = ODS + PIMG, OD = OLSE + 256, REGION = OD + 4 * 256;
    constexpr int NIQ = D * 8 / 256, NIV = DV * 8 / 256;    // items per thread: window x feature x 8 slot rows
    static_assert(D * 8 % 256 == 0 && DV * 8 % 256 == 0, "item split");
    __shared__ __attribute__((aligned(16))) char smem[NWIN * REGION];
    auto kswz = [](int f) { return ((f >> 1) & 1) << 1; };

    FA_STAMP(0);
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int W_ = g.S[0], H_ = g.S[1], P_ = g.P, ws = g.ws, st = g.stride;
    // NWIN horizontally adjacent windows (xcd_remap: contiguous runs per XCD), 4 waves each
    const int nperimg = g.O[0] * g.O[1];
    struct Win { int wx, wy, b, xs, y0, ax; bool ok; };
    auto win_of = [&](int wl) {
        Win w;
        const int id = xcd_remap(blockIdx.x, gridDim.x) * NWIN + wl;   // 32-bit: the host keeps L·B < 2^31
        w.ok = id < nwin_total;
        const int idc = w.ok ? id : 0;
        w.b = idc / nperimg;
        const int rem = idc - w.b * nperimg;
        w.wy = rem / g.O[0];
        w.wx = rem - w.wy * g.O[0];
        w.xs = w.wx * st - g.pad;
        w.y0 = w.wy * st - g.pad;
        w.ax = min(max(w.xs & ~1, 0), W_ - 8);
        return w;
    };
    // staging item it -> (window it % NWIN, feature (it / NWIN) >> 3, slot row (it / NWIN) & 7): the
    // NWIN windows' loads of one (feature, row) sit on adjacent lanes, 2·ws bytes apart, and share
    // their cache lines; every item of a lane belongs to window tid % NWIN (NTH % NWIN == 0).
    // Descriptors span the first window's image and the next (a pair may straddle images).
    const int b0 = win_of(0).b;
    const int nimg = min(NWIN == 1 ? 1 : 2, nwin_total / nperimg - b0);
    const int wl_me = NWIN == 1 ? 0 : (int)(tid % NWIN);
    const Win wme = win_of(wl_me);
    auto item_off = [&](int it, int C) {
        const int rest = NWIN == 1 ? it : it / NWIN, yy = rest & 7, f = rest >> 3, yr = wme.y0 + yy;
        const bool ok = wme.ok && yy < ws && yr >= 0 && yr < H_ && f < C;
        return ok ? (((wme.b - b0) * C + f) * P_ + yr * W_ + wme.ax) * 2 : 0x7FFFFFF0;
    };
    const auto qrs = slab_rsrc(q + (int64_t)b0 * d * P_, (uint32_t)(nimg * d * P_ * 2));
    const auto krs = slab_rsrc(k + (int64_t)b0 * d * P_, (uint32_t)(nimg * d * P_ * 2));
    const auto vrs = slab_rsrc(v + (int64_t)b0 * dv * P_, (uint32_t)(nimg * dv * P_ * 2));
    (void)y;
    const auto drs = slab_rsrc(dy + (int64_t)b0 * dv * P_, (uint32_t)(nimg * dv * P_ * 2));
    u32x4 rq[NIQ], rk[NIQ], rv[NIV], rd[NIV];
#pragma unroll
    for (int j = 0; j < NIQ; ++j) {
        const int o = item_off(tid + NTH * j, d);
        rq[j] = __builtin_amdgcn_raw_buffer_load_b128(qrs, o, 0, 0);
        rk[j] = __builtin_amdgcn_raw_buffer_load_b128(krs, o, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NIV; ++j) {
        const int o = item_off(tid + NTH * j, dv);
        rv[j] = __builtin_amdgcn_raw_buffer_load_b128(vrs, o, 0, 0);
        rd[j] = __builtin_amdgcn_raw_buffer_load_b128(drs, o, 0, 0);
    }
    // per-slot constant −lse/τ of window tid >> 6 (+inf lse outside the window)
    if (tid < 64 * NWIN) {
        const int wl = tid >> 6, tx = tid & 7, ty = (tid >> 3) & 7;
        const Win w = win_of(wl);
        float nl = kNegInf;
        if (w.ok && tx < ws && ty < ws) {
            const int64_t wid = (int64_t)(w.wx + g.O[0] * w.wy) + (int64_t)g.L * w.b;
            const int64_t li = ty * ws + tx + (int64_t)g.T * wid;
            nl = -(mw[li] + __logf(lw[li])) / scale;
        }
        ((float*)(smem + wl * REGION + OLSE))[tid & 63] = nl;
    }
    unsigned mask[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int t0 = 2 * j, t1 = 2 * j + 1;
        const bool v0 = t0 < ws && wme.xs + t0 >= 0 && wme.xs + t0 < W_;
        const bool v1 = t1 < ws && wme.xs + t1 >= 0 && wme.xs + t1 < W_;
        mask[j] = (v0 ? 0x0000FFFFu : 0u) | (v1 ? 0xFFFF0000u : 0u);
    }
    const int sh_me = wme.xs - wme.ax;
    // NWIN > 1: lanes of a wave shift by different amounts; away from the image's left and
    // right edges every shift is 0 or 1 pixel (one v_alignbyte per dword), as in win_rows1s
    const bool near_shift = NWIN > 1 && __builtin_amdgcn_ballot_w64((sh_me >> 1) != 0) == 0;
    const unsigned ab_me = (sh_me & 1) ? 2u : 0u;
    char* const sme = smem + wl_me * REGION;
    auto koff = [&](int it) {
        const int rest = NWIN == 1 ? it : it / NWIN, yy = rest & 7, f = rest >> 3;
        return f * KROW + (((yy >> 1) ^ kswz(f)) * 32) + (yy & 1) * 16;
    };
    auto stage_all = [&](auto fast) {
        auto shifted = [&](const u32x4& val) {
            u32x4 o;
            if constexpr (NWIN == 1) {
                o = shift_row(val, sh_me, mask);
            } else if constexpr (decltype(fast)::value) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    o[j] = __builtin_amdgcn_alignbyte(j < 3 ? val[j + 1] : 0u, val[j], ab_me) & mask[j];
            } else {
                o = shift_row_lane(val, sh_me, mask);
            }
            return o;
        };
#pragma unroll
        for (int j = 0; j < NIQ; ++j) {
            const int o = koff(tid + NTH * j);
            *(u32x4*)(sme + OQ + o) = shifted(rq[j]);
            *(u32x4*)(sme + OK_ + o) = shifted(rk[j]);
        }
        FA_STAMP(1);
#pragma unroll
        for (int j = 0; j < NIV; ++j) {
            const int o = koff(tid + NTH * j);
            *(u32x4*)(sme + OV + o) = shifted(rv[j]);
            *(u32x4*)(sme + ODO + o) = shifted(rd[j]);
        }
    };
    if (near_shift) stage_all(std::true_type{});
    else stage_all(std::false_type{});
    __syncthreads();
    FA_STAMP(2);

    // ---- this wave's window ----
    const Win w = win_of(wave >> 2);
    char* const wsm = smem + (wave >> 2) * REGION;
    const int b = w.b, xs = w.xs, y0 = w.y0;
    float* const lse_s = (float*)(wsm + OLSE);   // −lse/τ per query slot (raw score units)
    float* const dsum = (float*)(wsm + OD);      // D per query slot: one partial per key half [2][64]

    // ---- phase 1: S and dP blocks (qb, kb) of this wave ----
    const int qb = wave & 1, kb = (wave >> 1) & 1;
    const int g4 = lane >> 4, kh = g4 & 1, qq = (lane & 15) >> 2, pp = lane & 3;
    // tr-read of a [feature][slot] image: 32 slots of block sb, features 16 s + 8 h .. + 7
    auto frag_tr = [&](int img, int sb, int s16) {
        const int orow = (16 * s16 + 8 * h + qq) * KROW;
        const char* a = wsm + img + orow + (((sb * 2 + kh) ^ kswz(qq)) * 32) + 8 * pp;
        return __builtin_shufflevector(__builtin_bit_cast(F4, ds_read_tr16(a)),
                                       __builtin_bit_cast(F4, ds_read_tr16(a + 4 * KROW)), 0, 1, 2, 3, 4, 5, 6, 7);
    };
    f32x16 sa, pa;
#pragma unroll
    for (int x4 = 0; x4 < 4; ++x4) {
        const f32x4 l4 = *(const f32x4*)(lse_s + qb * 32 + acc_row(4 * x4, h));
#pragma unroll
        for (int e = 0; e < 4; ++e) { sa[4 * x4 + e] = l4[e]; pa[4 * x4 + e] = 0.0f; }
    }
#pragma unroll
    for (int s16 = 0; s16 < D / 16; ++s16) sa = mfma32x32x16(frag_tr(OQ, qb, s16), frag_tr(OK_, kb, s16), sa);
#pragma unroll
    for (int s16 = 0; s16 < DV / 16; ++s16) pa = mfma32x32x16(frag_tr(ODO, qb, s16), frag_tr(OV, kb, s16), pa);
    const int kslot = kb * 32 + r;
    const bool kvalid = (kslot & 7) < ws && (kslot >> 3) < ws;
    // P (fp32 for dS, bf16 into the [key][query] image, 4 consecutive queries per 8-byte
    // write) and this wave's 32-key partial of D = rowsum(P ∘ dP) for each of its queries
    float pr[16];
#pragma unroll
    for (int x4 = 0; x4 < 4; ++x4) {
        typename Frag8<T>::half p4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            pr[4 * x4 + e] = kvalid ? exp2_fast(sa[4 * x4 + e] * scale_log2) : 0.0f;
            p4[e] = (T)pr[4 * x4 + e];
        }
        *(typename Frag8<T>::half*)(wsm + OP + kslot * PROW + (qb * 32 + acc_row(4 * x4, h)) * 2) = p4;
    }
#pragma unroll
    for (int x = 0; x < 16; ++x) {
        float v = pr[x] * pa[x];   // keys on lanes: sum over the 32 lanes of this half (h)
        v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
        v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
        v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
        v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
        auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        v = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
        if (r == 0) dsum[kb * 64 + qb * 32 + acc_row(x, h)] = v;
    }
    lds_barrier();
    // dS = P ∘ (dP − D), D = the two key halves' partials
#pragma unroll
    for (int x4 = 0; x4 < 4; ++x4) {
        const int qrow = qb * 32 + acc_row(4 * x4, h);
        const f32x4 d4 = *(const f32x4*)(dsum + qrow) + *(const f32x4*)(dsum + 64 + qrow);
        typename Frag8<T>::half s4;
#pragma unroll
        for (int e = 0; e < 4; ++e) s4[e] = (T)(pr[4 * x4 + e] * (pa[4 * x4 + e] - d4[e]));
        *(typename Frag8<T>::half*)(wsm + ODS + kslot * PROW + qrow * 2) = s4;
    }
    lds_barrier();
    FA_STAMP(3);

    // ---- phase 2: dVᵀ, dKᵀ, dQᵀ blocks ----
    // row read: 8 consecutive slots 16 s + 8 h of feature row f of a [feature][slot] image
    auto frag_row = [&](int img, int f, int s16) {
        return *(const F8*)(wsm + img + f * KROW + ((s16 ^ kswz(f)) * 32) + 16 * h);
    };
    auto store_px = [&](T* out, int C, int slot, int fbase, const f32x16& acc, float mul) {
        const int tx = slot & 7, ty = slot >> 3, px = xs + tx, py = y0 + ty;
        if (w.ok && tx < ws && ty < ws && px >= 0 && px < W_ && py >= 0 && py < H_) {
            T* ob = out + (int64_t)b * C * P_ + (int64_t)py * W_ + px;
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int f = fbase + acc_row(x, h);
                if (f < C) ob[(int64_t)f * P_] = (T)(acc[x] * mul);
            }
        }
    };
    constexpr int NDV = DV / 32 * 2, NDK = D / 32 * 2, NBLK = NDV + 2 * NDK;
#pragma unroll
    for (int i = 0; i < (NBLK + 3) / 4; ++i) {
        const int blk = (wave & 3) + 4 * i;
        if (blk >= NBLK) break;
        f32x16 acc;
#pragma unroll
        for (int x = 0; x < 16; ++x) acc[x] = 0.0f;
        if (blk < NDV) {                              // dVᵀ[cb, kb2] = dOᵀ P
            const int cb = blk >> 1, kb2 = blk & 1, f = cb * 32 + r;
#pragma unroll
            for (int s16 = 0; s16 < 4; ++s16)
                acc = mfma32x32x16(frag_row(ODO, f, s16),
                                   *(const F8*)(wsm + OP + (kb2 * 32 + r) * PROW + (16 * s16 + 8 * h) * 2), acc);
            store_px(dvo, dv, kb2 * 32 + r, cb * 32, acc, 1.0f);
        } else if (blk < NDV + NDK) {                 // dKᵀ[fb, kb2] = τ Qᵀ dS
            const int b2 = blk - NDV, fb = b2 >> 1, kb2 = b2 & 1, f = fb * 32 + r;
#pragma unroll
            for (int s16 = 0; s16 < 4; ++s16)
                acc = mfma32x32x16(frag_row(OQ, f, s16),
                                   *(const F8*)(wsm + ODS + (kb2 * 32 + r) * PROW + (16 * s16 + 8 * h) * 2), acc);
            store_px(dk, d, kb2 * 32 + r, fb * 32, acc, scale);
        } else {                                      // dQᵀ[fb, qb2] = τ Kᵀ dSᵀ
            const int b2 = blk - NDV - NDK, fb = b2 >> 1, qb2 = b2 & 1, f = fb * 32 + r;
#pragma unroll
            for (int s16 = 0; s16 < 4; ++s16) {
                const char* a = wsm + ODS + (16 * s16 + 8 * h + qq) * PROW + (qb2 * 32 + kh * 16 + 4 * pp) * 2;
                const F8 bt = __builtin_shufflevector(__builtin_bit_cast(F4, ds_read_tr16(a)),
                                                      __builtin_bit_cast(F4, ds_read_tr16(a + 4 * PROW)),
                                                      0, 1, 2, 3, 4, 5, 6, 7);
                acc = mfma32x32x16(frag_row(OK_, f, s16), bt, acc);
            }
            store_px(dq, d, qb2 * 32 + r, fb * 32, acc, scale);
        }
    }
    FA_STAMP(4);
    FA_STAMP(5);
}

// --------------------------------------------------------------------------
// Strip BACKWARD: the eight windows of a forward strip per workgroup, one per
// wave (bf16/f16, 2-D, stride == ws <= 7, d, dv <= 64, width % 8 == 0, 16-B
// aligned tensors; the default from kStripBwdMin strips on).  Same strip
// geometry, rotated slots and swizzled LDS-DMA images as win_strip; every
// gradient leaves as whole 16-B chunks of the strip's pixels.
//
//   phase A  (16-feature chunks, Sᵀ-style images): Sᵀ = K·Qᵀ, keys on accumulator
//            rows, queries on lanes, as in the forward; P = exp(τS − lse) from the
//            forward's (l, m) (read by a dword DMA) as bf16 B fragments (n = query)
//            while the dO / V chunks land; then dPᵀ = V·dOᵀ in the same
//            accumulators; D = rowsum(P ∘ dP) in-lane (= rowsum(dO ∘ y): y is
//            never read); τ dS = τ P ∘ (dP − D) as bf16 B fragments.  The phase-B
//            A operands of K and Q (lane = feature) are read from the same images
//            into registers, so the strip's data is loaded from HBM once.
//   phase B  (no loads): Pᵀ and dSᵀ with keys on lanes by an identity MFMA
//            (C = A·I with the fragments as A: exact, no LDS round trip);
//            dVᵀ = dOᵀ P (dO rows from the (dO, V) images, still in the ring),
//            dKᵀ = Qᵀ (τ dS), dQᵀ = Kᵀ (τ dS)ᵀ, 32 output features at a time, each
//            written as a 16-feature strip image [16 f][8 rows][64 px] (twice) and
//            stored as whole 16-B chunks.
//   loads    : a ring of four 32-KB buffers refilled as soon as a slot is read
//            (Q / K slots at once, dO / V slots after dV), continuing into the
//            next strip (persistent: one workgroup per CU over consecutive
//            strips); exact vmcnt counts (loads, DMAs and stores retire in order);
//            LDS-only barriers.
// Keys / queries outside the window (slot row >= ws, columns outside [c0, c1))
// are masked (K / V fragments zeroed, -inf exponent bias, selects on the query
// lanes), so a non-finite neighbour pixel never enters this window's sums.
// --------------------------------------------------------------------------
#define FA_VM_CASE(N) \
    case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
__device__ __forceinline__ void wait_vm(int n) {   // n: even, 0 .. 46 (anything else waits for all)
    switch (n) {
        FA_VM_CASE(0) FA_VM_CASE(2) FA_VM_CASE(4) FA_VM_CASE(6) FA_VM_CASE(8) FA_VM_CASE(10) FA_VM_CASE(12)
        FA_VM_CASE(14) FA_VM_CASE(16) FA_VM_CASE(18) FA_VM_CASE(20) FA_VM_CASE(22) FA_VM_CASE(24) FA_VM_CASE(26)
        FA_VM_CASE(28) FA_VM_CASE(30) FA_VM_CASE(32) FA_VM_CASE(34) FA_VM_CASE(36) FA_VM_CASE(38) FA_VM_CASE(40)
        FA_VM_CASE(42) FA_VM_CASE(44) FA_VM_CASE(46)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}
#undef FA_VM_CASE

// Per-lane store plan of a 16-feature strip image, fixed for the strip: unit
// u = it * 512 + tid (it = 0, 1) is (feature it * 8 + (tid >> 6), row (tid >> 3) & 7,
// 16-B chunk tid & 7); the two units differ by constants.
struct StripStore {
    int go0;          // byte offset of the unit's chunk in the slab, feature 0
    int roff;         // LDS byte offset of unit 0 in the image
    bool full;        // a whole in-image 16-B chunk
    bool part;        // straddles a strip end (2-B stores; only when the ends are unaligned)
    int e0, e1;       // the straddling chunk's pixels inside the strip: [e0, e1)
};
__device__ __forceinline__ StripStore strip_store_plan(int tid, int y0, int ws, int H_, int W_, int X0, int xlo, int xhi) {
    const int f = tid >> 6, row = (tid >> 3) & 7, j = tid & 7;
    const int y = y0 + row, x0 = X0 + 8 * j;
    const bool rok = row < ws && y >= 0 && y < H_ && x0 + 8 > xlo && x0 < xhi;
    StripStore p;
    p.full = rok && x0 >= xlo && x0 + 8 <= xhi;
    p.part = rok && !p.full;
    p.go0 = (y * W_ + x0) * 2;                       // + feature * P * 2 at the store
    p.roff = f * 1024 + row * 128 + ((j ^ simg_swz(f, row)) << 4);
    p.e0 = max(xlo - x0, 0);
    p.e1 = min(xhi - x0, 8);
    return p;
}

// A 16-feature strip image [16 f][8 rows][64 px] (simg_pos) of output features
// fbase .. fbase + 15 as 16-B chunk stores, 2 per lane (invalid lanes get an
// out-of-range offset: the store is dropped); chunks straddling a strip end as
// 2-B stores (PARTIAL only).
template <class T, bool PARTIAL>
__device__ __forceinline__ void strip_store16(const char* img, __amdgpu_buffer_rsrc_t ors, const StripStore& sp, int tid,
                                              int fbase, int C, int P_) {
    if (FA_WIN_ABL & 32) return;
    const int f = tid >> 6;
    u32x4 val[2];
    const uint32_t ra = lds_off(img) + sp.roff;      // unit 1: + 8 KB
    asm volatile("ds_read_b128 %0, %1" : "=v"(val[0]) : "v"(ra) : "memory");
    asm volatile("ds_read_b128 %0, %1 offset:8192" : "=v"(val[1]) : "v"(ra) : "memory");
    lds_wait();
    lds_fence(val[0]);
    lds_fence(val[1]);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int fg = fbase + it * 8 + f;
        const bool ok = fg < C && sp.full;
        __builtin_amdgcn_raw_buffer_store_b128(val[it], ors, ok ? sp.go0 + fg * P_ * 2 : 0x7FFFFFF0, 0, 0);
    }
    if (PARTIAL && sp.part) {                        // only when some strip end is not on a 16-B chunk
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            const int fg = fbase + it * 8 + f;
            if (fg >= C) continue;
            const int go = sp.go0 + fg * P_ * 2;
            for (int e = 0; e < 8; ++e)
                if (e >= sp.e0 && e < sp.e1)
                    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(val[it][e >> 1] >> (16 * (e & 1))), ors,
                                                          go + 2 * e, 0, 0);
        }
    }
}

// 8 accumulator values (registers X0 .. X0 + 7: features acc_row(x, h) - 16 (X0 / 8) of one
// slot) into a 16-feature strip image at base (= simg_pos(4h, row, px)): the feature offsets
// are immediates (the swizzle depends on feature bit 2 = h only); pairs share one conversion.
template <class T, int X0, int X = X0>
__device__ __forceinline__ void img_w8(uint32_t base, const f32x16& acc) {
    if constexpr (X < X0 + 8) {
        typedef T T2 __attribute__((ext_vector_type(2)));
        typedef float F2 __attribute__((ext_vector_type(2)));
        const T2 pr = __builtin_convertvector((F2){acc[X], acc[X + 1]}, T2);
        const unsigned u = __builtin_bit_cast(unsigned, pr);
        constexpr int f0 = (X & 3) + 8 * (X >> 2) - 2 * X0, f1 = ((X + 1) & 3) + 8 * ((X + 1) >> 2) - 2 * X0;
        asm volatile("ds_write_b16 %0, %1 offset:%2" : : "v"(base), "v"(u), "i"(f0 * 1024) : "memory");
        asm volatile("ds_write_b16_d16_hi %0, %1 offset:%2" : : "v"(base), "v"(u), "i"(f1 * 1024) : "memory");
        img_w8<T, X0, X + 2>(base, acc);
    }
}

struct StripPos {                                    // one strip: batch slab, window row, first window
    int b, wy, y0, wx0, nvalid;
};

template <class T, int D, int DV, bool PARTIAL>
__global__ __launch_bounds__(512, 1) void win_bwd_strip(const T* __restrict__ q, const T* __restrict__ k,
                                                        const T* __restrict__ v, const T* __restrict__ dy,
                                                        const float* __restrict__ lw, const float* __restrict__ mw,
                                                        T* __restrict__ dq, T* __restrict__ dk, T* __restrict__ dvo,
                                                        WinDev g, int d, int dv, int nsx, int k0, int nstrip,
                                                        unsigned* __restrict__ ctr, float scale, float scale_log2) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    static_assert(D % 32 == 0 && D <= 64 && DV % 32 == 0 && DV <= 64, "head dims");
    constexpr int NQK = D / 16, NOV = DV / 16, NA = NQK + NOV;   // loads: (Q, K), then (dO, V) 16-feature chunks
    constexpr int NC = D / 32, NCV = DV / 32;        // 32-feature output chunks of dQ / dK and of dV
    constexpr int R = 4, BUF = 32768, IMG = 16384;
    static_assert(NA >= R, "every ring slot is a load of the strip");
    __shared__ __attribute__((aligned(16))) char smem[R * BUF + IMG + 2 * 2 * 8 * 64 * 4 + 16];
    char* const img = smem + R * BUF;                // 16-feature gradient image
    float* const lms = (float*)(img + IMG);          // l, m of a strip's windows: [parity][l | m][window][64]
    unsigned* const nsid_lds = (unsigned*)(img + IMG + 2 * 2 * 8 * 64 * 4);   // the next strip, broadcast

    // lane-derived values are re-derived from an opaque copy of threadIdx.x in every strip
    // iteration: hoisted out of the loop, their many per-lane addresses would stay live and spill
    int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int W_ = g.S[0], H_ = g.S[1], P_ = g.P, ws = g.ws, st = g.stride, nwx = g.O[0];
    auto pos_of = [&](int sid) __attribute__((always_inline)) {
        const int sxi = sid % nsx, t0 = sid / nsx;
        StripPos p;
        p.wy = t0 % g.O[1];
        p.b = t0 / g.O[1];
        p.wx0 = sxi == 0 ? 0 : k0 + (sxi - 1) * kStripW;
        p.y0 = p.wy * st - g.pad;
        p.nvalid = min(sxi == 0 ? k0 : kStripW, nwx - p.wx0);
        return p;
    };
    auto ax_of = [&](const StripPos& p, int w) __attribute__((always_inline)) {
        return min(max(((p.wx0 + w) * st - g.pad) & ~1, 0), W_ - 8);
    };
    // one DMA instruction = one feature row fl of an Sᵀ-style image: lane -> (slot row, window)
    auto dma_qk = [&](const StripPos& p, __amdgpu_buffer_rsrc_t rs, char* im, int fl, int fg, int C)
        __attribute__((always_inline)) {
        const int pc = lane >> 3, pw = lane & 7;
        const int w = pw ^ sqk_swz(fl, pc), y = p.y0 + pc;
        const bool ok = w < p.nvalid && pc < ws && y >= 0 && y < H_ && fg < C;
        const int off = ok ? (fg * P_ + y * W_ + ax_of(p, w)) * 2 : 0x7FFFFFF0;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(im + fl * 1024), 16,
                                                 off, 0, 0, 0);
    };
    // VMEM instructions this wave has issued (loads, DMAs, counted stores), and the count
    // right after each ring slot's load: the wait for a slot is vmcnt(issued - mark)
    // (loads, stores and DMA retire in issue order: MI355X_MICROARCH, vmcnt).  Slots are
    // runtime values (a strip's NA loads need not be a multiple of R), so the marks are
    // four scalars, not an array (which would go to scratch).
    int vm_issued = 0;
    int mark0 = 0, mark1 = 0, mark2 = 0, mark3 = 0;
    auto mark_of = [&](int slot) __attribute__((always_inline)) {
        return slot == 0 ? mark0 : slot == 1 ? mark1 : slot == 2 ? mark2 : mark3;
    };
    // load j of strip p into ring slot `slot`: 32 DMA instructions (one feature row each), 4 per
    // wave; a strip's l, m (2 DMA instructions per wave, into parity par) right after its load 0
    auto issue = [&](const StripPos& p, int j, int slot, int par) __attribute__((always_inline)) {
        char* buf = smem + slot * BUF;
        const int64_t bo = (int64_t)p.b;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int rr = i * 8 + wave;                 // 0..31
            if (j < NQK) {
                if (rr < 16) dma_qk(p, slab_rsrc(q + bo * d * P_, (uint32_t)(d * P_ * 2)), buf, rr, j * 16 + rr, d);
                else dma_qk(p, slab_rsrc(k + bo * d * P_, (uint32_t)(d * P_ * 2)), buf + 16384, rr - 16,
                            j * 16 + rr - 16, d);
            } else {
                if (rr < 16) dma_qk(p, slab_rsrc(dy + bo * dv * P_, (uint32_t)(dv * P_ * 2)), buf, rr,
                                    (j - NQK) * 16 + rr, dv);
                else dma_qk(p, slab_rsrc(v + bo * dv * P_, (uint32_t)(dv * P_ * 2)), buf + 16384, rr - 16,
                            (j - NQK) * 16 + rr - 16, dv);
            }
        }
        vm_issued += 4;
        mark0 = slot == 0 ? vm_issued : mark0;
        mark1 = slot == 1 ? vm_issued : mark1;
        mark2 = slot == 2 ? vm_issued : mark2;
        mark3 = slot == 3 ? vm_issued : mark3;
        if (j == 0) {
            const int64_t wrow = (int64_t)g.T * ((int64_t)nwx * p.wy + (int64_t)g.L * p.b);   // window (0, wy)
            const int off = (wave < p.nvalid && lane < g.T) ? (g.T * (p.wx0 + wave) + lane) * 4 : 0x7FFFFFF0;
            float* dst = lms + par * 1024 + wave * 64;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(slab_rsrc(lw + wrow, (uint32_t)(g.T * nwx * 4)),
                                                     (__attribute__((address_space(3))) void*)dst, 4, off, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(slab_rsrc(mw + wrow, (uint32_t)(g.T * nwx * 4)),
                                                     (__attribute__((address_space(3))) void*)(dst + 512), 4, off, 0, 0,
                                                     0);
            vm_issued += 2;
        }
    };

    // Strips are dealt dynamically within XCD groups.  Workgroup b belongs to group
    // x = b mod 8 (the XCD the dispatcher deals it to), and group x owns the contiguous
    // strip range [lo, hi), sized in proportion to its M workgroups (>= M strips, as
    // nstrip >= G): its workgroup l takes strips lo + l and lo + l + M, then lo + 2M + c
    // for each c it draws from the group's counter (zeroed by the launcher, 64 B apart).
    // So neighbouring strips of a window row, which share the 128-B lines at their ends,
    // run at about the same time on one XCD and meet in its L2 (dealt chip-wide, each
    // shared line was fetched once per XCD that touched it: 2.0x the algorithmic bytes
    // in FETCH_SIZE, r03_win_strip_pmc.txt).  Workgroups start up to ~20 us apart and run
    // at different speeds; a static deal of 8 strips each left ~11 % of the CUs idle and
    // a ~20 us tail.  The draw for the strip after next is issued by lane 0 of wave 0
    // right after a strip's first wait and counted as a vector-memory op; its answer is
    // certain to have landed at the next strip's first wait (every DMA of that strip was
    // issued after it), where it is broadcast through LDS.
    const int G = (int)gridDim.x;
    const int NG = G < 8 ? G : 8, grp = (int)blockIdx.x % NG;
    const int M = G / NG + (grp < G % NG ? 1 : 0);   // workgroups of the group
    auto cum = [&](int x) { return x * (G / NG) + min(x, G % NG); };   // workgroups of groups < x
    const int lo = (int)((int64_t)nstrip * cum(grp) / G), hi = (int)((int64_t)nstrip * cum(grp + 1) / G);
    unsigned* const gctr = ctr + 16 * grp;
    int sid = lo + (int)blockIdx.x / NG;
    int nsid = sid + M;                              // the strip after cur
    unsigned drawn = 0u;                             // lane 0 of wave 0: the counter's last answer
    StripPos cur = pos_of(sid);
#pragma unroll
    for (int j = 0; j < R; ++j) issue(cur, j, j, 0);
    int gbase = 0;                                   // ring slot of the current strip's load 0

    int g4, kh, qq, pp, sig;
    const unsigned one = std::is_same<T, bf16>::value ? 0x3F80u : 0x3C00u;
    // one-hot B fragment: element e of lane (r, h) is 1 iff 16 s2 + 8 h + e == r
    auto ident = [&](int s2) __attribute__((always_inline)) {
        const int e = r - 16 * s2 - 8 * h;
        u32x4 u = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (e == 2 * i) u[i] = one;
            if (e == 2 * i + 1) u[i] = one << 16;
        }
        return __builtin_bit_cast(F8, u);
    };
    const F8 id0 = ident(0), id1 = ident(1);

    for (int it = 0; sid < hi; ++it) {
        [[maybe_unused]] const int fa_sid = sid;
        FA_BSTAMP(0);
        tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        lane = tid & 63; r = lane & 31; h = lane >> 5;
        g4 = lane >> 4; kh = g4 & 1; qq = (lane & 15) >> 2; pp = lane & 3;
        sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
        bool has_next = false;                       // set at the first wait (refills use it later)
        StripPos nxt = cur;
        const int par = it & 1;
        auto slot_of = [&](int j) __attribute__((always_inline)) { return (gbase + j) & (R - 1); };
        // load j landed in every wave: its own DMA (counted wait), then the LDS barrier
        auto step_wait = [&](int j) __attribute__((always_inline)) {
            __builtin_amdgcn_sched_barrier(0);          // keep each step's work in its step (register pressure)
            wait_vm(vm_issued - mark_of(slot_of(j)));
            if (j == 0 && it > 0 && wave == 0) {
                asm volatile("" : "+v"(drawn));          // landed with this wait (see the deal above)
                if (lane == 0) lds_w32u(nsid_lds, (unsigned)(lo + 2 * M) + drawn);
            }
            lds_barrier();
            if (j == 0) {
                if (it > 0) {
                    nsid = (int)__builtin_bit_cast(unsigned, lds_b32(nsid_lds));
                    lds_wait();
                    asm volatile("" : "+v"(nsid));
                    nsid = __builtin_amdgcn_readfirstlane(nsid);
                }
                has_next = nsid < hi;
                nxt = has_next ? pos_of(nsid) : cur;
                if (wave == 0) {                         // draw the strip after nsid
                    if (lane == 0) drawn = atomic_add_ret(gctr, 1u);
                    vm_issued += 1;
                }
            }
            FA_BSTAMP(1 + j);
        };
        // ring slot of load j is free: issue the load R later in the stream (this strip's, or the next's)
        auto refill = [&](int j) __attribute__((always_inline)) {
            if (j + R < NA) issue(cur, j + R, slot_of(j), par);
            else if (has_next) issue(nxt, j + R - NA, slot_of(j), par ^ 1);
        };

        // ---- this wave's window ----
        const int wl = wave;
        const bool wok = wl < cur.nvalid;
        const int y0 = cur.y0, b = cur.b;
        const int wx = cur.wx0 + wl, xs = wx * st - g.pad, ax = ax_of(cur, wl);
        const int c0 = xs - ax, c1 = c0 + ws;
        auto slot_ok = [&](int s) __attribute__((always_inline)) {   // slot s of this window: a real token of the image
            const int sx = s & 7, sy = s >> 3;
            return wok && sy < ws && sx >= c0 && sx < c1 && y0 + sy >= 0 && y0 + sy < H_;
        };
        // Masking.  Keys: the K / V fragments (A operands; lane = key) are zeroed per lane for
        // keys outside the window (slot row >= ws or column outside [c0, c1)), so Sᵀ and dPᵀ are
        // finite there whatever the neighbour pixels hold; P gets a -inf exponent bias for those
        // keys: per column (register x & 7, wave-uniform) and per slot row (lane half, kb, x >> 3).
        // Queries (lanes): P and dS are selected to 0 outside the window.  Rows outside the image
        // are zero-padding tokens, as in the forward (P > 0, K = V = 0: no contribution).
        bool qv[2];
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            const int qs = qb * 32 + r;
            qv[qb] = wok && (qs >> 3) < ws && (qs & 7) >= c0 && (qs & 7) < c1;
        }
        bool kfv[2];                                     // this lane's key (A row) of tr-read block blk: lane i of
        {                                                // a 16-lane group receives column i, i.e. chunk qq
            const int sq = (qq == 1) ? 2 : (qq == 2) ? 1 : qq;   // sig of the supplying lanes
#pragma unroll
            for (int blk = 0; blk < 2; ++blk) {
                const int krow = 4 * blk + 2 * kh + (sq >> 1), kcol = 4 * (sq & 1) + (lane & 3);
                kfv[blk] = krow < ws && kcol >= c0 && kcol < c1;
            }
        }
        float colb[8], rowb[2][2];                       // 0 or -inf exponent bias
#pragma unroll
        for (int c = 0; c < 8; ++c) colb[c] = (c >= c0 && c < c1) ? 0.0f : kNegInf;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int x2 = 0; x2 < 2; ++x2) rowb[kb][x2] = (kb * 4 + 2 * x2 + h < ws) ? 0.0f : kNegInf;

        f32x16 acc[2][2];                                // Sᵀ over the (Q, K) chunks, then dPᵀ: [key block][query block]
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                for (int x = 0; x < 16; ++x) acc[kb][qb][x] = 0.0f;
        F8 pf[2][2][2], dsf[2][2][2];                    // P, τ dS: [query block][key block][16-key half]
        // phase-B A operands kept in registers (lane r = feature 32 c + r): K rows for dQ
        // (8 consecutive keys of a slot row), Q rows for dK (the transposed fragments'
        // query order 16 s' + 4h + {0..3, 8..11}); read from the phase-A images
        u32x4 kst[NC][2][2];
        u32x2 qlo[NC][2][2], qhi[NC][2][2];

        // ---- phase A ----
#pragma unroll
        for (int j = 0; j < NA; ++j) {
            step_wait(j);
            const char* buf = smem + slot_of(j) * BUF;
            s16x4 rk[2][2], rq[2][2];                    // keys (K / V, permuted), queries (Q / dO)
#pragma unroll
            for (int blk = 0; blk < 2; ++blk) {
                const char* a = buf + 16384 + sqk_pos(8 * h + qq, 4 * blk + 2 * kh + (sig >> 1), wl) + (sig & 1) * 8;
                rk[blk][0] = lds_tr16(a);
                rk[blk][1] = lds_tr16(buf + 16384 + sqk_pos(8 * h + qq + 4, 4 * blk + 2 * kh + (sig >> 1), wl) + (sig & 1) * 8);
                const char* aq = buf + sqk_pos(8 * h + qq, 4 * blk + 2 * kh + (pp >> 1), wl) + (pp & 1) * 8;
                rq[blk][0] = lds_tr16(aq);
                rq[blk][1] = lds_tr16(buf + sqk_pos(8 * h + qq + 4, 4 * blk + 2 * kh + (pp >> 1), wl) + (pp & 1) * 8);
            }
            if (j < NQK) {                               // this chunk's 16 features of the K / Q stashes
                const int c = j >> 1, fl = r & 15;
                if ((r >> 4) == (j & 1)) {
#pragma unroll
                    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                        for (int s2 = 0; s2 < 2; ++s2)
                            kst[c][kb][s2] = lds_b128(buf + 16384 + sqk_pos(fl, kb * 4 + s2 * 2 + h, wl));
#pragma unroll
                    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                        for (int s_ = 0; s_ < 2; ++s_) {
                            qlo[c][qb][s_] = lds_b64(buf + sqk_pos(fl, qb * 4 + 2 * s_, wl) + 8 * h);
                            qhi[c][qb][s_] = lds_b64(buf + sqk_pos(fl, qb * 4 + 2 * s_ + 1, wl) + 8 * h);
                        }
                }
            }
            lds_wait();
            if (j < NQK) {
                const int c = j >> 1;
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) lds_fence(kst[c][kb][s2]);
#pragma unroll
                for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                    for (int s_ = 0; s_ < 2; ++s_) { lds_fence(qlo[c][qb][s_]); lds_fence(qhi[c][qb][s_]); }
            }
            F8 kf[2], qf[2];
#pragma unroll
            for (int blk = 0; blk < 2; ++blk) {
#pragma unroll
                for (int i = 0; i < 2; ++i) { lds_fence(rk[blk][i]); lds_fence(rq[blk][i]); }
                u32x4 ku = __builtin_bit_cast(u32x4, __builtin_shufflevector(rk[blk][0], rk[blk][1], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
                for (int i = 0; i < 4; ++i) ku[i] = kfv[blk] ? ku[i] : 0u;
                kf[blk] = __builtin_bit_cast(F8, ku);
                qf[blk] = __builtin_shufflevector(__builtin_bit_cast(F4, rq[blk][0]), __builtin_bit_cast(F4, rq[blk][1]),
                                                  0, 1, 2, 3, 4, 5, 6, 7);
            }
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int qb = 0; qb < 2; ++qb) acc[kb][qb] = mfma32x32x16(kf[kb], qf[qb], acc[kb][qb]);
            if (j < NQK) {                               // a Q / K slot is free at once; dO / V stay for dV
                lds_barrier();
                refill(j);
            }
            if (j == NQK - 1) {                          // Sᵀ complete: P = exp(τS − lse) (bf16), while dO / V load
                const float* ls = lms + par * 1024 + wl * 64;
                float lq[2], mq[2];
#pragma unroll
                for (int qb = 0; qb < 2; ++qb) {
                    const int qs = qb * 32 + r;
                    const int tq = qv[qb] ? (qs >> 3) * ws + (qs & 7) - c0 : 0;   // window token of the query slot
                    lq[qb] = lds_b32(ls + tq);
                    mq[qb] = lds_b32(ls + 512 + tq);
                }
                lds_wait();
#pragma unroll
                for (int qb = 0; qb < 2; ++qb) {
                    lds_fence(lq[qb]);
                    lds_fence(mq[qb]);
                    const float nl = (mq[qb] + __logf(lq[qb])) * kLog2e;
#pragma unroll
                    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                        for (int x2 = 0; x2 < 2; ++x2) {
                            const float nlb = nl - rowb[kb][x2];           // +inf on slot rows >= ws
                            u32x4 pu;
#pragma unroll
                            for (int e = 0; e < 8; e += 2) {            // packed fp32: v_pk_fma / v_pk_add
                                const int x = 8 * x2 + e;
                                const f32x2 sv = {acc[kb][qb][x], acc[kb][qb][x + 1]};
                                const f32x2 arg = __builtin_elementwise_fma(sv, (f32x2){scale_log2, scale_log2},
                                                                            (f32x2){-nlb, -nlb}) +
                                                  (f32x2){colb[e], colb[e + 1]};
                                const f32x2 pr = {exp2_fast(arg[0]), exp2_fast(arg[1])};
                                pu[e >> 1] = qv[qb] ? pk2<T>(pr) : 0u;
                                acc[kb][qb][x] = acc[kb][qb][x + 1] = 0.0f;
                            }
                            pf[qb][kb][x2] = __builtin_bit_cast(F8, pu);
                        }
                }
                // pin P here, under the dO / V loads (the optimizer would sink it to its first use)
#pragma unroll
                for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                        for (int x2 = 0; x2 < 2; ++x2) asm volatile("" : "+v"(pf[qb][kb][x2]));
            }
        }

        // ---- D = rowsum(P ∘ dP), τ dS = τ P ∘ (dP − D) per query (lane) ----
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            f32x2 ds2 = {0.0f, 0.0f};
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int x = 0; x < 16; x += 2)
                    ds2 = __builtin_elementwise_fma(unpk2<T>(__builtin_bit_cast(u32x4, pf[qb][kb][x >> 3])[(x & 7) >> 1]),
                                                    (f32x2){acc[kb][qb][x], acc[kb][qb][x + 1]}, ds2);
            const float Dq = swap_halves_sum(ds2[0] + ds2[1]);
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int x2 = 0; x2 < 2; ++x2) {
                    u32x4 du;
#pragma unroll
                    for (int e = 0; e < 8; e += 2) {
                        const int x = 8 * x2 + e;
                        const f32x2 p2 = unpk2<T>(__builtin_bit_cast(u32x4, pf[qb][kb][x2])[e >> 1]);
                        const f32x2 t = (p2 * ((f32x2){acc[kb][qb][x], acc[kb][qb][x + 1]} - Dq)) * scale;
                        du[e >> 1] = qv[qb] ? pk2<T>(t) : 0u;   // (select: dPᵀ of a query outside the window may be inf)
                    }
                    dsf[qb][kb][x2] = __builtin_bit_cast(F8, du);
                }
        }

        // ---- phase B: dVᵀ = dOᵀ P, dKᵀ = Qᵀ (τ dS), dQᵀ = Kᵀ (τ dS)ᵀ, 32 output features at a time,
        //      each stored through the 16-feature image in two passes ----
        const int xs0 = cur.wx0 * st - g.pad, X0 = xs0 & ~7;   // strip start, its 16-B aligned base
        const int xlo = max(xs0, 0), xhi = min(xs0 + cur.nvalid * ws, W_);
        unsigned cm[4];                                  // slot-column mask of a 16-B row fragment
#pragma unroll
        for (int j = 0; j < 4; ++j)
            cm[j] = ((2 * j >= c0 && 2 * j < c1) ? 0x0000FFFFu : 0u) | ((2 * j + 1 >= c0 && 2 * j + 1 < c1) ? 0xFFFF0000u : 0u);
        const StripStore sp = strip_store_plan(tid, y0, ws, H_, W_, X0, xlo, xhi);
        // one 32 x 32 output block pair (features on accumulator rows, slot kb/qb * 32 + r on the
        // lane) through the image: features 0..15, then 16..31
        auto out_chunk = [&](const f32x16 (&oa)[2], T* base, int C, int fbase) __attribute__((always_inline)) {
            const auto ors = slab_rsrc(base + (int64_t)b * C * P_, (uint32_t)(C * P_ * 2));
#pragma unroll
            for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
                for (int blk = 0; blk < 2; ++blk) {
                    const int s = blk * 32 + r;
                    if (slot_ok(s) && !(FA_WIN_ABL & 64)) {
                        const uint32_t a0 = lds_off(img) + simg_pos(4 * h, s >> 3, ax + (s & 7) - X0);
                        if (pass == 0) img_w8<T, 0>(a0, oa[blk]);
                        else img_w8<T, 8>(a0, oa[blk]);
                    }
                }
                lds_barrier();
                strip_store16<T, PARTIAL>(img, ors, sp, tid, fbase + 16 * pass, C, P_);
                if (!PARTIAL && !(FA_WIN_ABL & 32)) vm_issued += 2;
                lds_barrier();                           // the image is free again
            }
        };
        // transpose: block (kb, qb) of X (B fragments, queries on lanes) -> keys on lanes, then
        // B fragments [key block][query block][s'] whose query order is 16 s' + 4h + {0..3, 8..11}
        auto transpose = [&](const F8 (&xf)[2][2][2], F8 (&xt)[2][2][2]) __attribute__((always_inline)) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int qb = 0; qb < 2; ++qb) {
                    f32x16 c;
#pragma unroll
                    for (int x = 0; x < 16; ++x) c[x] = 0.0f;
                    c = mfma32x32x16(xf[qb][kb][0], id0, c);
                    c = mfma32x32x16(xf[qb][kb][1], id1, c);
#pragma unroll
                    for (int x = 0; x < 16; ++x) xt[kb][qb][x >> 3][x & 7] = (T)c[x];
                }
        };
        // keys on lanes: oa[kb] = Σ A(f, queries) · xt[kb]
        // this lane's two column masks (selects, not a lane-indexed array: that went to scratch)
        const unsigned cmh0 = h ? cm[2] : cm[0], cmh1 = h ? cm[3] : cm[1];
        auto keys_out = [&](const u32x2 (&lo)[2][2], const u32x2 (&hi)[2][2], const F8 (&xt)[2][2][2], f32x16 (&oa)[2])
            __attribute__((always_inline)) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int x = 0; x < 16; ++x) oa[kb][x] = 0.0f;
#pragma unroll
            for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                for (int s_ = 0; s_ < 2; ++s_) {
                    const u32x4 u = {lo[qb][s_][0] & cmh0, lo[qb][s_][1] & cmh1, hi[qb][s_][0] & cmh0, hi[qb][s_][1] & cmh1};
                    const F8 af = __builtin_bit_cast(F8, u);
#pragma unroll
                    for (int kb = 0; kb < 2; ++kb) oa[kb] = mfma32x32x16(af, xt[kb][qb][s_], oa[kb]);
                }
        };
        FA_BSTAMP(18);
        F8 xt[2][2][2];
        transpose(pf, xt);
        FA_BSTAMP(19);
        // dVᵀ: dO rows from the (dO, V) images still in the ring; each frees two ring slots
#pragma unroll
        for (int c = 0; c < NCV; ++c) {
            u32x2 lo[2][2], hi[2][2];
            {
                const int j = NQK + 2 * c + (r >> 4);    // this lane's feature's (dO, V) load
                const char* buf = smem + slot_of(j) * BUF;
                const int fl = r & 15;
#pragma unroll
                for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                    for (int s_ = 0; s_ < 2; ++s_) {
                        lo[qb][s_] = lds_b64(buf + sqk_pos(fl, qb * 4 + 2 * s_, wl) + 8 * h);
                        hi[qb][s_] = lds_b64(buf + sqk_pos(fl, qb * 4 + 2 * s_ + 1, wl) + 8 * h);
                    }
                lds_wait();
#pragma unroll
                for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                    for (int s_ = 0; s_ < 2; ++s_) { lds_fence(lo[qb][s_]); lds_fence(hi[qb][s_]); }
            }
            lds_barrier();                               // every wave has read both slots
            if (c == 0) FA_BSTAMP(20);
            f32x16 oa[2];
            keys_out(lo, hi, xt, oa);
            refill(NQK + 2 * c);
            refill(NQK + 2 * c + 1);
            if (c == 0) FA_BSTAMP(21);
            out_chunk(oa, dvo, dv, 32 * c);
            FA_BSTAMP(9 + c);
        }
        // dKᵀ (keys on lanes), from the Q stash
        transpose(dsf, xt);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            f32x16 oa[2];
            keys_out(qlo[c], qhi[c], xt, oa);
            out_chunk(oa, dk, d, 32 * c);
            FA_BSTAMP(11 + c);
        }
        // dQᵀ (queries on lanes), from the K stash
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            f32x16 oa[2];
#pragma unroll
            for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                for (int x = 0; x < 16; ++x) oa[qb][x] = 0.0f;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    u32x4 kr = kst[c][kb][s2];
#pragma unroll
                    for (int i = 0; i < 4; ++i) kr[i] &= cm[i];
#pragma unroll
                    for (int qb = 0; qb < 2; ++qb)
                        oa[qb] = mfma32x32x16(__builtin_bit_cast(F8, kr), dsf[qb][kb][s2], oa[qb]);
                }
            out_chunk(oa, dq, d, 32 * c);
            FA_BSTAMP(13 + c);
        }
        FA_BSTAMP(15);
        cur = nxt;
        sid = nsid;
        gbase = (gbase + NA) & (R - 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the last draw and stores retire before exit
}

// --------------------------------------------------------------------------
// fp32 fused windowed forward (2-D, stride >= ws, ws <= 8, d, dv <= 64, W >= 8):
// one window per workgroup on the exact-f32 MFMA v_mfma_f32_32x32x2_f32 (the
// arithmetic of an fmaf chain, like the fp32 dense path).  Staging: each
// (feature, window row) item is two 16-B loads of the 8 pixels starting at
// a = clamp(xs, 0, W - 8) (fp32 pixels are dword aligned, so the window-uniform
// shift xs - a is a dword select), masked (slot < ws, pixel in the image) and
// written to [feature][65-float] LDS rows (conflict-free for both the column
// reads of the score product and the row reads of the PV product).  Wave
// (qb, vc): Sᵀ = K·Qᵀ for query block qb, exact softmax per query, then
// Oᵀ = Vᵀ·Pᵀ for its 32-feature chunk with the score accumulators as the B
// operand (register x of lane (r, h) holds key acc_row(x, h): k = h).
// --------------------------------------------------------------------------
template <int D, int DV>
__global__ __launch_bounds__(256) void win_rows_f32(const float* __restrict__ q, const float* __restrict__ k,
                                                    const float* __restrict__ v, float* __restrict__ out,
                                                    float* __restrict__ lo, float* __restrict__ mo, WinDev g,
                                                    int d, int dv, float scale, float scale_log2) {
    constexpr int NTH = 256, ROW = 65;
    constexpr int QI = 0, KI = D * ROW, VI = 2 * D * ROW, REGION = (2 * D + DV) * ROW;
    constexpr int NIQ = D * 8 / NTH, NIV = DV * 8 / NTH;
    static_assert(D * 8 % NTH == 0 && DV * 8 % NTH == 0, "item split");
    __shared__ float sm[REGION];
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int W_ = g.S[0], H_ = g.S[1], P_ = g.P, ws = g.ws, st = g.stride;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int wx = bid % g.O[0], wy = (bid / g.O[0]) % g.O[1], b = bid / (g.O[0] * g.O[1]);
    const int xs = wx * st - g.pad, y0 = wy * st - g.pad;
    const int ax = min(max(xs, 0), W_ - 8);
    const int sh = xs - ax;                                    // slot t <- loaded pixel t + sh
    auto item_off = [&](int it, int C) {
        const int yy = it & 7, f = it >> 3, yr = y0 + yy;
        const bool ok = yy < ws && yr >= 0 && yr < H_ && f < C;
        return ok ? (f * P_ + yr * W_ + ax) * 4 : 0x7FFFFFE0;
    };
    const auto qrs = slab_rsrc(q + (int64_t)b * d * P_, (uint32_t)(d * P_ * 4));
    const auto krs = slab_rsrc(k + (int64_t)b * d * P_, (uint32_t)(d * P_ * 4));
    const auto vrs = slab_rsrc(v + (int64_t)b * dv * P_, (uint32_t)(dv * P_ * 4));
    u32x4 rq[NIQ][2], rk[NIQ][2], rv[NIV][2];
#pragma unroll
    for (int j = 0; j < NIQ; ++j) {
        const int o = item_off(tid + NTH * j, d);
        rq[j][0] = __builtin_amdgcn_raw_buffer_load_b128(qrs, o, 0, 0);
        rq[j][1] = __builtin_amdgcn_raw_buffer_load_b128(qrs, o + 16, 0, 0);
        rk[j][0] = __builtin_amdgcn_raw_buffer_load_b128(krs, o, 0, 0);
        rk[j][1] = __builtin_amdgcn_raw_buffer_load_b128(krs, o + 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NIV; ++j) {
        const int o = item_off(tid + NTH * j, dv);
        rv[j][0] = __builtin_amdgcn_raw_buffer_load_b128(vrs, o, 0, 0);
        rv[j][1] = __builtin_amdgcn_raw_buffer_load_b128(vrs, o + 16, 0, 0);
    }
    bool valid[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) valid[t] = t < ws && xs + t >= 0 && xs + t < W_;
    auto stage = [&](const u32x4 (&raw)[2], int it, int img) {
        const int yy = it & 7, f = it >> 3;
        unsigned px[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) px[t] = t < 4 ? raw[0][t] : raw[1][t - 4];
        float* dst = sm + img + f * ROW + yy * 8;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int src = t + sh;
            unsigned val = 0u;
#pragma unroll
            for (int e = 0; e < 8; ++e) val = src == e ? px[e] : val;
            dst[t] = valid[t] ? __uint_as_float(val) : 0.0f;
        }
    };
#pragma unroll
    for (int j = 0; j < NIQ; ++j) {
        stage(rq[j], tid + NTH * j, QI);
        stage(rk[j], tid + NTH * j, KI);
    }
#pragma unroll
    for (int j = 0; j < NIV; ++j) stage(rv[j], tid + NTH * j, VI);
    __syncthreads();

    const int qb = wave & 1, vc = wave >> 1;
    f32x16 sa[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int x = 0; x < 16; ++x) sa[kb][x] = 0.0f;
#pragma unroll
        for (int t = 0; t < D / 2; ++t)
            sa[kb] = mfma32x32x2(sm[KI + (2 * t + h) * ROW + kb * 32 + r], sm[QI + (2 * t + h) * ROW + qb * 32 + r], sa[kb]);
    }
    // mask padding key slots, exact softmax per query (lanes r and r + 32 share query r)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int x = 0; x < 16; ++x) {
            const int kt = kb * 32 + acc_row(x, h);
            if ((kt & 7) >= ws || (kt >> 3) >= ws) sa[kb][x] = kNegInf;
        }
    const float mt = swap_halves_max(lane_max<2>(sa));
    const float mc = mt * scale_log2;
    float ps[4];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int x = 0; x < 16; ++x) {
            const float pr = exp2_fast(fmaf(sa[kb][x], scale_log2, -mc));
            if (kb == 0 && x < 4) ps[x] = pr; else ps[x & 3] += pr;
            sa[kb][x] = pr;
        }
    const float lt = swap_halves_sum((ps[0] + ps[1]) + (ps[2] + ps[3]));
    const int qslot = qb * 32 + r, qtx = qslot & 7, qty = qslot >> 3;
    if (vc < DV / 32) {
        f32x16 oa;
#pragma unroll
        for (int x = 0; x < 16; ++x) oa[x] = 0.0f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int x = 0; x < 16; ++x)
                oa = mfma32x32x2(sm[VI + (vc * 32 + r) * ROW + kb * 32 + acc_row(x, h)], sa[kb][x], oa);
        const int px = xs + qtx, py = y0 + qty;
        if (qtx < ws && qty < ws && px >= 0 && px < W_ && py >= 0 && py < H_) {
            const float inv = 1.0f / lt;
            float* yb = out + (int64_t)b * dv * P_ + (int64_t)py * W_ + px;
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int cc = vc * 32 + acc_row(x, h);
                if (cc < dv) yb[(int64_t)cc * P_] = oa[x] * inv;
            }
        }
    }
    if (vc == 0 && h == 0 && qtx < ws && qty < ws) {
        const int64_t wid = (int64_t)(wx + g.O[0] * wy) + (int64_t)g.L * b;
        const int64_t li = qty * ws + qtx + (int64_t)g.T * wid;
        mo[li] = mt * scale;
        lo[li] = lt;
    }
}

// fp32 fused windowed BACKWARD (same shapes as win_rows_f32, stride >= ws so
// dyw = dy and the fold is a direct store).  Staging as win_rows_f32 for q, k, v,
// dy; y rows feed D = rowsum(dy ∘ y) by LDS float adds.  Phase 1, wave (qb, kb):
// S and dP blocks (queries on accumulator rows, keys on lanes) on exact-f32 MFMA,
// P = exp2(c (S − lse/τ)), dS = P (dP − D), both written to [query][65] LDS rows.
// Phase 2: 12 output blocks over the 4 waves with every operand read from LDS:
// dVᵀ = dOᵀ P, dKᵀ = τ Qᵀ dS (contraction over queries), dQᵀ = τ Kᵀ dSᵀ
// (contraction over keys); each lane stores one slot's features to its pixel.
template <int D, int DV>
__global__ __launch_bounds__(256) void win_bwd_f32(const float* __restrict__ q, const float* __restrict__ k,
                                                   const float* __restrict__ v, const float* __restrict__ y,
                                                   const float* __restrict__ dy, const float* __restrict__ lw,
                                                   const float* __restrict__ mw, float* __restrict__ dq,
                                                   float* __restrict__ dk, float* __restrict__ dvo, WinDev g, int d,
                                                   int dv, float scale, float scale_log2) {
    constexpr int NTH = 256, ROW = 65;
    constexpr int QI = 0, KI = D * ROW, VI = 2 * D * ROW, DOI = VI + DV * ROW, PI = DOI + DV * ROW,
                  DSI = PI + 64 * ROW, LSEI = DSI + 64 * ROW, DI = LSEI + 64, REGION = DI + 64;
    constexpr int NIQ = D * 8 / NTH, NIV = DV * 8 / NTH;
    static_assert(D * 8 % NTH == 0 && DV * 8 % NTH == 0, "item split");
    extern __shared__ float sm[];
    (void)REGION;
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int W_ = g.S[0], H_ = g.S[1], P_ = g.P, ws = g.ws, st = g.stride;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int wx = bid % g.O[0], wy = (bid / g.O[0]) % g.O[1], b = bid / (g.O[0] * g.O[1]);
    const int xs = wx * st - g.pad, y0 = wy * st - g.pad;
    const int ax = min(max(xs, 0), W_ - 8);
    const int sh = xs - ax;
    const int64_t wid = (int64_t)(wx + g.O[0] * wy) + (int64_t)g.L * b;
    auto item_off = [&](int it, int C) {
        const int yy = it & 7, f = it >> 3, yr = y0 + yy;
        const bool ok = yy < ws && yr >= 0 && yr < H_ && f < C;
        return ok ? (f * P_ + yr * W_ + ax) * 4 : 0x7FFFFFE0;
    };
    const auto qrs = slab_rsrc(q + (int64_t)b * d * P_, (uint32_t)(d * P_ * 4));
    const auto krs = slab_rsrc(k + (int64_t)b * d * P_, (uint32_t)(d * P_ * 4));
    const auto vrs = slab_rsrc(v + (int64_t)b * dv * P_, (uint32_t)(dv * P_ * 4));
    const auto yrs = slab_rsrc(y + (int64_t)b * dv * P_, (uint32_t)(dv * P_ * 4));
    const auto drs = slab_rsrc(dy + (int64_t)b * dv * P_, (uint32_t)(dv * P_ * 4));
    u32x4 rq[NIQ][2], rk[NIQ][2], rv[NIV][2], rd[NIV][2], ry[NIV][2];
#pragma unroll
    for (int j = 0; j < NIQ; ++j) {
        const int o = item_off(tid + NTH * j, d);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            rq[j][hh] = __builtin_amdgcn_raw_buffer_load_b128(qrs, o + 16 * hh, 0, 0);
            rk[j][hh] = __builtin_amdgcn_raw_buffer_load_b128(krs, o + 16 * hh, 0, 0);
        }
    }
#pragma unroll
    for (int j = 0; j < NIV; ++j) {
        const int o = item_off(tid + NTH * j, dv);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            rv[j][hh] = __builtin_amdgcn_raw_buffer_load_b128(vrs, o + 16 * hh, 0, 0);
            rd[j][hh] = __builtin_amdgcn_raw_buffer_load_b128(drs, o + 16 * hh, 0, 0);
            ry[j][hh] = __builtin_amdgcn_raw_buffer_load_b128(yrs, o + 16 * hh, 0, 0);
        }
    }
    if (tid < 64) {
        const int tx = tid & 7, ty = tid >> 3;
        float nl = kNegInf;
        if (tx < ws && ty < ws) {
            const int64_t li = ty * ws + tx + (int64_t)g.T * wid;
            nl = -(mw[li] + __logf(lw[li])) / scale;
        }
        sm[LSEI + tid] = nl;
        sm[DI + tid] = 0.0f;
    }
    bool valid[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) valid[t] = t < ws && xs + t >= 0 && xs + t < W_;
    auto pix = [&](const u32x4 (&raw)[2], int t) {
        const int src = t + sh;
        unsigned val = 0u;
#pragma unroll
        for (int e = 0; e < 8; ++e) val = src == e ? (e < 4 ? raw[0][e] : raw[1][e - 4]) : val;
        return valid[t] ? __uint_as_float(val) : 0.0f;
    };
    auto stage = [&](const u32x4 (&raw)[2], int it, int img) {
        const int yy = it & 7, f = it >> 3;
#pragma unroll
        for (int t = 0; t < 8; ++t) sm[img + f * ROW + yy * 8 + t] = pix(raw, t);
    };
#pragma unroll
    for (int j = 0; j < NIQ; ++j) {
        stage(rq[j], tid + NTH * j, QI);
        stage(rk[j], tid + NTH * j, KI);
    }
    __syncthreads();   // D zeroed before the adds
#pragma unroll
    for (int j = 0; j < NIV; ++j) {
        const int it = tid + NTH * j, yy = it & 7, f = it >> 3;
        stage(rv[j], it, VI);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const float a = pix(rd[j], t), yv = pix(ry[j], t);
            sm[DOI + f * ROW + yy * 8 + t] = a;
            const float pr = a * yv;
            if (pr != 0.0f) atomicAdd(&sm[DI + yy * 8 + t], pr);
        }
    }
    __syncthreads();

    // ---- phase 1: S, dP blocks (qb, kb) of this wave ----
    const int qb = wave & 1, kb = wave >> 1;
    f32x16 sa, pa;
#pragma unroll
    for (int x = 0; x < 16; ++x) {
        const int qs = qb * 32 + acc_row(x, h);
        sa[x] = sm[LSEI + qs];
        pa[x] = -sm[DI + qs];
    }
#pragma unroll
    for (int t = 0; t < D / 2; ++t)
        sa = mfma32x32x2(sm[QI + (2 * t + h) * ROW + qb * 32 + r], sm[KI + (2 * t + h) * ROW + kb * 32 + r], sa);
#pragma unroll
    for (int t = 0; t < DV / 2; ++t)
        pa = mfma32x32x2(sm[DOI + (2 * t + h) * ROW + qb * 32 + r], sm[VI + (2 * t + h) * ROW + kb * 32 + r], pa);
    const int kslot = kb * 32 + r;
    const bool kvalid = (kslot & 7) < ws && (kslot >> 3) < ws;
#pragma unroll
    for (int x = 0; x < 16; ++x) {
        const int qs = qb * 32 + acc_row(x, h);
        const float pr = kvalid ? exp2_fast(sa[x] * scale_log2) : 0.0f;
        sm[PI + qs * ROW + kslot] = pr;
        sm[DSI + qs * ROW + kslot] = pr * pa[x];
    }
    __syncthreads();

    // ---- phase 2 ----
    auto store_px = [&](float* out, int C, int slot, int fbase, const f32x16& acc, float mul) {
        const int tx = slot & 7, ty = slot >> 3, px = xs + tx, py = y0 + ty;
        if (tx < ws && ty < ws && px >= 0 && px < W_ && py >= 0 && py < H_) {
            float* ob = out + (int64_t)b * C * P_ + (int64_t)py * W_ + px;
#pragma unroll
            for (int x = 0; x < 16; ++x) {
                const int f = fbase + acc_row(x, h);
                if (f < C) ob[(int64_t)f * P_] = acc[x] * mul;
            }
        }
    };
    constexpr int NDV = DV / 32 * 2, NDK = D / 32 * 2, NBLK = NDV + 2 * NDK;
#pragma unroll
    for (int i = 0; i < (NBLK + 3) / 4; ++i) {
        const int blk = wave + 4 * i;
        if (blk >= NBLK) break;
        f32x16 acc;
#pragma unroll
        for (int x = 0; x < 16; ++x) acc[x] = 0.0f;
        if (blk < NDV) {                              // dVᵀ[cb, kb2] = Σ_q dOᵀ P
            const int cb = blk >> 1, kb2 = blk & 1;
#pragma unroll 8
            for (int t = 0; t < 32; ++t)
                acc = mfma32x32x2(sm[DOI + (cb * 32 + r) * ROW + 2 * t + h], sm[PI + (2 * t + h) * ROW + kb2 * 32 + r], acc);
            store_px(dvo, dv, kb2 * 32 + r, cb * 32, acc, 1.0f);
        } else if (blk < NDV + NDK) {                 // dKᵀ[fb, kb2] = τ Σ_q Qᵀ dS
            const int b2 = blk - NDV, fb = b2 >> 1, kb2 = b2 & 1;
#pragma unroll 8
            for (int t = 0; t < 32; ++t)
                acc = mfma32x32x2(sm[QI + (fb * 32 + r) * ROW + 2 * t + h], sm[DSI + (2 * t + h) * ROW + kb2 * 32 + r], acc);
            store_px(dk, d, kb2 * 32 + r, fb * 32, acc, scale);
        } else {                                      // dQᵀ[fb, qb2] = τ Σ_key Kᵀ dSᵀ
            const int b2 = blk - NDV - NDK, fb = b2 >> 1, qb2 = b2 & 1;
#pragma unroll 8
            for (int t = 0; t < 32; ++t)
                acc = mfma32x32x2(sm[KI + (fb * 32 + r) * ROW + 2 * t + h], sm[DSI + (qb2 * 32 + r) * ROW + 2 * t + h], acc);
            store_px(dq, d, qb2 * 32 + r, fb * 32, acc, scale);
        }
    }
}

static bool rows_f32_ok(const WindowedArgs& a) {
    return g_win_force_composed != 1 && a.dtype == FA_DTYPE_F32 && a.g.nsp == 2 && a.g.stride >= a.g.ws &&
           a.g.ws <= 8 && a.g.S[0] >= 8 && a.d <= 64 && a.dv <= 64 &&
           a.g.P * (a.d > a.dv ? a.d : a.dv) * 4 < INT32_MAX - 64;
}

#if FA_WIN_PART != 1
thread_local int g_win_bwd_grid = 0;   // benchmark knob: the strip backward's workgroups (0: one per CU)
#endif
#if FA_WIN_PART != 2
thread_local int g_win_force_composed = 0;   // benchmark knob: 1 composed, 2 register-gather fused, 3 one-window row-shift (ws <= 7) / row-scatter, 4 four-window row-scatter, 5 one-window row-scatter, 6 two-window row-shift (the default for small launches), 10 eight-window strip (the default from kStripMin strips on); modes 7-9 (the rejected LDS-DMA and segment kernels) were removed in round 4
#endif

// The ONE place the fused-vs-composed decision is made: both the workspace
// query and the launcher call it, so they can never disagree.
static bool fused_ok(int dtype, const WindowGeom& g, int64_t d, int64_t dv) {
    return g_win_force_composed != 1 && (dtype == FA_DTYPE_BF16 || dtype == FA_DTYPE_F16) && g.T <= 64 && d <= 64 && dv <= 64 &&
           g.P * (d > dv ? d : dv) * 2 < INT32_MAX;
}

template <class T, int D, int DV>
static hipError_t launch_fused_dd(const WindowedArgs& a, const WinDev& g, void* out, bool direct, hipStream_t s) {
    const int64_t nw = a.g.L * a.batch;
    const dim3 grid((unsigned)((nw + 3) / 4)), blk(256);
    const float c = a.scale * kLog2e;
#define FA_FUSED(NKB, DIR) hipLaunchKernelGGL((win_fused<T, D, DV, NKB, DIR>), grid, blk, 0, s, (const T*)a.q, \
        (const T*)a.k, (const T*)a.v, (T*)out, a.l, a.m, g, (int)a.d, (int)a.dv, (int)a.batch, a.scale, c)
    if (a.g.T <= 32) { if (direct) FA_FUSED(1, true); else FA_FUSED(1, false); }
    else { if (direct) FA_FUSED(2, true); else FA_FUSED(2, false); }
#undef FA_FUSED
    return hipGetLastError();
}
// Row-staged kernels: 2-D, non-overlapping (direct store), ws <= 8, width % 8 == 0,
// 16-B aligned tensors.  ws <= 7: the one-window row-shift kernel at every size.
// ws = 8 (row scatter): four windows per workgroup from kRows4Min windows up, one
// window per workgroup below (where four per workgroup would leave CUs idle).
// Returns 0 (not eligible), 1 or 4.
constexpr int64_t kRows4Min = 1024;
static int rows_kind(const WindowedArgs& a) {
    if (g_win_force_composed == 1 || g_win_force_composed == 2) return 0;
    const bool shape = a.g.nsp == 2 && a.g.stride >= a.g.ws && a.g.ws <= 8 && a.g.S[0] % 8 == 0 &&
                       a.g.L * a.batch < INT32_MAX &&
                       ((uintptr_t)a.q & 15u) == 0 && ((uintptr_t)a.k & 15u) == 0 && ((uintptr_t)a.v & 15u) == 0;
    if (!shape) return 0;
    if (g_win_force_composed == 3 || g_win_force_composed >= 5) return 1;
    if (g_win_force_composed == 4) return 4;
    // ws <= 7: the row-shift kernel (two windows per workgroup) beats the
    // four-window row-scatter one at every batch size (128x128x64, ws 7:
    // B=1 6.8 vs 26.7 us, B=32 83-90 vs 123 us)
    if (a.g.ws <= 7) return 1;
    return a.g.L * a.batch >= kRows4Min ? 4 : 1;
}

// Strip kernel (win_strip) from this many workgroups on: below it the eight-window
// workgroups leave CUs idle and the two-window kernel's latency wins (configs[2] at
// B = 1 is 57 strips).
constexpr int64_t kStripMin = 256;

// Windows of the first strip: the smallest k0 in 1..8 with k0 * ws = pad (mod 8),
// so that every later strip starts on a 16-B chunk of y (8 otherwise).
static int strip_first(const WindowGeom& g) {
    for (int k0 = 1; k0 <= kStripW; ++k0)
        if (((k0 * g.ws - g.pad) % 8 + 8) % 8 == 0) return k0;
    return kStripW;
}
static int64_t strip_count(const WindowGeom& g, int k0) {
    return g.O[0] <= k0 ? 1 : 1 + (g.O[0] - k0 + kStripW - 1) / kStripW;
}

// Whether the forward picks the strip kernel for this geometry (no pointers).
static bool strip_applies(int dtype, const WindowGeom& g, int64_t d, int64_t dv, int64_t batch) {
    if ((dtype != FA_DTYPE_BF16 && dtype != FA_DTYPE_F16) || g.nsp != 2 || g.stride != g.ws || g.ws > 7 ||
        g.S[0] % 8 != 0 || d > 64 || dv > 64 || (g_win_force_composed != 0 && g_win_force_composed != 10))
        return false;
    const int64_t nsx = strip_count(g, strip_first(g)), nstrip = nsx * g.O[1] * batch;
    if (nstrip >= INT32_MAX || g.P * (d > dv ? d : dv) * 2 >= INT32_MAX || g.L * batch >= INT32_MAX) return false;
    return g_win_force_composed == 10 || nstrip >= kStripMin;
}

// Window counts between which the row-shift forward runs three windows per workgroup
// (768 threads) instead of two.
constexpr int64_t kRows3Min = 600, kRows3Max = 1000;

template <class T, int D, int DV>
static hipError_t launch_rows1_dd(const WindowedArgs& a, const WinDev& g, hipStream_t s) {
    if (a.g.ws <= 7 && g_win_force_composed != 5) {
        const int64_t nw = a.g.L * a.batch;
        if (strip_applies(a.dtype, a.g, a.d, a.dv, a.batch) && ((uintptr_t)a.y & 15u) == 0) {
            const int k0 = strip_first(a.g);
            const int64_t nsx = strip_count(a.g, k0), nstrip = nsx * a.g.O[1] * a.batch;
            hipLaunchKernelGGL((win_strip<T, D, DV>), dim3((unsigned)nstrip), dim3(512), 0, s, (const T*)a.q,
                               (const T*)a.k, (const T*)a.v, (T*)a.y, a.l, a.m, g, (int)a.d, (int)a.dv, (int)nsx, k0,
                               (int)nstrip, a.scale, a.scale * kLog2e);
            return hipGetLastError();
        }
        const bool two_img_ok = 2 * a.g.P * (a.d > a.dv ? a.d : a.dv) * 2 < INT32_MAX;
        // three windows per workgroup on mid-size grids (round 6, profiles/r06_win_nwin_ab.log,
        // configs[2] shape: B = 2 8.09-8.14 vs 8.82-8.95 us, B = 3 11.67 vs 11.41, B = 4 a tie, B = 1
        // 7.10 vs 6.23, r06_win_nwin_ab2.log; four windows
        // per workgroup slower at every B): fewer, longer workgroups than two windows give,
        // with one more window's row loads coalesced per (feature, row) line
        const bool three = g_win_force_composed == 12 ||
                           (g_win_force_composed == 0 && nw >= kRows3Min && nw < kRows3Max);
        if (three && two_img_ok) {
            hipLaunchKernelGGL((win_rows1s<T, D, DV, 3>), dim3((unsigned)((nw + 2) / 3)), dim3(768), 0, s,
                               (const T*)a.q, (const T*)a.k, (const T*)a.v, (T*)a.y, a.l, a.m, g, (int)a.d,
                               (int)a.dv, nw, a.scale, a.scale * kLog2e);
        } else if (g_win_force_composed != 3 && two_img_ok) {   // default: register-staged, two windows per workgroup
            hipLaunchKernelGGL((win_rows1s<T, D, DV, 2>), dim3((unsigned)((nw + 1) / 2)), dim3(512), 0, s,
                               (const T*)a.q, (const T*)a.k, (const T*)a.v, (T*)a.y, a.l, a.m, g, (int)a.d,
                               (int)a.dv, nw, a.scale, a.scale * kLog2e);
        } else {
            hipLaunchKernelGGL((win_rows1s<T, D, DV, 1>), dim3((unsigned)nw), dim3(256), 0, s,
                               (const T*)a.q, (const T*)a.k, (const T*)a.v, (T*)a.y, a.l, a.m, g, (int)a.d,
                               (int)a.dv, nw, a.scale, a.scale * kLog2e);
        }
        return hipGetLastError();
    }
    hipLaunchKernelGGL((win_rows1<T, D, DV>), dim3((unsigned)(a.g.L * a.batch)), dim3(256), 0, s, (const T*)a.q,
                       (const T*)a.k, (const T*)a.v, (T*)a.y, a.l, a.m, g, (int)a.d, (int)a.dv, a.scale,
                       a.scale * kLog2e);
    return hipGetLastError();
}

// d or dv in (64, 128] (bf16/f16, 2-D, non-overlapping, ws <= 7, width % 8 == 0,
// 16-B aligned): the one-window row-shift kernel at 128 features (50 KB of LDS,
// every wave runs two of the four 32-feature output chunks).  The workspace
// query cannot see the pointers, so it keeps the composed path's size.
static bool rows128_ok(const WindowedArgs& a) {
    return g_win_force_composed != 1 && g_win_force_composed != 2 && (a.dtype == FA_DTYPE_BF16 || a.dtype == FA_DTYPE_F16) &&
           (a.d > 64 || a.dv > 64) && a.d <= 128 && a.dv <= 128 && a.g.nsp == 2 && a.g.stride >= a.g.ws &&
           a.g.ws <= 7 && a.g.S[0] % 8 == 0 && ((uintptr_t)a.q & 15u) == 0 && ((uintptr_t)a.k & 15u) == 0 &&
           ((uintptr_t)a.v & 15u) == 0 && a.g.P * 128 * 2 < INT32_MAX &&
           a.g.L * a.batch < INT32_MAX;
}

template <class T, int D, int DV>
static hipError_t launch_rows_dd(const WindowedArgs& a, const WinDev& g, hipStream_t s) {
    const int ngx = (int)((a.g.O[0] + 3) / 4);
    const int64_t nwg = (int64_t)ngx * a.g.O[1] * a.batch;
    hipLaunchKernelGGL((win_rows<T, D, DV>), dim3((unsigned)nwg), dim3(256), 0, s, (const T*)a.q, (const T*)a.k,
                       (const T*)a.v, (T*)a.y, a.l, a.m, g, (int)a.d, (int)a.dv, (int)a.batch, ngx, a.scale,
                       a.scale * kLog2e);
    return hipGetLastError();
}

template <class T>
static hipError_t launch_fused(const WindowedArgs& a, const WinDev& g, void* out, bool direct, hipStream_t s) {
    const int Dc = a.d <= 32 ? 32 : 64, DVc = a.dv <= 32 ? 32 : 64;
    const int rk = direct && out == a.y ? rows_kind(a) : 0;
    if (rk == 4) {
        if (Dc == 32 && DVc == 32) return launch_rows_dd<T, 32, 32>(a, g, s);
        if (Dc == 32) return launch_rows_dd<T, 32, 64>(a, g, s);
        if (DVc == 32) return launch_rows_dd<T, 64, 32>(a, g, s);
        return launch_rows_dd<T, 64, 64>(a, g, s);
    }
    if (rk == 1) {
        if (Dc == 32 && DVc == 32) return launch_rows1_dd<T, 32, 32>(a, g, s);
        if (Dc == 32) return launch_rows1_dd<T, 32, 64>(a, g, s);
        if (DVc == 32) return launch_rows1_dd<T, 64, 32>(a, g, s);
        return launch_rows1_dd<T, 64, 64>(a, g, s);
    }
    if (Dc == 32 && DVc == 32) return launch_fused_dd<T, 32, 32>(a, g, out, direct, s);
    if (Dc == 32) return launch_fused_dd<T, 32, 64>(a, g, out, direct, s);
    if (DVc == 32) return launch_fused_dd<T, 64, 32>(a, g, out, direct, s);
    return launch_fused_dd<T, 64, 64>(a, g, out, direct, s);
}

static size_t esize(int dtype) { return dtype_size(dtype); }
static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

#if FA_WIN_PART != 2
size_t windowed_fwd_workspace(int dtype, const WindowGeom& g, int64_t d, int64_t dv, int64_t batch) {
    const size_t tok = (size_t)(g.T * g.L * batch);
    if (fused_ok(dtype, g, d, dv))   // direct (no overlap): none; overlap: the window outputs
        return g.stride >= g.ws ? 0 : align256(tok * dv * esize(dtype)) + 256;
    return align256(tok * d * esize(dtype)) * 2 + align256(tok * dv * esize(dtype)) * 2 +
           align256(dense_fwd_workspace(dtype, g.T, g.T, d, dv, g.L * batch)) + 256;
}
#endif

#if FA_WIN_PART != 2
size_t windowed_workspace(int dtype, const WindowGeom& g, int64_t d, int64_t dv, int64_t batch) {
    const size_t tok = (size_t)(g.T * g.L * batch);
    const size_t e = esize(dtype);
    return align256(tok * d * e) * 4 + align256(tok * dv * e) * 4 + align256(tok * 4) * 2 +
           align256(dense_bwd_workspace(dtype, g.T, g.T, d, dv, g.L * batch)) +
           align256(dense_fwd_workspace(dtype, g.T, g.T, d, dv, g.L * batch)) + 256;
}
#endif

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
    if (a.workspace_bytes < windowed_fwd_workspace(a.dtype, a.g, a.d, a.dv, a.batch)) {
        *why = "workspace smaller than fa_windowed_fwd_workspace()";
        return FA_ERR_WORKSPACE;
    }
    if constexpr (std::is_same<T, float>::value) {
        if (rows_f32_ok(a)) {
            const WinDev gd = to_dev(a.g);
            const dim3 grid((unsigned)(a.g.L * a.batch));
            const int Dc = a.d <= 32 ? 32 : 64, DVc = a.dv <= 32 ? 32 : 64;
#define FA_WF32(DD, DVV) hipLaunchKernelGGL((win_rows_f32<DD, DVV>), grid, dim3(256), 0, s, (const float*)a.q, \
                                            (const float*)a.k, (const float*)a.v, (float*)a.y, a.l, a.m, gd,    \
                                            (int)a.d, (int)a.dv, a.scale, a.scale * kLog2e)
            if (Dc == 32 && DVc == 32) FA_WF32(32, 32);
            else if (Dc == 32) FA_WF32(32, 64);
            else if (DVc == 32) FA_WF32(64, 32);
            else FA_WF32(64, 64);
#undef FA_WF32
            hipError_t e = hipGetLastError();
            if (e == hipSuccess && !fully_covered(a.g)) {
                const int64_t total = a.g.P * a.dv * a.batch;
                hipLaunchKernelGGL(win_nan_uncovered<float>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                                   (float*)a.y, (int)a.dv, total, gd);
                e = hipGetLastError();
            }
            if (e != hipSuccess) { *why = hipGetErrorString(e); return FA_ERR_HIP; }
            return FA_OK;
        }
    }
    if constexpr (sizeof(T) == 2) {
    if (rows128_ok(a)) {
        const int64_t nw = a.g.L * a.batch;
        hipLaunchKernelGGL((win_rows1s<T, 128, 128, 1>), dim3((unsigned)nw), dim3(256), 0, s, (const T*)a.q,
                           (const T*)a.k, (const T*)a.v, (T*)a.y, a.l, a.m, g, (int)a.d, (int)a.dv, nw, a.scale,
                           a.scale * kLog2e);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess && !fully_covered(a.g)) {
            const int64_t total = a.g.P * a.dv * a.batch;
            hipLaunchKernelGGL(win_nan_uncovered<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                               (T*)a.y, (int)a.dv, total, g);
            e = hipGetLastError();
        }
        if (e != hipSuccess) { *why = hipGetErrorString(e); return FA_ERR_HIP; }
        return FA_OK;
    }
    if (fused_ok(a.dtype, a.g, a.d, a.dv)) {
        hipError_t e;
        if (a.g.stride >= a.g.ws) {
            if ((e = launch_fused<T>(a, g, a.y, true, s)) != hipSuccess) { *why = hipGetErrorString(e); return FA_ERR_HIP; }
            if (!fully_covered(a.g)) {
                const int64_t total = a.g.P * a.dv * a.batch;
                hipLaunchKernelGGL(win_nan_uncovered<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                                   (T*)a.y, (int)a.dv, total, g);
                if ((e = hipGetLastError()) != hipSuccess) { *why = hipGetErrorString(e); return FA_ERR_HIP; }
            }
        } else {
            void* ow = (void*)(((uintptr_t)a.workspace + 255) & ~(uintptr_t)255);
            if ((e = launch_fused<T>(a, g, ow, false, s)) != hipSuccess ||
                (e = fold<T>(ow, a.y, (int)a.dv, a.batch, g, true, s)) != hipSuccess) {
                *why = hipGetErrorString(e);
                return FA_ERR_HIP;
            }
        }
        return FA_OK;
    }
    }
    const int64_t tok = a.g.T * a.g.L * a.batch;
    char* ws = (char*)(((uintptr_t)a.workspace + 255) & ~(uintptr_t)255);
    void* qw = ws;  ws += align256(tok * a.d * sizeof(T));
    void* kw = ws;  ws += align256(tok * a.d * sizeof(T));
    void* vw = ws;  ws += align256(tok * a.dv * sizeof(T));
    void* ow = ws;  ws += align256(tok * a.dv * sizeof(T));
    hipError_t e;
    if ((e = gather<T>(a.q, qw, (int)a.d, a.batch, g, false, s)) != hipSuccess ||
        (e = gather<T>(a.k, kw, (int)a.d, a.batch, g, false, s)) != hipSuccess ||
        (e = gather<T>(a.v, vw, (int)a.dv, a.batch, g, false, s)) != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    // the window batch has T = ws^k tokens (49 at ws 7): the dense workspace lets
    // the fast kernels run on padded key copies (or split-KV) instead of the generic one
    DenseArgs da{a.dtype, qw, kw, vw, ow, a.l, a.m, a.g.T, a.g.T, a.d, a.dv, a.g.L * a.batch, a.scale};
    da.scale64 = a.scale64;
    da.workspace = ws;
    da.workspace_bytes = dense_fwd_workspace(a.dtype, a.g.T, a.g.T, a.d, a.dv, a.g.L * a.batch);
    const int rc = launch_dense_fwd(da, s, why);
    if (rc != FA_OK) return rc;
    if ((e = fold<T>(ow, a.y, (int)a.dv, a.batch, g, true, s)) != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    return FA_OK;
}

#if FA_WIN_PART != 2
int launch_window(int dtype, const void* src, void* dst, const WindowGeom& geom, int64_t C, int64_t batch,
                  bool unwindow, hipStream_t s, const char** why) {
    if (!geom_fits(geom, C, C, batch) || C > INT32_MAX) {
        *why = "window geometry exceeds the 32-bit index range";
        return FA_ERR_UNSUPPORTED;
    }
    const WinDev g = to_dev(geom);
    const int64_t total = unwindow ? geom.P * C * batch : geom.T * C * geom.L * batch;
    if (total == 0) return FA_OK;
    if ((total + 255) / 256 > INT32_MAX) {
        *why = "grid too large";
        return FA_ERR_UNSUPPORTED;
    }
    hipError_t e;
    switch (dtype) {
        case FA_DTYPE_BF16: e = unwindow ? fold<bf16>(src, dst, (int)C, batch, g, false, s)
                                         : gather<bf16>(src, dst, (int)C, batch, g, false, s); break;
        case FA_DTYPE_F16: e = unwindow ? fold<f16>(src, dst, (int)C, batch, g, false, s)
                                        : gather<f16>(src, dst, (int)C, batch, g, false, s); break;
        case FA_DTYPE_F32: e = unwindow ? fold<float>(src, dst, (int)C, batch, g, false, s)
                                        : gather<float>(src, dst, (int)C, batch, g, false, s); break;
        case FA_DTYPE_F64: e = unwindow ? fold<double>(src, dst, (int)C, batch, g, false, s)
                                        : gather<double>(src, dst, (int)C, batch, g, false, s); break;
        default: *why = "unknown dtype"; return FA_ERR_INVALID_ARG;
    }
    if (e != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    return FA_OK;
}
#endif

#if FA_WIN_PART != 2
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
        case FA_DTYPE_F64: return windowed_fwd_typed<double>(a, s, why);
    }
    *why = "unknown dtype";
    return FA_ERR_INVALID_ARG;
}
#endif

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
    const size_t fws = dense_fwd_workspace(a.dtype, a.g.T, a.g.T, a.d, a.dv, nb);
    void* fwork = take(fws);
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
    da.scale64 = a.scale64;
    da.workspace = fwork;
    da.workspace_bytes = fws;
    int rc = launch_dense_fwd(da, s, why);
    if (rc != FA_OK) return rc;
    DenseBwdArgs ba{a.dtype, qw, kw, vw, ow, dyw, a.l, a.m, dqw, dkw, dvw, a.g.T, a.g.T, a.d, a.dv, nb,
                    a.scale, dwork, dws};
    ba.scale64 = a.scale64;
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

// fused windowed backward eligibility (the row-shift forward's shapes)
static bool bwd_rows_ok(const WindowedBwdArgs& a) {
    const bool al = ((uintptr_t)a.q & 15u) == 0 && ((uintptr_t)a.k & 15u) == 0 && ((uintptr_t)a.v & 15u) == 0 &&
                    ((uintptr_t)a.y & 15u) == 0 && ((uintptr_t)a.dy & 15u) == 0;
    return g_win_force_composed != 1 && (a.dtype == FA_DTYPE_BF16 || a.dtype == FA_DTYPE_F16) && a.g.nsp == 2 && a.g.stride >= a.g.ws &&
           a.g.ws <= 7 && a.g.S[0] % 8 == 0 && a.d <= 128 && a.dv <= 128 && al &&
           a.g.P * 128 * 2 < INT32_MAX && a.g.L * a.batch < INT32_MAX;
}

// The strip backward (win_bwd_strip): the forward strip kernel's shapes, d, dv <= 64,
// 16-B aligned gradients too; from kStripBwdMin strips on (or forced by mode 10).
constexpr int64_t kStripBwdMin = 256;
// The per-window backward pairs windows up to this many windows per CU (1.5: configs[2] at
// B = 1 is 361 windows on 256 CUs).
constexpr double kBwdPairMaxPerCu = 1.5;
static bool bwd_strip_ok(const WindowedBwdArgs& a) {
    auto al = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
    if ((a.dtype != FA_DTYPE_BF16 && a.dtype != FA_DTYPE_F16) || a.g.nsp != 2 || a.g.stride != a.g.ws || a.g.ws > 7 ||
        a.g.S[0] % 8 != 0 || a.d > 64 || a.dv > 64 || !al(a.q) || !al(a.k) || !al(a.v) || !al(a.dy) || !al(a.dq) ||
        !al(a.dk) || !al(a.dv_) || (g_win_force_composed != 0 && g_win_force_composed != 10))
        return false;
    const int64_t nstrip = strip_count(a.g, strip_first(a.g)) * a.g.O[1] * a.batch;
    if (nstrip >= INT32_MAX || a.g.P * 64 * 2 >= INT32_MAX || a.g.T * a.g.O[0] * 4 >= INT32_MAX) return false;
    return g_win_force_composed == 10 || nstrip >= kStripBwdMin;
}

template <class T>
static int windowed_bwd_rows(const WindowedBwdArgs& a, hipStream_t s, const char** why) {
    const WinDev g = to_dev(a.g);
    hipError_t e = hipSuccess;
    if (!fully_covered(a.g)) {   // pixels no window covers get zero gradient
        if ((e = hipMemsetAsync(a.dq, 0, (size_t)(a.g.P * a.d * a.batch) * sizeof(T), s)) != hipSuccess ||
            (e = hipMemsetAsync(a.dk, 0, (size_t)(a.g.P * a.d * a.batch) * sizeof(T), s)) != hipSuccess ||
            (e = hipMemsetAsync(a.dv_, 0, (size_t)(a.g.P * a.dv * a.batch) * sizeof(T), s)) != hipSuccess) {
            *why = hipGetErrorString(e);
            return FA_ERR_HIP;
        }
    }
    if (bwd_strip_ok(a)) {
        const int k0 = strip_first(a.g);
        const int64_t nsx = strip_count(a.g, k0), nstrip = nsx * a.g.O[1] * a.batch;
        // persistent: one workgroup per CU, strips dealt by 8 XCD-group counters in the workspace
        const int64_t cus = device_cus(s) > 0 ? device_cus(s) : 256;
        const int64_t gmax = g_win_bwd_grid > 0 ? (int64_t)g_win_bwd_grid : cus;
        const int64_t grid = nstrip < gmax ? nstrip : gmax;
        // the counters are atomic words: round their address up to 256 B as the dense
        // backward does (the header allows any workspace alignment; windowed_workspace
        // reserves the 256-B slack, and its buffers are far larger than the 512 B used)
        unsigned* const ctr = (unsigned*)(((uintptr_t)a.workspace + 255) & ~(uintptr_t)255);
        if (!a.workspace || a.workspace_bytes < (size_t)((char*)ctr - (char*)a.workspace) + 512) {
            *why = "workspace missing (the strip backward keeps its strip counters there)";
            return FA_ERR_WORKSPACE;
        }
        if ((e = hipMemsetAsync(ctr, 0, 512, s)) != hipSuccess) {   // 8 group counters, 64 B apart
            *why = hipGetErrorString(e);
            return FA_ERR_HIP;
        }
        // strip ends on 16-B chunks: every strip boundary (k0 aligns them) and the covered right end
        const int64_t xend = a.g.O[0] * a.g.ws - a.g.pad;
        const bool aligned = ((k0 * a.g.ws - a.g.pad) % 8 + 8) % 8 == 0 && (xend >= a.g.S[0] || xend % 8 == 0);
#define FA_BWD_STRIP2(DD, DVV, PA)                                                                              \
    hipLaunchKernelGGL((win_bwd_strip<T, DD, DVV, PA>), dim3((unsigned)grid), dim3(512), 0, s, (const T*)a.q,  \
                       (const T*)a.k, (const T*)a.v, (const T*)a.dy, a.l, a.m, (T*)a.dq, (T*)a.dk, (T*)a.dv_, g, \
                       (int)a.d, (int)a.dv, (int)nsx, k0, (int)nstrip, ctr, a.scale, a.scale * kLog2e)
#define FA_BWD_STRIP(DD, DVV)                           \
    do {                                                \
        if (aligned) FA_BWD_STRIP2(DD, DVV, false);     \
        else FA_BWD_STRIP2(DD, DVV, true);              \
    } while (0)
        const int Dc = a.d <= 32 ? 32 : 64, DVc = a.dv <= 32 ? 32 : 64;
        if (Dc == 32 && DVc == 32) FA_BWD_STRIP(32, 32);
        else if (Dc == 32) FA_BWD_STRIP(32, 64);
        else if (DVc == 32) FA_BWD_STRIP(64, 32);
        else FA_BWD_STRIP(64, 64);
#undef FA_BWD_STRIP
#undef FA_BWD_STRIP2
        if ((e = hipGetLastError()) != hipSuccess) {
            *why = hipGetErrorString(e);
            return FA_ERR_HIP;
        }
        return FA_OK;
    }
    const int64_t nw = a.g.L * a.batch;
    // two adjacent windows per workgroup (their row loads share lines, as in win_rows1s) while
    // the grid is at most about one round of CUs; one window per workgroup, several per CU,
    // above it (round 6)
    const int64_t cus = device_cus(s) > 0 ? device_cus(s) : 256;
    const bool pair = a.d <= 64 && a.dv <= 64 && 2 * a.g.P * (a.d > a.dv ? a.d : a.dv) * 2 < INT32_MAX &&
                      (g_win_force_composed == 13 || (g_win_force_composed == 0 && nw <= kBwdPairMaxPerCu * cus));
#define FA_BWD_ROWS(DD, DVV, NW)                                                                               \
    hipLaunchKernelGGL((win_bwd_rows<T, DD, DVV, NW>), dim3((unsigned)((nw + NW - 1) / NW)), dim3(256 * NW), 0, s,  \
                       (const T*)a.q, (const T*)a.k, (const T*)a.v, (const T*)a.y, (const T*)a.dy, a.l, a.m,       \
                       (T*)a.dq, (T*)a.dk, (T*)a.dv_, g, (int)a.d, (int)a.dv, (int)nw, a.scale, a.scale * kLog2e)
    const int Dc = a.d <= 32 ? 32 : 64, DVc = a.dv <= 32 ? 32 : 64;
    if (a.d > 64 || a.dv > 64) FA_BWD_ROWS(128, 128, 1);   // 83 KB of LDS: one workgroup per CU
    else if (pair) {
        if (Dc == 32 && DVc == 32) FA_BWD_ROWS(32, 32, 2);
        else if (Dc == 32) FA_BWD_ROWS(32, 64, 2);
        else if (DVc == 32) FA_BWD_ROWS(64, 32, 2);
        else FA_BWD_ROWS(64, 64, 2);
    }
    else if (Dc == 32 && DVc == 32) FA_BWD_ROWS(32, 32, 1);
    else if (Dc == 32) FA_BWD_ROWS(32, 64, 1);
    else if (DVc == 32) FA_BWD_ROWS(64, 32, 1);
    else FA_BWD_ROWS(64, 64, 1);
#undef FA_BWD_ROWS
    if ((e = hipGetLastError()) != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    return FA_OK;
}

static bool bwd_f32_ok(const WindowedBwdArgs& a) {
    return g_win_force_composed != 1 && a.dtype == FA_DTYPE_F32 && a.g.nsp == 2 && a.g.stride >= a.g.ws &&
           a.g.ws <= 8 && a.g.S[0] >= 8 && a.d <= 64 && a.dv <= 64 &&
           a.g.P * (a.d > a.dv ? a.d : a.dv) * 4 < INT32_MAX - 64;
}

static int windowed_bwd_f32(const WindowedBwdArgs& a, hipStream_t s, const char** why) {
    const WinDev g = to_dev(a.g);
    hipError_t e = hipSuccess;
    if (!fully_covered(a.g)) {
        if ((e = hipMemsetAsync(a.dq, 0, (size_t)(a.g.P * a.d * a.batch) * 4, s)) != hipSuccess ||
            (e = hipMemsetAsync(a.dk, 0, (size_t)(a.g.P * a.d * a.batch) * 4, s)) != hipSuccess ||
            (e = hipMemsetAsync(a.dv_, 0, (size_t)(a.g.P * a.dv * a.batch) * 4, s)) != hipSuccess) {
            *why = hipGetErrorString(e);
            return FA_ERR_HIP;
        }
    }
    const dim3 grid((unsigned)(a.g.L * a.batch));
    const int Dc = a.d <= 32 ? 32 : 64, DVc = a.dv <= 32 ? 32 : 64;
    const size_t lds = (size_t)(2 * Dc * 65 + 2 * DVc * 65 + 2 * 64 * 65 + 128) * 4;
#define FA_BWD_F32(DD, DVV)                                                                                     \
    (void)hipFuncSetAttribute((const void*)win_bwd_f32<DD, DVV>, hipFuncAttributeMaxDynamicSharedMemorySize,   \
                              (int)lds);                                                                        \
    hipLaunchKernelGGL((win_bwd_f32<DD, DVV>), grid, dim3(256), lds, s, (const float*)a.q, (const float*)a.k,   \
                       (const float*)a.v, (const float*)a.y, (const float*)a.dy, a.l, a.m, (float*)a.dq,        \
                       (float*)a.dk, (float*)a.dv_, g, (int)a.d, (int)a.dv, a.scale, a.scale * kLog2e)
    if (Dc == 32 && DVc == 32) { FA_BWD_F32(32, 32); }
    else if (Dc == 32) { FA_BWD_F32(32, 64); }
    else if (DVc == 32) { FA_BWD_F32(64, 32); }
    else { FA_BWD_F32(64, 64); }
#undef FA_BWD_F32
    if ((e = hipGetLastError()) != hipSuccess) {
        *why = hipGetErrorString(e);
        return FA_ERR_HIP;
    }
    return FA_OK;
}

#if FA_WIN_PART != 1
int launch_windowed_bwd(const WindowedBwdArgs& a, hipStream_t s, const char** why) {
    if (a.d > kMaxHeadDim || a.dv > kMaxHeadDim) {
        *why = "head dimension exceeds the compiled maximum (128)";
        return FA_ERR_UNSUPPORTED;
    }
    if (!geom_fits(a.g, a.d, a.dv, a.batch)) {
        *why = "windowed problem too large for 32-bit window indexing";
        return FA_ERR_UNSUPPORTED;
    }
    if (bwd_rows_ok(a)) {
        switch (a.dtype) {
            case FA_DTYPE_BF16: return windowed_bwd_rows<bf16>(a, s, why);
            case FA_DTYPE_F16: return windowed_bwd_rows<f16>(a, s, why);
        }
    }
    if (bwd_f32_ok(a)) return windowed_bwd_f32(a, s, why);
    switch (a.dtype) {
        case FA_DTYPE_BF16: return windowed_bwd_typed<bf16>(a, s, why);
        case FA_DTYPE_F16: return windowed_bwd_typed<f16>(a, s, why);
        case FA_DTYPE_F32: return windowed_bwd_typed<float>(a, s, why);
        case FA_DTYPE_F64: return windowed_bwd_typed<double>(a, s, why);
    }
    *why = "unknown dtype";
    return FA_ERR_INVALID_ARG;
}
#endif

}  // namespace fa
