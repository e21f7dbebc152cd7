// fa_fwd_pers.hip — dense flash-attention forward at head dims <= 64, persistent
// 8-wave workgroups (gfx950).  Same result, bit for bit, as dense_fwd_w8q2_wide
// (fa_fwd.hip) and so the reference dense_fa! (src/dense.jl:21-102, update :78-91):
// the per-tile arithmetic below is that kernel's, in the same order.  What changes is
// how the launch spends the time around it:
//
//  * grid = min(blocks, CUs) workgroups of 8 waves (two per SIMD); workgroup w walks
//    the 512-row query blocks w, w + G, w + 2G, ... (G = grid), so a CU keeps one
//    workgroup for the whole launch instead of retiring and re-dispatching one per
//    block.  The (b·h) slab of block id is id / nqb: with w = xcd_remap(blockIdx.x, G)
//    every block of a slab runs on one XCD (its L2 serves the slab's K/V re-reads).
//  * the K/V tile stream runs on across block seams: the last tile of block i
//    prefetches tile 0 of block i + G into the other LDS stage, one barrier per tile
//    as in the 8-wave kernel.
//  * each wave owns an 8-KB image [64 features][64 tokens] (128-B rows, 32-B blocks
//    XOR-ed with bit 1 of the row: conflict-free transposed reads).  It carries the
//    wave's Q in and its O out:
//      - at a seam the wave reads its Q fragments of block i + G from the image
//        (DMA'd there during block i), then writes block i's normalised O into it;
//      - in tiles 0..7 of block i + G it stores O(i) one 1-KiB piece per tile (16-B
//        row stores) and DMAs piece j of Q(i + 2G) over the piece it has just stored.
//    Nothing about the image is shared between waves, so the seam needs no barrier;
//    the Q DMA (buffer_load ... lds, inline asm, outside the compiler's wait model) is
//    waited for once per block, by the wave that issued it, before its Q reads.
//  * what a block launch paid per block — the prologue's Q / first-tile load burst,
//    the epilogue's O store tail, the workgroup re-dispatch — is paid once per launch.
//
// Conditions (launch_dense_fwd_pers): bf16 / f16, head-dim classes D, DV in {32, 64},
// the LDS-staged fast shapes (N % 8 == 0, Nk % 8 == 0, 16-B aligned tensors), whole
// pairs of 64-key tiles (Nk % 128 == 0, ldk == Nk) and at least 8 tiles per block.
#include "fa_common.h"
#include "fa_internal.h"
#include "fa_fwd_params.h"
#include "../../include/fa_hip.h"

namespace fa {

namespace {

__device__ __forceinline__ uint32_t pers_lds(const void* ptr) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)ptr;
}
__device__ __forceinline__ u32x4 pers_desc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)base;
    return u32x4{(unsigned)a, (unsigned)(a >> 32), bytes, 0x00020000u};
}
// One 1-KiB LDS-DMA piece (64 lanes x 16 B, lane-linear at the M0 base).  Inline asm:
// the compiler's wait model does not see it (a compiler-issued LDS-DMA would make it
// wait for the piece before the next LDS read of the tile loop); the issuing wave waits
// for it by its own s_waitcnt vmcnt(0) before reading the image.  The whole offset goes
// in voffset: the descriptor's range check does not cover soffset.
__device__ __forceinline__ void pers_dma(const u32x4& desc, uint32_t lds_base, int voff, int soff) {
    // s_nop 4: five wait states after a VALU write of the descriptor SGPRs (a v_readlane
    // restore, invisible to the hazard recognizer across the asm boundary)
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" : : "v"(voff), "s"(desc), "s"(soff), "{m0}"(lds_base) : "memory");
}

}  // namespace

template <class T, int D, int DV>
__global__ __launch_bounds__(512, 1) void dense_fwd_pers(FwdParams p) {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    constexpr int NW = 8, NTH = 64 * NW, NQB = 2, BN = 64, BM = 32 * NW * NQB, NKB = BN / 32;
    constexpr int KROW = BN * 2, VROW = BN * 2 + 16;            // the 8-wave kernel's stage images
    constexpr int KBYTES = D * KROW, VBYTES = DV * VROW, STAGE = KBYTES + VBYTES;
    constexpr int CPR = BN / 8, KTOT = D * CPR, VTOT = DV * CPR;
    constexpr int KCH = (KTOT + NTH - 1) / NTH, VCH = (VTOT + NTH - 1) / NTH;
    static_assert(KTOT % NTH == 0 || KTOT < NTH, "tile split");
    static_assert(VTOT % NTH == 0 || VTOT < NTH, "tile split");
    constexpr int FR = D > DV ? D : DV;
    constexpr int WIMG = FR * 128;                                // per-wave Q / O image: [FR][64 tokens]
    constexpr int QP = D / 8, OP = DV / 8;                        // 1-KiB pieces of the Q / O image
    constexpr int IMGOFF = (2 * STAGE + 16 + 255) & ~255;         // +16 past the stages: dump slot
    __shared__ __attribute__((aligned(256))) char smem[IMGOFF + NW * WIMG];
    // 32-B block XOR of image row f (K stage and wave image alike): bit 1 of f
    auto swz = [](int f) { return ((f >> 1) & 1) << 1; };

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int N = p.N, d = p.d, dv = p.dv, ldk = p.ldk, nqb = p.nqb, nblk = p.total_wg;
    const int G = gridDim.x;
    const int NT = p.Nk / BN;   // even (launch_dense_fwd_pers)
    char* const wimg = smem + IMGOFF + wave * WIMG;
    const uint32_t wimg_lds = pers_lds(wimg);
    const float c = p.scale_log2;
    const float thr_raw = p.rescale_log2 / c;

    // 16-B slot `lane` of image piece `it`: feature row 8 it + (lane >> 3), physical
    // chunk lane & 7 → logical byte lb (= 2 x token).  qlane = its byte offset in a
    // slab at token 0, piece 0; both the Q DMA and the O stores use it.
    int qlane, qtok;
    {
        const int fl = lane >> 3, pb = (lane & 7) * 16;
        const int lb = (((pb >> 5) ^ swz(fl)) << 5) | (pb & 31);
        qlane = fl * N * 2 + lb;
        qtok = lb >> 1;
    }
    const int g = lane >> 4, kh = g & 1, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
    int koff[NKB];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) koff[kb] = (8 * h + qq) * KROW + (((kb * 2 + kh) ^ swz(qq)) * 32) + 8 * sig;
    const int voff = r * VROW + 16 * h;

    int kgo[KCH], kso[KCH], vgo[VCH], vso[VCH];
    const bool kact = KTOT >= NTH || tid < KTOT, vact = VTOT >= NTH || tid < VTOT;
#pragma unroll
    for (int it = 0; it < KCH; ++it) {
        const int ch = tid + NTH * it, f = ch / CPR, pc = ch % CPR;
        kgo[it] = kact ? (f * ldk + pc * 8) * 2 : 0x7FFFFFF0;
        kso[it] = kact ? f * KROW + (((pc >> 1) ^ swz(f)) * 32) + (pc & 1) * 16 : 2 * STAGE;
    }
#pragma unroll
    for (int it = 0; it < VCH; ++it) {
        const int ch = tid + NTH * it, f = ch / CPR, pc = ch % CPR;
        vgo[it] = vact ? (f * ldk + pc * 8) * 2 : 0x7FFFFFF0;
        vso[it] = vact ? f * VROW + pc * 16 : 2 * STAGE - KBYTES;
    }

    // slab descriptors of block id (blocks past the end: slab 0, never read)
    auto slab_of = [&](int id) __attribute__((always_inline)) { return id < nblk ? id / nqb : 0; };
    auto krs_of = [&](int id) __attribute__((always_inline)) {
        return slab_rsrc((const T*)p.K + (int64_t)slab_of(id) * ldk * d, (uint32_t)(ldk * d * (int)sizeof(T)));
    };
    auto vrs_of = [&](int id) __attribute__((always_inline)) {
        return slab_rsrc((const T*)p.V + (int64_t)slab_of(id) * ldk * dv, (uint32_t)(ldk * dv * (int)sizeof(T)));
    };
    auto qdesc_of = [&](int id) __attribute__((always_inline)) {
        return pers_desc((const T*)p.Q + (int64_t)slab_of(id) * N * d, id < nblk ? (uint32_t)(N * d * (int)sizeof(T)) : 0u);
    };
    // first token of this wave's 64 rows in block id
    auto q0_of = [&](int id) __attribute__((always_inline)) { return (id % nqb) * BM + wave * 64; };

    u32x4 kreg[KCH], vreg[VCH];
    auto gload = [&](const __amdgpu_buffer_rsrc_t& krs, const __amdgpu_buffer_rsrc_t& vrs, int j) __attribute__((always_inline)) {
        const int kb0 = j * BN * 2;
#pragma unroll
        for (int it = 0; it < KCH; ++it) kreg[it] = __builtin_amdgcn_raw_buffer_load_b128(krs, kgo[it] + kb0, 0, 0);
#pragma unroll
        for (int it = 0; it < VCH; ++it) vreg[it] = __builtin_amdgcn_raw_buffer_load_b128(vrs, vgo[it] + kb0, 0, 0);
    };
    auto lstore = [&](char* buf) __attribute__((always_inline)) {
#pragma unroll
        for (int it = 0; it < KCH; ++it) *(u32x4*)((kact ? buf : smem) + kso[it]) = kreg[it];
#pragma unroll
        for (int it = 0; it < VCH; ++it) *(u32x4*)((vact ? buf : smem) + KBYTES + vso[it]) = vreg[it];
    };

    F8 qf[NQB][D / 16];
    // this wave's Q fragments from its image (transposed reads, 4 feature rows each)
    // (the lane id re-enters opaque in the seam and side work: their lane-dependent
    // addresses are recomputed there instead of hoisted out of the block loop, where
    // they would hold VGPRs through every tile)
    auto opaque_lane = [&]() __attribute__((always_inline)) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        return ln;
    };
    auto read_qf = [&]() __attribute__((always_inline)) {
        const int ln = opaque_lane();
        const int lh = ln >> 5, lkh = (ln >> 4) & 1, lqq = (ln >> 2) & 3, lpp = ln & 3;
#pragma unroll
        for (int u = 0; u < NQB; ++u)
#pragma unroll
            for (int s = 0; s < D / 16; ++s) {
                const int f = 16 * s + 8 * lh + lqq, blk = 2 * u + lkh;
                const char* a = wimg + f * 128 + ((blk ^ swz(f)) << 5) + 8 * lpp;
                const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(a));
                const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(a + 4 * 128));
                qf[u][s] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
            }
    };

    f32x16 oacc[NQB][DV / 32];
    float m_used[NQB], m_true[NQB], l_run[NQB];

    // one 64-key tile: the 8-wave kernel's compute (dense_fwd_tiled, whole tiles)
    auto compute = [&](const char* klds, const char* vlds) __attribute__((always_inline)) {
        f32x16 sacc[NQB][NKB];
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
#pragma unroll
            for (int u = 0; u < NQB; ++u)
#pragma unroll
                for (int x = 0; x < 16; ++x) sacc[u][kb][x] = 0.0f;
#pragma unroll
            for (int s = 0; s < D / 16; ++s) {
                const char* a = klds + koff[kb] + 16 * s * KROW;
                const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(a));
                const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(a + 4 * KROW));
                const F8 af = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
                for (int u = 0; u < NQB; ++u) sacc[u][kb] = mfma32x32x16(af, qf[u][s], sacc[u][kb]);
            }
        }
        F8 pf[NQB][NKB][2];
#pragma unroll
        for (int u = 0; u < NQB; ++u) {
            const float mt = lane_max<NKB>(sacc[u]);
            m_true[u] = vmax(m_true[u], mt);
            if (__builtin_amdgcn_ballot_w64(mt > m_used[u] + thr_raw) != 0) {
                const float m_new = fmaxf(m_used[u], swap_halves_max(mt));
                const float alpha = exp2_fast((m_used[u] - m_new) * c);
                l_run[u] *= alpha;
#pragma unroll
                for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                    for (int x = 0; x < 16; ++x) oacc[u][cb][x] *= alpha;
                m_used[u] = m_new;
            }
            const float mc = m_used[u] * c;
            float ps[4];
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int x = 0; x < 16; ++x) {
                    const float pv = exp2_fast(fmaf(sacc[u][kb][x], c, -mc));
                    if (kb == 0 && x < 4) ps[x] = pv; else ps[x & 3] += pv;
                    pf[u][kb][x >> 3][x & 7] = (T)pv;
                }
            l_run[u] += (ps[0] + ps[1]) + (ps[2] + ps[3]);
        }
#pragma unroll
        for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const F8 va = *(const F8*)(vlds + voff + cb * 32 * VROW + (kb * 32 + 16 * s) * 2);
#pragma unroll
                    for (int u = 0; u < NQB; ++u) oacc[u][cb] = mfma32x32x16(va, pf[u][kb][s], oacc[u][cb]);
                }
    };

    char* const buf0 = smem;
    char* const buf1 = smem + STAGE;

    // ---- prologue: the first block's Q (this wave's image) and K/V tile 0 ----
    int id = xcd_remap(blockIdx.x, G);
    {
        const u32x4 qd = qdesc_of(id);
        const int q0 = q0_of(id);
#pragma unroll
        for (int it = 0; it < QP; ++it) pers_dma(qd, wimg_lds + it * 1024, qlane + it * 8 * N * 2 + q0 * 2, 0);
    }
    __amdgpu_buffer_rsrc_t krs = krs_of(id), vrs = vrs_of(id);
    gload(krs, vrs, 0);
    lstore(buf0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's Q pieces landed
    __syncthreads();
    read_qf();

    // O of the previous block waiting in the image (stored in tiles 0..OP-1)
    bool have_prev = false;
    __amdgpu_buffer_rsrc_t ors_prev = krs;
    int q0_prev = 0;
    for (;;) {
        const int b = id / nqb, qb = id - b * nqb;
        const bool more = id + G < nblk;
        const int idn = id + G;
        const __amdgpu_buffer_rsrc_t krs_n = krs_of(idn), vrs_n = vrs_of(idn);
        const u32x4 qd_n = qdesc_of(idn);
        const int q0_n = q0_of(idn);
#pragma unroll
        for (int u = 0; u < NQB; ++u) {
            m_used[u] = kNegInf;
            m_true[u] = kNegInf;
            l_run[u] = 0.0f;
#pragma unroll
            for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                for (int x = 0; x < 16; ++x) oacc[u][cb][x] = 0.0f;
        }
        // tile j's side work: piece j of the previous block's O out, then piece j of the
        // next block's Q in over it (the O read has returned: the store consumed it)
        auto side = [&](int j) __attribute__((always_inline)) {
            if (j < OP && have_prev) {
                const int ln = opaque_lane();
                const u32x4 v4 = *(const u32x4*)(wimg + j * 1024 + ln * 16);
                const int f = 8 * j + (ln >> 3), q = q0_prev + qtok;
                const int off = (f < dv && q < N) ? qlane + j * 8 * N * 2 + q0_prev * 2 : 0x7FFFFFF0;
                __builtin_amdgcn_raw_buffer_store_b128(v4, ors_prev, off, 0, 0);
            }
            if (j < QP && more) pers_dma(qd_n, wimg_lds + j * 1024, qlane + j * 8 * N * 2 + q0_n * 2, 0);
        };
        for (int j = 0; j < NT; j += 2) {
            gload(krs, vrs, j + 1);
            side(j);
            compute(buf0, buf0 + KBYTES);
            lstore(buf1);
            __syncthreads();
            // the next tile: this block's, or tile 0 of the next block (of this block
            // again after the last one: loaded, never used)
            if (j + 2 < NT) gload(krs, vrs, j + 2);
            else gload(krs_n, vrs_n, 0);
            side(j + 1);
            compute(buf1, buf1 + KBYTES);
            lstore(buf0);
            __syncthreads();
        }

        // ---- block seam: l, m out; the next block's Q fragments; O into the image ----
        if (more) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's Q(next) pieces landed
            read_qf();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // read before the O writes below
        }
        float inv[NQB];
#pragma unroll
        for (int u = 0; u < NQB; ++u) {
            const float mt = swap_halves_max(m_true[u]);
            const float lt = swap_halves_sum(l_run[u]);
            inv[u] = 1.0f / lt;
            const int qi = qb * BM + (wave * NQB + u) * 32 + r;
            if (qi < N && h == 0) {
                p.m[(int64_t)b * N + qi] = mt * p.scale;
                p.l[(int64_t)b * N + qi] = lt * exp2_fast((m_used[u] - mt) * c);
            }
        }
        const int lno = opaque_lane(), lr = lno & 31, lh = lno >> 5;
#pragma unroll
        for (int u = 0; u < NQB; ++u)
#pragma unroll
            for (int cb = 0; cb < DV / 32; ++cb)
#pragma unroll
                for (int x = 0; x < 16; ++x) {
                    const int f = cb * 32 + acc_row(x, lh), tb = (u * 32 + lr) * 2;
                    *(T*)(wimg + f * 128 + (((tb >> 5) ^ swz(f)) << 5) + (tb & 31)) = (T)(oacc[u][cb][x] * inv[u]);
                }
        const __amdgpu_buffer_rsrc_t ors = slab_rsrc((T*)p.O + (int64_t)b * N * dv, (uint32_t)(N * dv * (int)sizeof(T)));
        if (!more) {   // the last block: its O leaves now
#pragma unroll
            for (int it = 0; it < OP; ++it) {
                const u32x4 v4 = *(const u32x4*)(wimg + it * 1024 + lane * 16);
                const int f = 8 * it + (lane >> 3), q = q0_of(id) + qtok;
                const int off = (f < dv && q < N) ? qlane + it * 8 * N * 2 + q0_of(id) * 2 : 0x7FFFFFF0;
                __builtin_amdgcn_raw_buffer_store_b128(v4, ors, off, 0, 0);
            }
            break;
        }
        have_prev = true;
        ors_prev = ors;
        q0_prev = q0_of(id);
        id = idn;
        krs = krs_n;
        vrs = vrs_n;
    }
}

// Launch on the persistent grid; returns false when the shape is not this kernel's.
bool launch_dense_fwd_pers(const FwdParams& p, int Dc, int DVc, int dtype, hipStream_t s, hipError_t* err) {
    if (!p.fast || !p.wide || p.nsplit > 1 || Dc > 64 || DVc > 64) return false;
    if (p.Nk % 128 != 0 || p.ldk != p.Nk || p.Nk / 64 < 8) return false;
    const int cus = device_cus(s);
    if (cus <= 0) return false;
    FwdParams q = p;
    q.nqb = (p.N + 511) / 512;
    const int64_t nblk = (int64_t)q.nqb * p.batch;
    if (nblk > INT32_MAX / 2) return false;
    q.total_wg = (int)nblk;
    const dim3 grid((unsigned)(nblk < cus ? nblk : cus)), blk(512);
#define FA_PERS_LAUNCH(TT)                                                                                \
    if (Dc == 64 && DVc == 64) hipLaunchKernelGGL((dense_fwd_pers<TT, 64, 64>), grid, blk, 0, s, q);     \
    else if (Dc == 64) hipLaunchKernelGGL((dense_fwd_pers<TT, 64, 32>), grid, blk, 0, s, q);             \
    else if (DVc == 64) hipLaunchKernelGGL((dense_fwd_pers<TT, 32, 64>), grid, blk, 0, s, q);            \
    else hipLaunchKernelGGL((dense_fwd_pers<TT, 32, 32>), grid, blk, 0, s, q);
    if (dtype == FA_DTYPE_BF16) { FA_PERS_LAUNCH(bf16) }
    else if (dtype == FA_DTYPE_F16) { FA_PERS_LAUNCH(f16) }
    else return false;
#undef FA_PERS_LAUNCH
    *err = hipGetLastError();
    return true;
}

}  // namespace fa
