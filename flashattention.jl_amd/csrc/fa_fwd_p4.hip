// fa_fwd_p4.hip — dense flash-attention forward, one wave per SIMD, persistent
// workgroups (gfx950).  Same result as dense_fwd_tiled (fa_fwd.hip) and the
// reference dense_fa! (src/dense.jl:21-102, update :78-91), built for a different
// machine use:
//
//  * a workgroup is 4 waves (one per SIMD, up to 512 registers each) and stays
//    resident: grid = min(blocks, CUs), workgroup w walks the 256-row query blocks
//    w, w + G, w + 2G, ... (G = grid).  Each wave owns two 32-row query blocks.
//  * K and V tiles (64 keys) arrive by LDS-DMA (buffer_load ... lds, issued by inline
//    asm and counted by hand) into rings of 3 (K) and 2 (V) slots, K three tiles
//    ahead and V one tile ahead; the stream continues across query-block seams, and
//    the next block's Q is DMA'd into its image while the current block runs.
//  * the loop is software-pipelined inside the wave.  Tile j runs two phases:
//      A(j): Sᵀ(j+1) = K(j+1)·Qᵀ (MFMA)   ∥ softmax of tile j, query block 1
//      B(j): Oᵀ += Vᵀ(j)·Pᵀ(j)   (MFMA)   ∥ row max of tile j+1 and the softmax of
//                                             tile j+1, query block 0 (speculative on
//                                             the running max), DMA issue
//    with one barrier per tile between A and B.  The lazy-rescale decision for tile
//    j+1 (a wave-wide ballot) is taken after B(j); a rescale of query block 0
//    recomputes its speculative P.  The instruction order inside a phase is set
//    here, not by the scheduler: each MFMA is followed by its share of the softmax
//    and of the next LDS reads, and sched_barrier(0) fences every such group.
//  * the MFMAs are inline asm: O and Q live in AGPRs, the score tiles in VGPRs (the
//    compiler would put every accumulator of a 512-register kernel in AGPRs and copy
//    each score out for the softmax).  The hazard recognizer does not see into asm,
//    so every VALU read of an asm MFMA result sits behind p4_mfma_drain().
//  * layouts are the dense kernels': K image [D][64] 128-B rows with the 32-B chunk
//    XOR (conflict-free ds_read_b64_tr_b16), V image [DV][64] 128-B rows with the
//    16-B chunk XOR (f>>1)&7 (conflict-free ds_read_b128 for the 32x32x16 A operand,
//    and DMA-friendly: no padding), Q image [D][256] through qo-swizzled 32-B blocks.
//  * O leaves per wave through a 4-KB staging image as 16-B row stores.
//
// Taken for the LDS-staged fast shapes (bf16/f16, Nk % 8 == 0, N % 8 == 0, 16-B
// aligned tensors), d = dv = 64 or 128, at least one block per CU and enough key
// tiles per block for the Q prefetch (launch_dense_fwd_p4).
#include "fa_common.h"
#include "fa_internal.h"
#include "fa_fwd_params.h"
#include "../../include/fa_hip.h"

#ifndef FA_P4_STAMP
#define FA_P4_STAMP(k)
#endif

namespace fa {

namespace {

constexpr int kP4Rows = 256;   // query rows per block: 4 waves x 2 x 32
constexpr int kP4KS = 3;       // K ring slots (K(t+3) issued in phase B(t))
constexpr int kP4VS = 2;       // V ring slots (V(t+1) issued in phase B(t))

__device__ __forceinline__ uint32_t p4_lds(const void* ptr) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)ptr;
}
__device__ __forceinline__ u32x4 p4_desc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)base;
    return u32x4{(unsigned)a, (unsigned)(a >> 32), bytes, 0x00020000u};
}
// One 1-KiB LDS-DMA piece (64 lanes x 16 B, lane-linear at the M0 base).  Hidden
// from the compiler's waitcnt model: the kernel waits for it in p4_wait_all_barrier().
__device__ __forceinline__ void p4_dma(const u32x4& desc, uint32_t lds_base, int voff, int soff) {
    asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" : : "v"(voff), "s"(desc), "s"(soff), "{m0}"(lds_base) : "memory");
}
// Every vector-memory operation of this wave retired, then the workgroup barrier (the
// DMA'd tiles of all four waves are visible after it), then >= 18 wait states: the
// asm MFMAs before the barrier have retired before any VALU reads their results.
__device__ __forceinline__ void p4_wait_all_barrier() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
}
// >= 18 wait states after the last asm MFMA before VALU touches its accumulator
__device__ __forceinline__ void p4_mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }
__device__ __forceinline__ void p4_fence() { __builtin_amdgcn_sched_barrier(0); }

// Oᵀ += A·B with the accumulator in AGPRs
__device__ __forceinline__ void p4_mfma_acc(f32x16& acc, const bf16x8& a, const bf16x8& b) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void p4_mfma_acc(f32x16& acc, const f16x8& a, const f16x8& b) {
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// Sᵀ (+)= K·Qᵀ with Qᵀ in AGPRs and the score accumulator in VGPRs
__device__ __forceinline__ void p4_mfma_s(f32x16& acc, const bf16x8& a, const bf16x8& q, bool first) {
    if (first) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(q));
    else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(q));
}
__device__ __forceinline__ void p4_mfma_s(f32x16& acc, const f16x8& a, const f16x8& q, bool first) {
    if (first) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(q));
    else asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(q));
}

template <class T, int D, int DV>
struct P4 {
    typedef typename Frag8<T>::type F8;
    typedef typename Frag8<T>::half F4;
    static constexpr int KSLOT = D * 128, VSLOT = DV * 128;
    static constexpr int QROWB = kP4Rows * 2;              // Q image row: 256 tokens
    static constexpr int QIMG = D * QROWB;
    static constexpr int OST = 32 * 128;                   // per-wave O staging image: 32 features x 64 tokens
    static constexpr int KOFF = 0;
    static constexpr int VOFF = KOFF + kP4KS * KSLOT;
    static constexpr int QOFF = VOFF + kP4VS * VSLOT;
    static constexpr int OOFF = QOFF + QIMG;
    static constexpr int LDSB = OOFF + 4 * OST;
    static constexpr int KP = D / 32;                      // K DMA pieces per wave and tile
    static constexpr int VP = DV / 32;                     // V DMA pieces per wave and tile
    static constexpr int QP = D / 8;                       // Q DMA pieces per wave and block
    static constexpr int NCB = DV / 32;                    // 32-feature output blocks
    static constexpr int NKS = D / 16;                     // k-steps of the score product
    static constexpr int NKQ = 2 * NKS;                    // (key block, k-step) pairs: K fragments per tile
    static constexpr int NVQ = 4 * NCB;                    // (output block, key block, k-step): V fragments per tile
    static_assert(LDSB <= 163840, "LDS budget");
};

// Q image position of logical byte `lb` (= 2 x token) of feature row f (the qo_at of
// dense_fwd_tiled at 256 rows): 32-B blocks XOR (f & 3) | (bit 2 of f) << 2.
__device__ __forceinline__ int p4_qpos(int f, int lb) {
    const int X = (f & 3) | (((f >> 2) & 1) << 2);
    return f * (kP4Rows * 2) + (((lb >> 5) ^ X) << 5) + (lb & 31);
}

// Register fences: an empty volatile asm that "redefines" a value pins the work that
// produces it before that point and the work that consumes it after (volatile asm
// keeps its order against the MFMA and DMA asm).  Fencing a private value costs
// nothing; work whose inputs are shared (the scores) is pinned through a scalar
// operand fenced at its slot (an s_mov, no vector issue).
__device__ __forceinline__ void p4_pin(float& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ float p4_pin_s(float x) { asm volatile("" : "+s"(x)); return x; }
template <class V> __device__ __forceinline__ void p4_pin_vec(V& x) { asm volatile("" : "+v"(x)); }

// The softmax of one query block's 64 scores per lane pair (32 per lane), cut into
// 16 chunks of two scores, each in two parts: part 0 = two FMAs (c·s − c·m) and two
// exponentials, part 1 = the two sum adds and the bf16/f16 pack.
template <class T>
struct SoftmaxQB {
    typedef typename Frag8<T>::type F8;
    float mc, c;
    float e[2][2];   // exponentials of chunk c in e[c & 1]
    float ps[4];
    __device__ __forceinline__ void part0(const f32x16 (&S)[2], int ch) {
        const int kb = ch >> 3, x = 2 * (ch & 7);
        float* ee = e[ch & 1];
        const float cs = p4_pin_s(c);   // c is uniform (SGPR); the running max is per lane
        ee[0] = exp2_fast(fmaf(S[kb][x], cs, -mc));
        ee[1] = exp2_fast(fmaf(S[kb][x + 1], cs, -mc));
        p4_pin(ee[0]);
        p4_pin(ee[1]);
    }
    __device__ __forceinline__ void part1(F8 (&P)[2][2], int ch) {
        const int kb = ch >> 3, x = 2 * (ch & 7);
        float* ee = e[ch & 1];
        p4_pin(ee[0]);
        p4_pin(ee[1]);
        if (ch < 2) {   // the first four exponentials seed the partial sums
            ps[x & 3] = ee[0];
            ps[(x + 1) & 3] = ee[1];
        } else {
            ps[x & 3] += ee[0];
            ps[(x + 1) & 3] += ee[1];
        }
        p4_pin(ps[x & 3]);
        p4_pin(ps[(x + 1) & 3]);
        P[kb][x >> 3][x & 7] = (T)ee[0];
        P[kb][x >> 3][(x & 7) + 1] = (T)ee[1];
        if ((x & 7) == 6) p4_pin_vec(P[kb][x >> 3]);
    }
    // part k of 32 in issue order: part0 of chunk 0, then (part0 of chunk c+1, part1
    // of chunk c) pairs, then part1 of chunk 15 — an exponential's consumer never
    // follows it directly (the trans-use wait state)
    __device__ __forceinline__ void part(const f32x16 (&S)[2], F8 (&P)[2][2], int k) {
        if (k == 0) part0(S, 0);
        else if (k == 31) part1(P, 15);
        else if (k & 1) part0(S, (k + 1) >> 1);
        else part1(P, (k >> 1) - 1);
    }
    __device__ __forceinline__ float sum() const { return (ps[0] + ps[1]) + (ps[2] + ps[3]); }
};

// Lane maximum of one query block's 32 scores in 18 steps: four v_maximum3 chains
// seeded with two scores each (steps 0-3), twelve chain steps of two scores, then
// the combine (steps 16, 17 leave the result in mt).
struct MaxQB {
    float a[4], t, mt;
    static constexpr int NOPS = 18;
    __device__ __forceinline__ void op(const f32x16 (&S)[2], int m) {
        auto v = [&](int k) { return S[k >> 4][k & 15]; };
        if (m < 4) {
            a[m] = vmax3(v(2 * m), v(2 * m + 1), p4_pin_s(kNegInf));
            p4_pin(a[m]);
        } else if (m < 16) {
            const int k = 8 + 2 * (m - 4), cc = m & 3;
            p4_pin(a[cc]);
            a[cc] = vmax3(a[cc], v(k), v(k + 1));
            p4_pin(a[cc]);
        } else if (m == 16) {
            t = vmax3(a[0], a[1], a[2]);
            p4_pin(t);
        } else {
            mt = vmax(t, a[3]);
        }
    }
};

}  // namespace

template <class T, int D, int DV>
__global__ __launch_bounds__(256, 1) void dense_fwd_p4(FwdParams p) {
    typedef P4<T, D, DV> C;
    typedef typename C::F8 F8;
    typedef typename C::F4 F4;
    __shared__ __attribute__((aligned(1024))) char smem[C::LDSB];
    char* const kring = smem + C::KOFF;
    char* const vring = smem + C::VOFF;
    char* const qimg = smem + C::QOFF;
    char* const ost = smem + C::OOFF;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: LDS-DMA bases are scalar
    const int r = lane & 31, h = lane >> 5;
    const int g = lane >> 4, kh = g & 1, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
    const int sig = (pp == 1) ? 2 : (pp == 2) ? 1 : pp;
    const int N = p.N, Nk = p.Nk, d = p.d, dv = p.dv, ldk = p.ldk, nqb = p.nqb;
    const int nblk = p.total_wg;
    const int G = gridDim.x;
    const int w = xcd_remap(blockIdx.x, G);
    const int NT = Nk >> 6;   // Nk % 64 == 0 (launch_dense_fwd_p4)
    const float c = p.scale_log2;
    const float thr_raw = p.rescale_log2 / c;
    const uint32_t lds0 = p4_lds(smem);

    // ---- per-lane constants ----
    // transposed K reads: lane 4q+pp of 16-lane group g supplies feature row q and the
    // 4-key chunk sig(pp) (key order permuted so each lane's 8 P values are 8
    // consecutive keys: the Vᵀ fragment is then one 16-B read)
    int koff[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) koff[kb] = (8 * h + qq) * 128 + (((kb * 2 + kh) ^ (((qq >> 1) & 1) << 1)) * 32) + 8 * sig;
    // Vᵀ row reads: row r (+32 cb), logical 16-B chunk 4kb + 2s + h, XOR (r >> 1) & 7
    int voff[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) voff[kb][s] = r * 128 + (((4 * kb + 2 * s + h) ^ ((r >> 1) & 7)) << 4);
    // DMA pieces: lane-linear 16-B slots of a 1-KiB piece → (feature row, key chunk);
    // the per-lane byte offset within the slab at key 0 (the tile's key offset goes in
    // the scalar soffset)
    int kgo[C::KP], vgo[C::VP];
#pragma unroll
    for (int it = 0; it < C::KP; ++it) {
        const int P = (it * 4 + wave) * 1024 + lane * 16, f = P >> 7;
        const int pc = ((((P >> 5) & 3) ^ (((f >> 1) & 1) << 1)) << 1) | ((P >> 4) & 1);
        kgo[it] = (f * ldk + pc * 8) * 2;
    }
#pragma unroll
    for (int it = 0; it < C::VP; ++it) {
        const int P = (it * 4 + wave) * 1024 + lane * 16, f = P >> 7;
        vgo[it] = (f * ldk + (((P >> 4) & 7) ^ ((f >> 1) & 7)) * 8) * 2;
    }
    // Q image pieces: piece `it` covers feature rows 8 it + 2 wave + (0, 1); the row's
    // 32-B block XOR depends on f & 7 only, so the lane part of the offset is constant
    int qgo;
    {
        const int f = 2 * wave + h, pb = (lane & 31) * 16;
        const int X = (f & 3) | (((f >> 2) & 1) << 2);
        qgo = f * N * 2 + ((((pb >> 5) ^ X) << 5) | (pb & 31));
    }

    const uint32_t kbytes = (uint32_t)(ldk * d * (int)sizeof(T)), vbytes = (uint32_t)(ldk * dv * (int)sizeof(T));
    const uint32_t qbytes = (uint32_t)(N * d * (int)sizeof(T));
    // a slab's K / V base; blocks past the end get a zero-length descriptor (reads → 0)
    auto kbase_of = [&](int id) { return (const T*)p.K + (int64_t)(id < nblk ? id / nqb : 0) * ldk * d; };
    auto vbase_of = [&](int id) { return (const T*)p.V + (int64_t)(id < nblk ? id / nqb : 0) * ldk * dv; };
    // K tile `j` of the slab behind `ds` into K slot `slot`
    auto dma_k1 = [&](const u32x4& ds, int slot, int j, int it) {
        p4_dma(ds, lds0 + C::KOFF + slot * C::KSLOT + (it * 4 + wave) * 1024, kgo[it], j * 128);
    };
    auto dma_v1 = [&](const u32x4& ds, int slot, int j, int it) {
        p4_dma(ds, lds0 + C::VOFF + slot * C::VSLOT + (it * 4 + wave) * 1024, vgo[it], j * 128);
    };
    // piece `it` of the Q image of the block whose Q slab is `ds` and query block qb;
    // `dst` = the piece's place in the image (or a scratch place: see phase B)
    auto dma_q1 = [&](const u32x4& ds, int qb, int it, uint32_t dst) {
        p4_dma(ds, dst, qgo, it * 16 * N + qb * (kP4Rows * 2));
    };
    auto qdst = [&](int it) { return lds0 + C::QOFF + (uint32_t)(it * 4 + wave) * 1024u; };

    F8 qf[2][C::NKS];
    f32x16 oacc[2][C::NCB];
    float m_used[2], m_true[2], l_run[2];
    f32x16 sA[2][2], sB[2][2];
    F8 pA0[2][2], pB0[2][2], p1[2][2];

    // ---- phase A: S = K(slot)·Qᵀ, each MFMA followed by valu(slot index) ----
    auto phaseA = [&](f32x16 (&S)[2][2], const char* kslot, auto&& valu) {
        F8 kf[3];
        // the lane offsets re-enter here (opaque), so the per-read addresses are one
        // base + immediate each instead of ~70 loop-invariant VGPRs the compiler would
        // hoist out of the tile loop (and spill)
        int ko[2] = {koff[0], koff[1]};
        asm volatile("" : "+v"(ko[0]), "+v"(ko[1]));
        auto rd = [&](int i) {
            const int kb = i / C::NKS, s = i % C::NKS;
            const char* a = kslot + ko[kb] + 16 * s * 128;
            const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(a));
            const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(a + 4 * 128));
            kf[i % 3] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        };
        rd(0);
        rd(1);
        p4_fence();
#pragma unroll
        for (int i = 0; i < C::NKQ; ++i) {
            const int kb = i / C::NKS, s = i % C::NKS;
            if (i + 2 < C::NKQ) rd(i + 2);
            p4_mfma_s(S[0][kb], kf[i % 3], qf[0][s], s == 0);
            valu(2 * i);
            p4_mfma_s(S[1][kb], kf[i % 3], qf[1][s], s == 0);
            valu(2 * i + 1);
            p4_fence();
        }
    };
    // ---- phase B: Oᵀ += Vᵀ(slot)·Pᵀ, each MFMA followed by valu(slot index) ----
    auto phaseB = [&](const char* vslot, const F8 (&P0)[2][2], const F8 (&P1)[2][2], auto&& valu) {
        F8 vf[3];
        int vo[2][2] = {{voff[0][0], voff[0][1]}, {voff[1][0], voff[1][1]}};
        asm volatile("" : "+v"(vo[0][0]), "+v"(vo[0][1]), "+v"(vo[1][0]), "+v"(vo[1][1]));
        auto rd = [&](int i) {
            const int cb = i >> 2, kb = (i >> 1) & 1, s = i & 1;
            vf[i % 3] = *(const F8*)(vslot + cb * 32 * 128 + vo[kb][s]);
        };
        rd(0);
        rd(1);
        p4_fence();
#pragma unroll
        for (int i = 0; i < C::NVQ; ++i) {
            const int cb = i >> 2, kb = (i >> 1) & 1, s = i & 1;
            if (i + 2 < C::NVQ) rd(i + 2);
            oacc[0][cb] = mfma32x32x16(vf[i % 3], P0[kb][s], oacc[0][cb]);
            valu(2 * i);
            oacc[1][cb] = mfma32x32x16(vf[i % 3], P1[kb][s], oacc[1][cb]);
            valu(2 * i + 1);
            p4_fence();
        }
    };
    auto no_valu = [](int) {};

    auto softmax_p = [&](const f32x16 (&S)[2], float mused, F8 (&P)[2][2]) -> float {
        SoftmaxQB<T> sm;
        sm.c = c;
        sm.mc = mused * c;
#pragma unroll
        for (int ch = 0; ch < 16; ++ch) {
            sm.part0(S, ch);
            sm.part1(P, ch);
        }
        return sm.sum();
    };

    // per-block DMA context: this block's and the next block's slabs
    const T *kp0 = nullptr, *kp1 = nullptr, *vp0 = nullptr, *vp1 = nullptr, *qpn = nullptr;
    uint32_t kn1 = 0, vn1 = 0, qnn = 0;   // the next block's descriptor lengths (0: none)
    int qbn = 0;

    // One pipelined tile j (K slot of tile j+1 = ksl1, of tile j = ksl0; V slot vsl):
    // Sc = S(j) with query block 0 already in Pc0; leaves Sn = S(j+1) and Pn0.
    auto step = [&](int j, int ksl0, int ksl1, int vsl, f32x16 (&Sc)[2][2], f32x16 (&Sn)[2][2], F8 (&Pc0)[2][2],
                    F8 (&Pn0)[2][2]) {
        // ---- phase A(j): Sn = K(j+1)·Qᵀ ∥ softmax of Sc, query block 1 ----
        {
            SoftmaxQB<T> sm;
            sm.c = c;
            sm.mc = m_used[1] * c;
            phaseA(Sn, kring + ksl1 * C::KSLOT, [&](int slot) {
                constexpr int NS = 2 * C::NKQ;   // MFMA slots: softmax parts [32 slot / NS, 32 (slot + 1) / NS)
#pragma unroll
                for (int part = 32 * slot / NS; part < 32 * (slot + 1) / NS; ++part) sm.part(Sc[1], p1, part);
            });
            l_run[1] += sm.sum();
        }
        p4_wait_all_barrier();
        // ---- phase B(j): O += V(j)·P(j) ∥ max of Sn, speculative softmax of Sn block 0, DMA ----
        MaxQB mx0, mx1;
        SoftmaxQB<T> sm;
        sm.c = c;
        sm.mc = m_used[0] * c;
        // DMA of this phase: K(j+3) → slot ksl0, V(j+1) → the other V slot, Q piece j
        const int jk = j + 3, jv = j + 1;
        const bool kn = jk >= NT, vn = jv >= NT;
        const u32x4 kds = p4_desc(kn ? kp1 : kp0, kn ? kn1 : kbytes), vds = p4_desc(vn ? vp1 : vp0, vn ? vn1 : vbytes);
        const int jk2 = kn ? jk - NT : jk, jv2 = vn ? jv - NT : jv;
        phaseB(vring + vsl * C::VSLOT, Pc0, p1, [&](int slot) {
            constexpr int NS = 2 * C::NVQ;   // MFMA slots; softmax parts and max steps spread evenly
            constexpr int NM = 2 * MaxQB::NOPS;
#pragma unroll
            for (int m = NM * slot / NS; m < NM * (slot + 1) / NS; ++m) {
                if (m < MaxQB::NOPS) mx0.op(Sn[0], m); else mx1.op(Sn[1], m - MaxQB::NOPS);
            }
#pragma unroll
            for (int part = 32 * slot / NS; part < 32 * (slot + 1) / NS; ++part) sm.part(Sn[0], Pn0, part);
            // DMA: spread over the phase
            constexpr int ND = C::KP + C::VP;
            if (slot % (NS / ND) == 1 && slot / (NS / ND) < ND) {
                const int it = slot / (NS / ND);
                if (it < C::KP) dma_k1(kds, ksl0, jk2, it);
                else dma_v1(vds, vsl ^ 1, jv2, it - C::KP);
            }
            // the next block's Q piece j; past the last piece the DMA goes to this wave's
            // O staging image (idle during the loop) from offset 0: no branch in the phase
            if (slot == NS - 2) {
                const bool qv = j < C::QP;
                dma_q1(p4_desc(qpn, qv ? qnn : 0u), qbn, qv ? j : 0, qv ? qdst(j) : lds0 + C::OOFF + (uint32_t)wave * C::OST);
            }
        });
        m_true[0] = vmax(m_true[0], mx0.mt);
        m_true[1] = vmax(m_true[1], mx1.mt);
        const bool f0 = __builtin_amdgcn_ballot_w64(mx0.mt > m_used[0] + thr_raw) != 0;
        const bool f1 = __builtin_amdgcn_ballot_w64(mx1.mt > m_used[1] + thr_raw) != 0;
        float ps0 = sm.sum();
        FA_P4_STAMP(2);
        if (f0 || f1) {   // rare: the running max moved by more than the threshold
            p4_mfma_drain();
            if (f0) {
                const float mn = fmaxf(m_used[0], swap_halves_max(mx0.mt));
                const float al = exp2_fast((m_used[0] - mn) * c);
                l_run[0] *= al;
#pragma unroll
                for (int cb = 0; cb < C::NCB; ++cb)
#pragma unroll
                    for (int x = 0; x < 16; ++x) oacc[0][cb][x] *= al;
                m_used[0] = mn;
                ps0 = softmax_p(Sn[0], mn, Pn0);
            }
            if (f1) {
                const float mn = fmaxf(m_used[1], swap_halves_max(mx1.mt));
                const float al = exp2_fast((m_used[1] - mn) * c);
                l_run[1] *= al;
#pragma unroll
                for (int cb = 0; cb < C::NCB; ++cb)
#pragma unroll
                    for (int x = 0; x < 16; ++x) oacc[1][cb][x] *= al;
                m_used[1] = mn;
            }
        }
        l_run[0] += ps0;
    };

    // ---- prologue: the first block's Q and the first K / V tiles ----
    {
        const int id0 = w;
        const u32x4 kd0 = p4_desc(kbase_of(id0), id0 < nblk ? kbytes : 0u);
        const u32x4 vd0 = p4_desc(vbase_of(id0), id0 < nblk ? vbytes : 0u);
        const u32x4 qd = p4_desc((const T*)p.Q + (int64_t)(id0 < nblk ? id0 / nqb : 0) * N * d, id0 < nblk ? qbytes : 0u);
        const int qb0 = id0 % nqb;
#pragma unroll
        for (int it = 0; it < C::QP; ++it) dma_q1(qd, qb0, it, qdst(it));
#pragma unroll
        for (int it = 0; it < C::KP; ++it) {
            dma_k1(kd0, 0, 0, it);
            dma_k1(kd0, 1, 1, it);
            dma_k1(kd0, 2, 2, it);
        }
#pragma unroll
        for (int it = 0; it < C::VP; ++it) dma_v1(vd0, 0, 0, it);
        p4_wait_all_barrier();
    }
    FA_P4_STAMP(0);

    int ks = 0, vs = 0;   // ring slots of this block's tile 0
    for (int k = 0;; ++k) {
        const int id = w + k * G;
        if (id >= nblk) break;
        const int b = id / nqb, qb = id - b * nqb;
        const bool more = id + G < nblk;
        kp0 = kbase_of(id);
        vp0 = vbase_of(id);
        kp1 = kbase_of(id + G);
        vp1 = vbase_of(id + G);
        kn1 = more ? kbytes : 0u;
        vn1 = more ? vbytes : 0u;
        qpn = (const T*)p.Q + (int64_t)(more ? (id + G) / nqb : 0) * N * d;
        qnn = more ? qbytes : 0u;
        qbn = (id + G) % nqb;
        // Q fragments of this block (its image landed behind an earlier barrier)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int s = 0; s < C::NKS; ++s) {
                const int tb = ((wave * 2 + u) * 32 + 16 * kh + 4 * pp) * 2;
                const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(qimg + p4_qpos(16 * s + 8 * h + qq, tb)));
                const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(qimg + p4_qpos(16 * s + 8 * h + 4 + qq, tb)));
                qf[u][s] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
            }
        // S(0) (the pipeline restarts at each block)
        phaseA(sA, kring + ks * C::KSLOT, no_valu);
        p4_mfma_drain();
        {
            MaxQB m0, m1;
#pragma unroll
            for (int m = 0; m < MaxQB::NOPS; ++m) { m0.op(sA[0], m); m1.op(sA[1], m); }
            m_true[0] = m0.mt;
            m_true[1] = m1.mt;
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            m_used[u] = swap_halves_max(m_true[u]);
#pragma unroll
            for (int cb = 0; cb < C::NCB; ++cb)
#pragma unroll
                for (int x = 0; x < 16; ++x) oacc[u][cb][x] = 0.0f;
        }
        l_run[0] = softmax_p(sA[0], m_used[0], pA0);
        l_run[1] = 0.0f;
        FA_P4_STAMP(1);

        // tiles 0 .. NT-2 in pairs (the S / P buffers alternate), then the last tile
        int j = 0;
        int k0 = ks, k1 = ks == 2 ? 0 : ks + 1, v0 = vs;
        auto adv = [&]() {
            k0 = k1;
            k1 = k1 == 2 ? 0 : k1 + 1;
            v0 ^= 1;
        };
        bool lastB = false;
        for (;;) {
            if (j + 1 >= NT) break;
            step(j, k0, k1, v0, sA, sB, pA0, pB0);
            ++j;
            adv();
            if (j + 1 >= NT) { lastB = true; break; }
            step(j, k0, k1, v0, sB, sA, pB0, pA0);
            ++j;
            adv();
        }
        // ---- last tile j = NT-1 (in sB / pB0 when lastB) ----
        auto last = [&](f32x16 (&Sc)[2][2], F8 (&Pc0)[2][2]) {
            l_run[1] += softmax_p(Sc[1], m_used[1], p1);
            p4_wait_all_barrier();
            const int jk = j + 3 - NT, jv = j + 1 - NT;   // both in the next block
            phaseB(vring + v0 * C::VSLOT, Pc0, p1, [&](int slot) {
                constexpr int ND = C::KP + C::VP;
                constexpr int NS = 2 * C::NVQ;
                if (slot % (NS / ND) == 1 && slot / (NS / ND) < ND) {
                    const int it = slot / (NS / ND);
                    if (it < C::KP) dma_k1(p4_desc(kp1, kn1), k0, jk, it);
                    else dma_v1(p4_desc(vp1, vn1), v0 ^ 1, jv, it - C::KP);
                }
            });
        };
        if (lastB) last(sB, pB0); else last(sA, pA0);
        // next block's ring slots: tile NT of this stream
        ks = k1;
        vs = v0 ^ 1;
        FA_P4_STAMP(3);

        // ---- epilogue: O / l through the wave's staging image, l and m ----
        p4_mfma_drain();
        const auto ors = slab_rsrc((T*)p.O + (int64_t)b * N * dv, (uint32_t)(N * dv * (int)sizeof(T)));
        float inv[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const float mt = swap_halves_max(m_true[u]);
            const float lt = swap_halves_sum(l_run[u]);
            inv[u] = 1.0f / lt;
            const int qi = qb * kP4Rows + (wave * 2 + u) * 32 + r;
            if (qi < N && h == 0) {
                p.m[(int64_t)b * N + qi] = mt * p.scale;
                p.l[(int64_t)b * N + qi] = lt * exp2_fast((m_used[u] - mt) * c);
            }
        }
        char* const myost = ost + wave * C::OST;
#pragma unroll
        for (int cb = 0; cb < C::NCB; ++cb) {
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int x = 0; x < 16; ++x) {
                    const int f = acc_row(x, h), tok = u * 32 + r;
                    *(T*)(myost + f * 128 + (((tok >> 3) ^ (f & 7)) << 4) + (tok & 7) * 2) = (T)(oacc[u][cb][x] * inv[u]);
                }
#pragma unroll
            for (int it = 0; it < 4; ++it) {
                const int idx = it * 64 + lane, f = idx >> 3, ch = idx & 7;
                const u32x4 v4 = *(const u32x4*)(myost + f * 128 + ((ch ^ (f & 7)) << 4));
                const int fo = cb * 32 + f, q = qb * kP4Rows + wave * 64 + ch * 8;
                const int off = (fo < dv && q < N) ? (fo * N + q) * 2 : 0x7FFFFFF0;
                __builtin_amdgcn_raw_buffer_store_b128(v4, ors, off, 0, 0);
            }
        }
        FA_P4_STAMP(4);
    }
}

// Launch on the persistent grid; returns false when the shape is not this kernel's.
bool launch_dense_fwd_p4(const FwdParams& p, int Dc, int DVc, int dtype, hipStream_t s, hipError_t* err) {
    if (!p.fast || !p.wide || p.nsplit > 1 || Dc != DVc || p.d != Dc || p.dv != DVc) return false;
    const int cus = device_cus(s);
    if (cus <= 0) return false;
    // the Q prefetch goes out in phases B(0 .. QP-1) of the previous block; whole key tiles
    if (p.Nk % 64 != 0 || p.Nk / 64 < Dc / 8 + 1 || p.ldk != p.Nk) return false;
    FwdParams q = p;
    q.nqb = (p.N + kP4Rows - 1) / kP4Rows;
    const int64_t nblk = (int64_t)q.nqb * p.batch;
    if (nblk < cus || nblk > INT32_MAX / 2) return false;
    q.total_wg = (int)nblk;
    const dim3 grid((unsigned)cus), blk(256);
#define FA_P4_LAUNCH(TT)                                                                                         \
    switch (Dc) {                                                                                                \
        case 64: hipLaunchKernelGGL((dense_fwd_p4<TT, 64, 64>), grid, blk, 0, s, q); break;                     \
        case 128: hipLaunchKernelGGL((dense_fwd_p4<TT, 128, 128>), grid, blk, 0, s, q); break;                  \
        default: return false;                                                                                   \
    }
    if (dtype == FA_DTYPE_BF16) { FA_P4_LAUNCH(bf16) }
    else if (dtype == FA_DTYPE_F16) { FA_P4_LAUNCH(f16) }
    else return false;
#undef FA_P4_LAUNCH
    *err = hipGetLastError();
    return true;
}

}  // namespace fa
