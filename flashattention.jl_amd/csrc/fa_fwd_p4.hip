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
#include <type_traits>

#include "fa_common.h"
#include "fa_internal.h"
#include "fa_fwd_params.h"
#include "../../include/fa_hip.h"

// Diagnostic hooks (tools/exp/p4_lab.hip; empty in the product build):
// FA_P4_STAMP(point, tile) records s_memtime at a phase boundary.
#ifndef FA_P4_STAMP
#define FA_P4_STAMP(pt, j)
#endif
// FA_P4_SLOT(i): a sample of s_memtime at MFMA slot i of a tile's X/Y stream (no wait
// there); FA_P4_SLOT_FLUSH(j) waits for the samples and records them.
#ifndef FA_P4_SLOT
#define FA_P4_SLOT_DECL
#define FA_P4_SLOT(i)
#define FA_P4_SLOT_FLUSH(j)
#endif
// FA_P4_ABL: timing-only ablations of the diagnostic build (WRONG results): 1 no K/V/Q
// DMA in the tile loop, 2 no exponentials, 4 no LDS operand reads in the tile loop,
// 8 no softmax / max VALU work at all, 16 one transposed read per K fragment (of two),
// 32 no V fragment reads.
#ifndef FA_P4_ABL
#define FA_P4_ABL 0
#endif

namespace fa {

namespace {

constexpr int kP4Rows = 256;   // query rows per block: 4 waves x 2 x 32
constexpr int kP4KS = 3;       // K ring slots (K(t+3) issued in phase B(t))
constexpr int kP4VS = 2;       // V ring slots (V(t+1) issued in phase B(t))
#ifndef FA_P4_PF
#define FA_P4_PF 4
#endif
constexpr int kP4Prefetch = FA_P4_PF;   // MFMA slots an LDS operand read runs ahead (LDS latency ~100+ cycles)
#ifndef FA_P4_DMA
#define FA_P4_DMA 0
#endif
#ifndef FA_P4_EARLYMAX
#define FA_P4_EARLYMAX 0
#endif
// 1: a query block's tile maximum runs in the phase that computes its scores (after
// those MFMAs have retired), so the next phase can spend every MFMA gap on the
// exponentials (the lazy-rescale decision moves to that phase's first slot)
constexpr bool kP4EarlyMax = FA_P4_EARLYMAX != 0;
// MFMA slot of DMA piece q of n in a phase of NM slots whose softmax starts at slot np:
// 0 = back to back from np, 1 = spread evenly over [np, NM), 2 = the last n slots
__host__ __device__ constexpr int p4_dma_slot(int q, int n, int np, int NM) {
    return FA_P4_DMA == 1 ? np + q * ((NM - np) / n) : FA_P4_DMA == 2 ? NM - n + q : np + q;
}

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

// Compile-time loop: f(std::integral_constant<int, I>) for I = 0 .. N-1 (every index
// is a constant, whatever the body's size; #pragma unroll may stop short of a full
// unroll of a big body and leave register arrays dynamically indexed, i.e. in scratch).
template <class F, int... I>
__device__ __forceinline__ void p4_static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void p4_static_for(F&& f) { p4_static_for_impl(f, std::make_integer_sequence<int, N>{}); }

// Q image position of logical byte `lb` (= 2 x token) of feature row f (the qo_at of
// dense_fwd_tiled at 256 rows): 32-B blocks XOR (f & 3) | (bit 2 of f) << 2.
__device__ __forceinline__ int p4_qpos(int f, int lb) {
    const int X = (f & 3) | (((f >> 2) & 1) << 2);
    return f * (kP4Rows * 2) + (((lb >> 5) ^ X) << 5) + (lb & 31);
}

// The softmax and row-max VALU work is written as inline asm, one short statement per
// step: volatile asm keeps program order against the MFMA asm, so each step stays in
// the MFMA slot it is written in (compiler-generated arithmetic floats across
// sched_barrier, and pinning it with register fences costs s_nop / s_mov per fence).
// Hazards inside the hot loop are the kernel's: an exponential's consumer is never the
// next instruction (part1 of chunk c follows part0 of chunk c+1), and the scores an
// asm MFMA writes are read a phase later.
__device__ __forceinline__ void p4_exp2x2(float& e0, float& e1, float s0, float s1, float c, float nmc) {
    float t0, t1;
    if (FA_P4_ABL & 2)
        asm volatile("v_fma_f32 %0, %2, %4, %5\n\tv_fma_f32 %1, %3, %4, %5" : "=&v"(e0), "=&v"(e1) : "v"(s0), "v"(s1), "s"(c), "v"(nmc));
    else
        asm volatile("v_fma_f32 %2, %4, %6, %7\n\tv_fma_f32 %3, %5, %6, %7\n\tv_exp_f32 %0, %2\n\tv_exp_f32 %1, %3"
                     : "=&v"(e0), "=&v"(e1), "=&v"(t0), "=&v"(t1)
                     : "v"(s0), "v"(s1), "s"(c), "v"(nmc));
}
template <class T>
__device__ __forceinline__ unsigned p4_pack(float e0, float e1) {
    unsigned r;
    if constexpr (std::is_same<T, bf16>::value) asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(e0), "v"(e1));
    else asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(e0), "v"(e1));
    return r;
}
__device__ __forceinline__ void p4_add2(float& a0, float& a1, float e0, float e1) {
    asm volatile("v_add_f32 %0, %0, %2\n\tv_add_f32 %1, %1, %3" : "+v"(a0), "+v"(a1) : "v"(e0), "v"(e1));
}
__device__ __forceinline__ float p4_max3(float a, float b, float c) {
    float r;
    asm volatile("v_maximum3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// The softmax of one query block's 64 scores per lane pair (32 per lane), cut into
// 16 chunks of two scores, each in two parts: part 0 = two FMAs (c·s − c·m) and two
// exponentials, part 1 = the two sum adds and the bf16/f16 pack into P (dword view).
template <class T>
struct SoftmaxQB {
    float nmc, c;    // −c·m_used, c
    float e[2][2];   // exponentials of chunk c in e[c & 1]
    float ps[4];
    __device__ __forceinline__ void part0(const f32x16 (&S)[2], int ch) {
        const int kb = ch >> 3, x = 2 * (ch & 7);
        p4_exp2x2(e[ch & 1][0], e[ch & 1][1], S[kb][x], S[kb][x + 1], c, nmc);
    }
    __device__ __forceinline__ void part1(u32x4 (&P)[2][2], int ch) {
        const int kb = ch >> 3, x = 2 * (ch & 7);
        const float e0 = e[ch & 1][0], e1 = e[ch & 1][1];
        if (ch < 2) {   // the first four exponentials seed the partial sums
            ps[x & 3] = e0;
            ps[(x + 1) & 3] = e1;
        } else {
            p4_add2(ps[x & 3], ps[(x + 1) & 3], e0, e1);
        }
        P[kb][x >> 3][(x & 7) >> 1] = p4_pack<T>(e0, e1);
    }
    // part k of 32 in issue order: part0 of chunk 0, then (part0 of chunk c+1, part1
    // of chunk c) pairs, then part1 of chunk 15
    __device__ __forceinline__ void part(const f32x16 (&S)[2], u32x4 (&P)[2][2], int k) {
        if (k == 0) part0(S, 0);
        else if (k == 31) part1(P, 15);
        else if (k & 1) part0(S, (k + 1) >> 1);
        else part1(P, (k >> 1) - 1);
    }
    __device__ __forceinline__ float sum() const { return (ps[0] + ps[1]) + (ps[2] + ps[3]); }
};

// Lane maximum of one query block's 32 scores in 16 v_maximum3 steps: four chains
// seeded with three scores each (steps 0-3), ten chain steps of two scores, then the
// combine (steps 14, 15 leave the result in mt).
struct MaxQB {
    float a[4], t, mt;
    static constexpr int NOPS = 16;
    __device__ __forceinline__ void op(const f32x16 (&S)[2], int m) {
        auto v = [&](int k) { return S[k >> 4][k & 15]; };
        if (m < 4) a[m] = p4_max3(v(3 * m), v(3 * m + 1), v(3 * m + 2));
        else if (m < 14) { const int k = 12 + 2 * (m - 4), cc = m & 3; a[cc] = p4_max3(a[cc], v(k), v(k + 1)); }
        else if (m == 14) t = p4_max3(a[0], a[1], a[2]);
        else mt = p4_max3(t, a[3], a[3]);
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
    auto kbase_of = [&](int id) __attribute__((always_inline)) { return (const T*)p.K + (int64_t)(id < nblk ? id / nqb : 0) * ldk * d; };
    auto vbase_of = [&](int id) __attribute__((always_inline)) { return (const T*)p.V + (int64_t)(id < nblk ? id / nqb : 0) * ldk * dv; };
    // K tile `j` of the slab behind `ds` into K slot `slot`
    auto dma_k1 = [&](const u32x4& ds, int slot, int j, int it) __attribute__((always_inline)) {
        p4_dma(ds, lds0 + C::KOFF + slot * C::KSLOT + (it * 4 + wave) * 1024, kgo[it], j * 128);
    };
    auto dma_v1 = [&](const u32x4& ds, int slot, int j, int it) __attribute__((always_inline)) {
        p4_dma(ds, lds0 + C::VOFF + slot * C::VSLOT + (it * 4 + wave) * 1024, vgo[it], j * 128);
    };
    // piece `it` of the Q image of the block whose Q slab is `ds` and query block qb;
    // `dst` = the piece's place in the image (or a scratch place: see phase B)
    auto dma_q1 = [&](const u32x4& ds, int qb, int it, uint32_t dst) __attribute__((always_inline)) {
        p4_dma(ds, dst, qgo, it * 16 * N + qb * (kP4Rows * 2));
    };
    auto qdst = [&](int it) __attribute__((always_inline)) { return lds0 + C::QOFF + (uint32_t)(it * 4 + wave) * 1024u; };

    F8 qf[2][C::NKS];
    f32x16 oacc[2][C::NCB];
    f32x16 S[2][2];        // [query block][key block]: one score tile per query block
    u32x4 P[2][2][2];      // [query block][key block][k-step], packed P (dword view of the bf16x8 operand)
    float m_used[2], m_true[2], l_run[2];
    FA_P4_SLOT_DECL

    // ---- one phase: the MFMAs of query block u — Sᵀ_u = K·Qᵀ_u (QK) then Oᵀ_u += Vᵀ·Pᵀ_u
    // (PV) — with valu(slot) after each MFMA and mid() before MFMA slot NPRE.  The LDS
    // operands stream two fragments ahead; sched_barrier(0) fences every slot.
    auto phase = [&](auto QKt, auto PVt, auto NPREt, int u, const char* kslot, const char* vslot, auto&& valu,
                     auto&& mid) __attribute__((always_inline)) {
        constexpr bool QK = decltype(QKt)::value, PV = decltype(PVt)::value;
        constexpr int NPRE = decltype(NPREt)::value;
        constexpr int NKQ = QK ? C::NKQ : 0;
        constexpr int NM = NKQ + (PV ? C::NVQ : 0);
        // the lane offsets re-enter here (opaque), so each read is one base + immediate
        // instead of ~70 loop-invariant address VGPRs the compiler would hoist and spill
        int ko[2] = {koff[0], koff[1]};
        int vo[2][2] = {{voff[0][0], voff[0][1]}, {voff[1][0], voff[1][1]}};
        asm volatile("" : "+v"(ko[0]), "+v"(ko[1]), "+v"(vo[0][0]), "+v"(vo[0][1]), "+v"(vo[1][0]), "+v"(vo[1][1]));
        constexpr int PF = kP4Prefetch;   // LDS operand reads run PF MFMA slots ahead
        F8 fr[PF + 1];
        auto rd = [&](int i) __attribute__((always_inline)) {
            if ((FA_P4_ABL & 4) && i >= 2 && (PV || QK) && NM > 8) return;
            if (i < NKQ) {
                const int kb = i / C::NKS, s = i % C::NKS;
                const char* a = kslot + ko[kb] + 16 * s * 128;
                const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(a));
                const F4 hi = __builtin_bit_cast(F4, ds_read_tr16(a + 4 * 128));
                fr[i % (PF + 1)] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
            } else {
                const int j = i - NKQ, cb = j >> 2, kb = (j >> 1) & 1, s = j & 1;
                fr[i % (PF + 1)] = *(const F8*)(vslot + cb * 32 * 128 + vo[kb][s]);
            }
        };
        p4_static_for<(PF < NM ? PF : NM)>([&](auto It) __attribute__((always_inline)) { rd(decltype(It)::value); });
        p4_fence();
        p4_static_for<NM>([&](auto It) __attribute__((always_inline)) {
            constexpr int i = decltype(It)::value;
            if constexpr (i == NPRE) {
                mid();
                p4_fence();
            }
            if constexpr (i + PF < NM) rd(i + PF);
            if constexpr (i < NKQ) {
                constexpr int kb = i / C::NKS, s = i % C::NKS;
                p4_mfma_s(S[u][kb], fr[i % (PF + 1)], qf[u][s], s == 0);
            } else {
                constexpr int j = i - NKQ, cb = j >> 2, kb = (j >> 1) & 1, s = j & 1;
                oacc[u][cb] = mfma32x32x16(fr[i % (PF + 1)], __builtin_bit_cast(F8, P[u][kb][s]), oacc[u][cb]);
            }
            valu(i);
            p4_fence();
        });
        if constexpr (NPRE >= NM) mid();
    };
    // Both phases of a tile in one stream: X = query block 0's MFMAs with valx / midx,
    // then Y = block 1's with valy / midy (same kinds of MFMA, so the same K / V fragments
    // in the same order: block 1 reads what block 0 read).  The operand prefetch runs on
    // across the seam, so Y's first reads are in flight under X's last MFMAs instead of
    // waited for at Y's start; seam() runs between the two.
    auto phase2 = [&](auto QKt, auto PVt, auto NPXt, auto NPYt, const char* kslot, const char* vslot, auto&& valx,
                      auto&& midx, auto&& seam, auto&& valy, auto&& midy) __attribute__((always_inline)) {
        constexpr bool QK = decltype(QKt)::value, PV = decltype(PVt)::value;
        constexpr int NPX = decltype(NPXt)::value, NPY = decltype(NPYt)::value;
        constexpr int NKQ = QK ? C::NKQ : 0;
        constexpr int NM = NKQ + (PV ? C::NVQ : 0);
        int ko[2] = {koff[0], koff[1]};
        int vo[2][2] = {{voff[0][0], voff[0][1]}, {voff[1][0], voff[1][1]}};
        asm volatile("" : "+v"(ko[0]), "+v"(ko[1]), "+v"(vo[0][0]), "+v"(vo[0][1]), "+v"(vo[1][0]), "+v"(vo[1][1]));
        constexpr int PF = kP4Prefetch;
        F8 fr[PF + 1];
        auto rd = [&](int i) __attribute__((always_inline)) {
            const int f = i % NM;
            if ((FA_P4_ABL & 4) && f >= 2 && NM > 8) return;
            if ((FA_P4_ABL & 32) && f >= NKQ && f >= 2) return;
            if (f < NKQ) {
                const int kb = f / C::NKS, s = f % C::NKS;
                const char* a = kslot + ko[kb] + 16 * s * 128;
                const F4 lo = __builtin_bit_cast(F4, ds_read_tr16(a));
                const F4 hi = (FA_P4_ABL & 16) ? lo : __builtin_bit_cast(F4, ds_read_tr16(a + 4 * 128));
                fr[i % (PF + 1)] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
            } else {
                const int j = f - NKQ, cb = j >> 2, kb = (j >> 1) & 1, s = j & 1;
                fr[i % (PF + 1)] = *(const F8*)(vslot + cb * 32 * 128 + vo[kb][s]);
            }
        };
        p4_static_for<(PF < NM ? PF : NM)>([&](auto It) __attribute__((always_inline)) { rd(decltype(It)::value); });
        p4_fence();
        p4_static_for<2 * NM>([&](auto It) __attribute__((always_inline)) {
            constexpr int i = decltype(It)::value;
            constexpr int u = i / NM, k = i % NM;
            if constexpr (u == 0 && k == NPX) {
                midx();
                p4_fence();
            }
            if constexpr (u == 1 && k == NPY) {
                midy();
                p4_fence();
            }
            if constexpr (i + PF < 2 * NM) rd(i + PF);
            if constexpr (k < NKQ) {
                constexpr int kb = k / C::NKS, s = k % C::NKS;
                p4_mfma_s(S[u][kb], fr[i % (PF + 1)], qf[u][s], s == 0);
            } else {
                constexpr int j = k - NKQ, cb = j >> 2, kb = (j >> 1) & 1, s = j & 1;
                oacc[u][cb] = mfma32x32x16(fr[i % (PF + 1)], __builtin_bit_cast(F8, P[u][kb][s]), oacc[u][cb]);
            }
            if constexpr (u == 0) valx(k);
            else valy(k);
            FA_P4_SLOT(i);
            p4_fence();
            if constexpr (i == NM - 1) {
                if constexpr (NPX >= NM) midx();
                seam();
                p4_fence();
            }
        });
        if constexpr (NPY >= NM) midy();
    };
    auto none = [](int) __attribute__((always_inline)) {};
    auto nomid = []() __attribute__((always_inline)) {};

    // the lazy-rescale decision for query block v after its tile max: the running max
    // used for the exponentials is raised only when some lane's tile max exceeds it by
    // more than the threshold (a wave-uniform branch); O_v's last MFMAs ran in the
    // previous phase, l_v and O_v are scaled together.  m_used starts at −inf, so the
    // first tile always takes the branch (scaling O = 0, l = 0 by 0).
    auto decide = [&](int v, float mt) __attribute__((always_inline)) {
        if (FA_P4_ABL & 8) mt = 0.0f;
        m_true[v] = vmax(m_true[v], mt);
        if (__builtin_amdgcn_ballot_w64(mt > m_used[v] + thr_raw) != 0) {
            const float mn = fmaxf(m_used[v], swap_halves_max(mt));
            const float al = exp2_fast((m_used[v] - mn) * c);
            l_run[v] *= al;
#pragma unroll
            for (int cb = 0; cb < C::NCB; ++cb)
#pragma unroll
                for (int x = 0; x < 16; ++x) oacc[v][cb][x] *= al;
            m_used[v] = mn;
        }
    };

    // The VALU side of a phase for query block v: its tile max in the first NPRE MFMA
    // slots, the decision, then its softmax (P_v, l_v) over the remaining slots.
    // NM = MFMA slots of the phase.
    auto softmax_side = [&](auto NMt, auto NPREt, int v, MaxQB& mx, SoftmaxQB<T>& sm) __attribute__((always_inline)) {
        constexpr int NM = decltype(NMt)::value, NPRE = decltype(NPREt)::value;
        return [&, v](int i) __attribute__((always_inline)) {
            if (FA_P4_ABL & 8) return;
            if (i < NPRE) {
#pragma unroll
                for (int m = MaxQB::NOPS * i / NPRE; m < MaxQB::NOPS * (i + 1) / NPRE; ++m) mx.op(S[v], m);
            } else {
                const int k = i - NPRE;
#pragma unroll
                for (int part = 32 * k / (NM - NPRE); part < 32 * (k + 1) / (NM - NPRE); ++part) sm.part(S[v], P[v], part);
            }
        };
    };

    float mt1c = 0.0f;   // early max: block 1's tile max for the next X phase
    // per-block DMA context: this block's and the next block's slabs
    int p4_blk = 0;   // block counter of this workgroup (read by the diagnostic stamps only)
    (void)p4_blk;
    const T *kp0 = nullptr, *kp1 = nullptr, *vp0 = nullptr, *vp1 = nullptr, *qpn = nullptr;
    uint32_t kn1 = 0, vn1 = 0, qnn = 0;   // the next block's descriptor lengths (0: none)
    int qbn = 0;

    typedef std::integral_constant<bool, true> Yes;
    typedef std::integral_constant<bool, false> No;
    constexpr int NMF = C::NKQ + C::NVQ;              // MFMA slots of a full phase
    constexpr int NPRE = NMF >= 32 ? 6 : 4;           // slots carrying the max chains
    typedef std::integral_constant<int, NMF> NMt;
    typedef std::integral_constant<int, C::NVQ> NMvt;  // PV-only phase (last tile)

    // One tile t (block tile j): X = query block 0's MFMAs ∥ block 1's softmax of tile
    // j; Y = block 1's MFMAs ∥ block 0's softmax of tile j+1.  DMA: the next V tile and
    // the next block's Q piece in X, the K tile three ahead in Y; then the wait for
    // everything but that K tile, and the tile's barrier.
    auto tile = [&](auto LASTt, int j, int ks1, int ks0, int vs0) __attribute__((always_inline)) {
        constexpr bool LAST = decltype(LASTt)::value;
        const char* kslot = kring + ks1 * C::KSLOT;   // K(j+1)
        const char* vslot = vring + vs0 * C::VSLOT;   // V(j)
        // DMA targets: V(j+1) → the other V slot, K(j+3) → the slot of K(j)
        const int jv = j + 1, jk = j + 3;
        const bool vn = jv >= NT, kn = jk >= NT;
        const u32x4 vds = p4_desc(vn ? vp1 : vp0, vn ? vn1 : vbytes), kds = p4_desc(kn ? kp1 : kp0, kn ? kn1 : kbytes);
        const int jv2 = vn ? jv - NT : jv, jk2 = kn ? jk - NT : jk;
        FA_P4_STAMP(2, j);
        // ---- X: block 0 MFMAs ∥ block 1 softmax (tile j); Y: block 1 MFMAs ∥ block 0
        //      softmax (tile j+1), or on the last tile block 1's PV only ----
        constexpr int NMx = LAST ? C::NVQ : NMF;
        constexpr int NPx = kP4EarlyMax ? 0 : LAST ? (C::NVQ >= 16 ? 4 : 2) : NPRE;   // max slots before the exps
        constexpr int NPy = kP4EarlyMax ? 0 : NPRE;
        constexpr int DMx = kP4EarlyMax ? 2 : NPx, DMy = kP4EarlyMax ? 2 : NPRE;     // first DMA slot
        constexpr int MX0 = C::NKQ + 2;   // early max: first slot after this phase's score MFMAs retired
        MaxQB mx1, mx0;
        SoftmaxQB<T> sm1, sm0;
        sm1.c = c;
        sm0.c = c;
        auto side1 = softmax_side(std::conditional_t<LAST, NMvt, NMt>{}, std::integral_constant<int, NPx>{}, 1, mx1, sm1);
        auto side0 = softmax_side(NMt{}, std::integral_constant<int, NPy>{}, 0, mx0, sm0);
        // early max of block v's scores computed in this phase (slots MX0 .. NMF-1)
        auto early_max = [&](int i, int v, MaxQB& mx) __attribute__((always_inline)) {
            if (FA_P4_ABL & 8) return;
            if (i >= MX0) {
#pragma unroll
                for (int m = MaxQB::NOPS * (i - MX0) / (NMF - MX0); m < MaxQB::NOPS * (i - MX0 + 1) / (NMF - MX0); ++m)
                    mx.op(S[v], m);
            }
        };
        auto valx = [&](int i) __attribute__((always_inline)) {
            side1(i);
            if constexpr (kP4EarlyMax && !LAST) early_max(i, 0, mx0);
            // V(j+1) pieces, then the Q piece (slots: p4_dma_slot)
            if (FA_P4_ABL & 1) return;
#pragma unroll
            for (int q = 0; q < C::VP; ++q)
                if (i == p4_dma_slot(q, C::VP + 1, DMx, NMx)) dma_v1(vds, vs0 ^ 1, jv2, q);
            if (i == p4_dma_slot(C::VP, C::VP + 1, DMx, NMx)) {
                const bool qv = j < C::QP;
                dma_q1(p4_desc(qpn, qv ? qnn : 0u), qbn, qv ? j : 0, qv ? qdst(j) : lds0 + C::OOFF + (uint32_t)wave * C::OST);
            }
        };
        auto midx = [&]() __attribute__((always_inline)) {
            decide(1, kP4EarlyMax ? mt1c : mx1.mt);
            sm1.nmc = -m_used[1] * c;
        };
        auto seam = [&]() __attribute__((always_inline)) {
            l_run[1] += sm1.sum();
            FA_P4_STAMP(3, j);
        };
        auto valy = [&](int i) __attribute__((always_inline)) {
            if constexpr (!LAST) {
                side0(i);
                if constexpr (kP4EarlyMax) early_max(i, 1, mx1);
#pragma unroll
                for (int q = 0; q < C::KP; ++q)
                    if (!(FA_P4_ABL & 1) && i == p4_dma_slot(q, C::KP, DMy, NMF)) dma_k1(kds, ks0, jk2, q);
            } else {
                if (!(FA_P4_ABL & 1) && i < C::KP) dma_k1(kds, ks0, jk2, i);
            }
        };
        auto midy = [&]() __attribute__((always_inline)) {
            if constexpr (!LAST) {
                decide(0, mx0.mt);
                sm0.nmc = -m_used[0] * c;
            }
        };
        phase2(std::integral_constant<bool, !LAST>{}, Yes{}, std::integral_constant<int, NPx>{},
               std::integral_constant<int, LAST ? 1000 : NPy>{}, kslot, vslot, valx, midx, seam, valy, midy);
        if constexpr (!LAST) l_run[0] += sm0.sum();
        if constexpr (kP4EarlyMax && !LAST) mt1c = mx1.mt;
        FA_P4_SLOT_FLUSH(j);
        FA_P4_STAMP(5, j);
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(C::KP) : "memory");
        FA_P4_STAMP(6, j);
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
    FA_P4_STAMP(0, -1);

    int ks = 0, vs = 0;   // ring slots of this block's tile 0
    for (int k = 0;; ++k) {
        const int id = w + k * G;
        if (id >= nblk) break;
        p4_blk = k;
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
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            m_used[u] = kNegInf;
            m_true[u] = kNegInf;
            l_run[u] = 0.0f;
#pragma unroll
            for (int cb = 0; cb < C::NCB; ++cb)
#pragma unroll
                for (int x = 0; x < 16; ++x) oacc[u][cb][x] = 0.0f;
        }
        // S(0) of both query blocks (the pipeline restarts at each block)
        phase(Yes{}, No{}, std::integral_constant<int, 1000>{}, 0, kring + ks * C::KSLOT, nullptr, none, nomid);
        phase(Yes{}, No{}, std::integral_constant<int, 1000>{}, 1, kring + ks * C::KSLOT, nullptr, none, nomid);
        // every wave's K(0) and Q reads are done before any wave DMAs into those places
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
        {   // block 0's tile-0 softmax (not overlapped)
            MaxQB mx;
#pragma unroll
            for (int m = 0; m < MaxQB::NOPS; ++m) mx.op(S[0], m);
            decide(0, mx.mt);
            SoftmaxQB<T> sm;
            sm.c = c;
            sm.nmc = -m_used[0] * c;
#pragma unroll
            for (int part = 0; part < 32; ++part) sm.part(S[0], P[0], part);
            l_run[0] += sm.sum();
            if constexpr (kP4EarlyMax) {   // block 1's tile-0 max for the first X phase
                MaxQB mx1;
#pragma unroll
                for (int m = 0; m < MaxQB::NOPS; ++m) mx1.op(S[1], m);
                mt1c = (FA_P4_ABL & 8) ? 0.0f : mx1.mt;
            }
        }
        FA_P4_STAMP(1, -1);

        int k1 = ks == 2 ? 0 : ks + 1, k0 = ks, v0 = vs;   // slots of K(j+1), K(j), V(j)
        for (int j = 0; j < NT - 1; ++j) {
            tile(No{}, j, k1, k0, v0);
            k0 = k1;
            k1 = k1 == 2 ? 0 : k1 + 1;
            v0 ^= 1;
        }
        tile(Yes{}, NT - 1, k1, k0, v0);
        // next block's ring slots: tile NT of this stream
        ks = k1;
        vs = v0 ^ 1;
        FA_P4_STAMP(7, -1);

        // ---- epilogue: O / l through the wave's staging image, l and m ----
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
        FA_P4_STAMP(8, -1);
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
