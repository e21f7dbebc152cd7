// fa_common.h — device-side helpers shared by the gfx950 flash-attention kernels.
//
// Data layout in HBM (all kernels): the reference's Julia column-major
// (N, d, B) arrays, i.e. per batch slab b a row-major [d][N] matrix whose
// rows are FEATURES and whose columns are TOKENS (tokens contiguous).
// src/dense.jl:6-8 reshapes every input to this form.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fa {

typedef __bf16 bf16;
typedef _Float16 f16;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

typedef __attribute__((address_space(3))) void lds_void;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNegInf = -__builtin_huge_valf();

template <class T> struct Frag8;
template <> struct Frag8<bf16> { typedef bf16x8 type; typedef bf16x4 half; };
template <> struct Frag8<f16>  { typedef f16x8 type;  typedef f16x4 half; };

__device__ __forceinline__ f32x16 mfma32x32x16(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32x32x16(f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32x32x2(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Raw v_exp_f32 (2^x); exp2(-inf) = 0.
__device__ __forceinline__ float exp2_fast(float x) { return __builtin_amdgcn_exp2f(x); }

// IEEE-2019 maximum (v_maximum3_f32 on gfx950): NaN-propagating like Julia's
// `maximum`, and unlike fmaxf it needs no NaN-canonicalising `v_max_f32 x, x, x`
// per MFMA-result operand.
__device__ __forceinline__ float vmax(float a, float b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ float vmax3(float a, float b, float c) { return vmax(vmax(a, b), c); }

// Max over the NB x 16 scores a lane holds: four interleaved v_maximum3 chains.
template <int NB>
__device__ __forceinline__ float lane_max(const f32x16 (&s)[NB]) {
    static_assert(NB * 16 >= 12 && (NB * 16 - 12) % 2 == 0, "lane_max");
    float a[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) a[c] = vmax3(s[0][3 * c], s[0][3 * c + 1], s[0][3 * c + 2]);
#pragma unroll
    for (int k = 12, c = 0; k < NB * 16; k += 2, c = (c + 1) & 3)
        a[c] = vmax3(a[c], s[k >> 4][k & 15], s[(k + 1) >> 4][(k + 1) & 15]);
    return vmax(vmax3(a[0], a[1], a[2]), a[3]);
}

// Value of x held by lane (l ^ 32): v_permlane32_swap on a copy.
__device__ __forceinline__ float swap_halves_max(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return vmax(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float swap_halves_sum(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p supplies row q / 4-column
// chunk p of a 4x16 block; lane i receives column i, row q in element q.
__device__ __forceinline__ s16x4 ds_read_tr16(const char* lds_ptr) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(lds_void*)lds_ptr);
}

// Row index (0..31) of accumulator register rho of a 32x32 MFMA tile for lane
// half h: row = (rho&3) + 8*(rho>>2) + 4*h  (C/D map, cdna_hip_programming §3).
__device__ __forceinline__ constexpr int acc_row(int rho, int h) {
    return (rho & 3) + 8 * (rho >> 2) + 4 * h;
}

// Blocks b and b+8 run on one XCD (round-robin dispatch; speed only, never
// correctness).  Bijective remap so that consecutive LOGICAL ids — which share
// a batch slab's K/V — land on one XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int n) {
    const int q = n >> 3, r = n & 7, xcd = bid & 7, loc = bid >> 3;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// Lazy-rescale threshold (log2 units) of the online softmax: the running max
// used for the exponentials is raised only when a tile exceeds it by more than
// this, so P <= 2^kRescaleLog2 and the O/l rescale is a rare uniform branch.
constexpr float kRescaleLog2 = 8.0f;

// Buffer descriptor over one slab: out-of-range offsets read as 0.
template <class T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab_rsrc(const T* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

template <class T> __device__ __forceinline__ T zero_val() { return (T)0.0f; }

}  // namespace fa
