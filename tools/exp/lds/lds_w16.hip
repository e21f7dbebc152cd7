// Microbenchmark: LDS write cost of ds_write_b16 with adjacent lanes writing the two halves of
// one dword (the strip images' pattern) vs ds_write_b16 to distinct dwords vs ds_write_b32.
// One workgroup of 512 threads per CU, every wave loops; cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ __launch_bounds__(512) void k(unsigned long long* out, int iters) {
    __shared__ __attribute__((aligned(16))) char sm[65536];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned a;
    if (MODE == 0) a = (wave * 8192) + lane * 2;            // b16, lanes 2i / 2i+1 share a dword
    else if (MODE <= 3) a = (wave * 8192) + lane * 4;       // b16 / b32 / or_b32, one dword per lane
    else if (MODE == 4 || MODE == 7 || MODE == 8) a = (wave * 1024) + lane * 8;   // b64 / tr_b16 reads
    else a = (wave * 8192) + lane * 16;                     // b128 (wraps within 8 KB per wave: offsets below)
    unsigned v = threadIdx.x;
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    u4 v4 = {v, v, v, v};
    u2 v2 = {v, v};
    u4 acc4 = {0u, 0u, 0u, 0u};
    u2 acc2 = {0u, 0u};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (MODE == 2) asm volatile("ds_write_b32 %0, %1 offset:%2" : : "v"(a), "v"(v), "i"(j * 512) : "memory");
            else if (MODE == 3) asm volatile("ds_or_b32 %0, %1 offset:%2" : : "v"(a), "v"(v), "i"(j * 512) : "memory");
            else if (MODE == 4) asm volatile("ds_write_b64 %0, %1 offset:%2" : : "v"(a), "v"(v2), "i"((j & 7) * 512) : "memory");
            else if (MODE == 5) asm volatile("ds_write_b128 %0, %1 offset:%2" : : "v"(a & 8191), "v"(v4), "i"((j & 3) * 16384) : "memory");
            else if (MODE == 6) { u4 r; asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a & 8191), "i"((j & 3) * 16384) : "memory"); acc4 += r; }
            else if (MODE == 7) { u2 r; asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a & 8191), "i"((j & 7) * 8192) : "memory"); acc2 += r; }
            else if (MODE == 8) { u2 r; asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r) : "v"(a & 8191), "i"((j & 7) * 8192) : "memory"); acc2 += r; }
            else asm volatile("ds_write_b16 %0, %1 offset:%2" : : "v"(a), "v"(v), "i"(j * 512) : "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) out[blockIdx.x * 8 + wave] = t1 - t0;
    if (threadIdx.x == 0) out[256 * 8 + blockIdx.x] = r1 - r0;   // 100-MHz ticks
    if (acc4[0] + acc4[1] + acc4[2] + acc4[3] + acc2[0] + acc2[1] == 0xFFFFFFFFu) out[0] = 0;   // keep the reads
}
int main() {
    unsigned long long* d; hipMalloc(&d, 256 * 9 * 8);
    unsigned long long h[256 * 9];
    const int iters = 2000;
    const char* names[9] = {"b16 two lanes per dword", "b16 one dword per lane", "b32 one dword per lane",
                            "or_b32 one dword per lane", "b64", "b128", "read b128", "read b64_tr_b16", "read b64"};
    const int bytes[9] = {128, 128, 256, 256, 512, 1024, 1024, 512, 512};
    for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 9; ++m) {
        if (m == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(512), 0, 0, d, iters);
        if (m == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(512), 0, 0, d, iters);
        if (m == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(512), 0, 0, d, iters);
        if (m == 3) hipLaunchKernelGGL(k<3>, dim3(256), dim3(512), 0, 0, d, iters);
        if (m == 4) hipLaunchKernelGGL(k<4>, dim3(256), dim3(512), 0, 0, d, iters);
        if (m == 5) hipLaunchKernelGGL(k<5>, dim3(256), dim3(512), 0, 0, d, iters);
        if (m == 6) hipLaunchKernelGGL(k<6>, dim3(256), dim3(512), 0, 0, d, iters);
        if (m == 7) hipLaunchKernelGGL(k<7>, dim3(256), dim3(512), 0, 0, d, iters);
        if (m == 8) hipLaunchKernelGGL(k<8>, dim3(256), dim3(512), 0, 0, d, iters);
        hipDeviceSynchronize();
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        double s = 0; for (int i = 0; i < 256 * 8; ++i) s += h[i];
        s /= 256 * 8;
        // memtime ticks at the shader clock on gfx9 (s_memtime): cycles per wave per instruction,
        // and per CU (8 waves share the LDS)
        const double cu = s / (iters * 16.0 * 8);
        double rt = 0; for (int i = 0; i < 256; ++i) rt += h[256 * 8 + i];
        rt /= 256;
        printf("  (memtime %.0f ticks over %.1f us: %.0f MHz)\n", s, rt / 100.0, s / (rt / 100.0));
        printf("%-26s: %.2f cycles per wave-instruction (%.2f per CU-instruction, %.1f B/clk per CU)\n", names[m], s / (iters * 16.0), cu, bytes[m] / cu);
    }
    return 0;
}
