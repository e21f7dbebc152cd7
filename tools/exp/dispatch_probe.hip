// Workgroup dispatch probe: grids of workgroups that each hold LDS and spin for a fixed
// time (s_memrealtime, 100 MHz), timed with hipEvents.  If the kernel takes longer than
// waves-of-workgroups x spin time, the dispatcher (not the work) limits occupancy.
// Build: hipcc -O3 --offload-arch=gfx950 tools/exp/dispatch_probe.hip -o tools/exp/dispatch_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int THREADS, int LDS>
__global__ __launch_bounds__(THREADS) void spin(int ticks, int* out) {
    __shared__ char buf[LDS];
    buf[threadIdx.x * 16 % LDS] = (char)threadIdx.x;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)ticks) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0 && buf[(threadIdx.x + 1) * 16 % LDS] == 127) out[blockIdx.x] = 1;
}

template <int THREADS, int LDS>
static void run(const char* name, int grid, int us, int per_cu, int* out) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int ticks = us * 100;
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((spin<THREADS, LDS>), dim3(grid), dim3(THREADS), 0, 0, ticks, out);
    hipDeviceSynchronize();
    std::vector<float> ts;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(a);
        hipLaunchKernelGGL((spin<THREADS, LDS>), dim3(grid), dim3(THREADS), 0, 0, ticks, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); ts.push_back(ms * 1000.0f);
    }
    float best = ts[0]; for (float t : ts) best = t < best ? t : best;
    const double rounds = (double)grid / (256.0 * per_cu);
    printf("%-34s grid %5d x %4d thr, LDS %6d B, spin %2d us: %7.1f us (ideal %.2f rounds x spin = %6.1f us)\n", name, grid,
           THREADS, LDS, us, best, rounds, rounds * us);
}

int main() {
    int* out; hipMalloc(&out, 1 << 20);
    run<512, 65536>("win_strip-like (2/CU)", 1824, 13, 2, out);
    run<512, 65536>("win_strip-like, 6.5 us", 1824, 6, 2, out);
    run<512, 65536>("512 WGs (one round)", 512, 13, 2, out);
    run<256, 32768>("256 thr, 4/CU", 3648, 13, 4, out);
    run<512, 155648>("win_bwd_strip-like (1/CU)", 256, 20, 1, out);
    run<512, 131072>("bwd_fused-like (1/CU)", 2048, 50, 1, out);
    run<512, 102400>("dense fwd-like (1/CU)", 512, 130, 1, out);
    return 0;
}
