// Store-pattern micro-benchmark for the windowed forward's y (128 x 128 px, 64
// features, B images, bf16; ws 7, stride 7, pad 3 windows).  Timing only.
//   P1: the windowed kernel's pattern: per window, 64 lanes = 32 query slots
//       (4 slot rows x 8) x 2 feature halves, 2-B stores, 16 per lane per
//       32-feature chunk (4 waves per window, 2 windows per 512-thread WG);
//   P2: the same bytes as 16-B stores, 8 pixels of one (feature, row) per lane;
//   P3: per window, 2-B stores with lanes along x: lane -> (feature, row, pixel)
//       with the window's 7 pixels contiguous (9 segments per instruction).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/exp/store_pattern tools/exp/store_pattern.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

constexpr int W = 128, H = 128, C = 64, WS = 7, ST = 7, PAD = 3, OW = 19;

__global__ __launch_bounds__(512) void p1(unsigned short* y, int nwin) {
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5, wave = tid >> 6;
    const int wid = blockIdx.x * 2 + (wave >> 2);
    if (wid >= nwin) return;
    const int b = wid / (OW * OW), rem = wid % (OW * OW), wy = rem / OW, wx = rem % OW;
    const int xs = wx * ST - PAD, y0 = wy * ST - PAD;
    const int qb = wave & 1, vc = (wave >> 1) & 1;
    const int qslot = qb * 32 + r, qtx = qslot & 7, qty = qslot >> 3;
    const int px = xs + qtx, py = y0 + qty;
    if (qtx < WS && qty < WS && px >= 0 && px < W && py >= 0 && py < H) {
        unsigned short* yb = y + (size_t)b * C * W * H + (size_t)py * W + px;
#pragma unroll
        for (int x = 0; x < 16; ++x) {
            const int cc = vc * 32 + (x & 3) + 8 * (x >> 2) + 4 * h;
            yb[(size_t)cc * W * H] = (unsigned short)(x + wid);
        }
    }
}

__global__ __launch_bounds__(256) void p2(uint4* y, size_t nchunks) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < nchunks; i += (size_t)gridDim.x * 256)
        y[i] = make_uint4(i, i, i, i);
}

// P3: one 256-thread WG per window; items (feature f, row j, pixel t): 64 x 7 x 7,
// lanes along t then j then f: each instruction covers 64 consecutive items
__global__ __launch_bounds__(256) void p3(unsigned short* y, int nwin) {
    const int wid = blockIdx.x;
    const int b = wid / (OW * OW), rem = wid % (OW * OW), wy = rem / OW, wx = rem % OW;
    const int xs = wx * ST - PAD, y0 = wy * ST - PAD;
    for (int it = threadIdx.x; it < C * WS * WS; it += 256) {
        const int t = it % WS, j = (it / WS) % WS, f = it / (WS * WS);
        const int px = xs + t, py = y0 + j;
        if (px >= 0 && px < W && py >= 0 && py < H)
            y[(size_t)b * C * W * H + (size_t)f * W * H + (size_t)py * W + px] = (unsigned short)it;
    }
}

// P4/P5/P6: exact own pixels of each window row as one b96 + one b16 store per
// (feature, row) item; NI windows interleaved on adjacent lanes (1, 2, 8).
template <int NI>
__global__ __launch_bounds__(256) void p_rows(unsigned short* y, int nwin) {
    // workgroup: NI windows x 448 items; lane order: window fastest
    const int wbase = blockIdx.x * NI;
    for (int it = threadIdx.x; it < NI * C * WS; it += 256) {
        const int wl = it % NI, item = it / NI, j = item % WS, f = item / WS;
        const int wid = wbase + wl;
        if (wid >= nwin) continue;
        const int b = wid / (OW * OW), rem = wid % (OW * OW), wy = rem / OW, wx = rem % OW;
        const int xs = wx * ST - PAD, py = wy * ST - PAD + j;
        if (py < 0 || py >= H || xs < 0 || xs + WS > W) continue;   // interior windows only (timing)
        unsigned short* row = y + (size_t)b * C * W * H + (size_t)f * W * H + (size_t)py * W;
        if (xs & 1) {
            row[xs] = (unsigned short)it;
            *(uint3*)(row + xs + 1) = make_uint3(it, it, it);
        } else {
            *(uint3*)(row + xs) = make_uint3(it, it, it);
            row[xs + 6] = (unsigned short)it;
        }
    }
}

__global__ __launch_bounds__(256) void p7(unsigned* y, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) y[i] = (unsigned)i;
}

// P8: 16-B stores, lane -> (feature, row) line, one 16-B chunk per instruction
// (64 lines per instruction); a workgroup covers 64 (feature,row) lines x 16 chunks
__global__ __launch_bounds__(256) void p8(uint4* y, size_t nlines) {
    const size_t l0 = (size_t)blockIdx.x * 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int ch = wave; ch < 16; ch += 4) {
        const size_t line = l0 + lane;
        if (line < nlines) y[line * 16 + ch] = make_uint4(ch, ch, ch, ch);
    }
}

// P9: a window pair (2 windows per 512-thread WG, as P1): 16-B stores of the aligned
// chunks inside the pair's pixel span (lanes = (feature, row) per chunk), 2-B stores
// (P1's lane pattern) for the pair's remaining pixels
__global__ __launch_bounds__(512) void p9(unsigned short* y, int nwin) {
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5, wave = tid >> 6;
    const int w0 = blockIdx.x * 2;
    if (w0 + 1 >= nwin) return;
    const int b = w0 / (OW * OW), rem = w0 % (OW * OW), wy = rem / OW, wx = rem % OW;
    if (wx + 1 >= OW) return;                                     // pair in one row (timing only)
    const int xs = wx * ST - PAD, y0 = wy * ST - PAD;
    const int lo = xs < 0 ? 0 : xs, hi = min(xs + 2 * WS, W);   // pair's pixels [lo, hi)
    const int c0 = (lo + 7) >> 3, c1 = hi >> 3;                   // full chunks [c0, c1)
    // 16-B part: items (f, row j, chunk) over 512 threads
    const int nfull = c1 > c0 ? c1 - c0 : 0;
    for (int it = tid; it < C * WS * nfull; it += 512) {
        const int f = it % C, rest = it / C, j = rest % WS, c = c0 + rest / WS;
        const int py = y0 + j;
        if (py < 0 || py >= H) continue;
        *(uint4*)(y + (size_t)b * C * W * H + (size_t)f * W * H + (size_t)py * W + 8 * c) = make_uint4(it, it, it, it);
    }
    // 2-B part: P1's pattern, pixels outside the full chunks
    const int wl = wave >> 2, qb = wave & 1, vc = (wave >> 1) & 1;
    const int qslot = qb * 32 + r, qtx = qslot & 7, qty = qslot >> 3;
    const int px = xs + wl * WS + qtx, py = y0 + qty;
    const bool full = px >= 8 * c0 && px < 8 * c1;
    if (qtx < WS && qty < WS && px >= 0 && px < W && py >= 0 && py < H && !full) {
        unsigned short* yb = y + (size_t)b * C * W * H + (size_t)py * W + px;
#pragma unroll
        for (int x = 0; x < 16; ++x) {
            const int cc = vc * 32 + (x & 3) + 8 * (x >> 2) + 4 * h;
            yb[(size_t)cc * W * H] = (unsigned short)(x + w0);
        }
    }
}

// P10: 16-B stores, a workgroup writes 64-B half lines (SEG = 32 px) or whole lines
// (SEG = 64 px) of every (feature, row): lane -> (line, chunk), chunks fastest
template <int SEG>
__global__ __launch_bounds__(256) void p10(uint4* y, size_t nlines) {
    constexpr int CPL = SEG / 8;                       // 16-B chunks per segment
    const size_t seg0 = (size_t)blockIdx.x * 64;      // 64 segments per workgroup
    for (int it = threadIdx.x; it < 64 * CPL; it += 256) {
        const size_t sg = seg0 + it / CPL;            // segment index: (line, half)
        const int c = it % CPL;
        const size_t line = sg / (64 / SEG), part = sg % (64 / SEG);
        // interleave: consecutive workgroups write the two halves of a line
        if (line < nlines) y[line * 8 + part * CPL + c] = make_uint4(it, it, it, it);   // 8 chunks per 128-B line
    }
}

int main() {
    const int B = 32, nwin = OW * OW * B;
    const size_t bytes = (size_t)B * C * W * H * 2;
    unsigned short* y;
    hipMalloc(&y, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    auto time = [&](auto launch) {
        for (int i = 0; i < 50; ++i) launch();
        std::vector<float> ts;
        for (int rep = 0; rep < 7; ++rep) {
            hipEventRecord(e0);
            for (int i = 0; i < 20; ++i) launch();
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); ts.push_back(ms * 1000 / 20);
        }
        std::sort(ts.begin(), ts.end());
        return ts[3];
    };
    const float t1 = time([&] { hipLaunchKernelGGL(p1, dim3((nwin + 1) / 2), dim3(512), 0, 0, y, nwin); });
    const float t2 = time([&] { hipLaunchKernelGGL(p2, dim3(2048), dim3(256), 0, 0, (uint4*)y, bytes / 16); });
    const float t3 = time([&] { hipLaunchKernelGGL(p3, dim3(nwin), dim3(256), 0, 0, y, nwin); });
    const float t4 = time([&] { hipLaunchKernelGGL(p_rows<1>, dim3(nwin), dim3(256), 0, 0, y, nwin); });
    const float t5 = time([&] { hipLaunchKernelGGL(p_rows<2>, dim3((nwin + 1) / 2), dim3(256), 0, 0, y, nwin); });
    const float t6 = time([&] { hipLaunchKernelGGL(p_rows<8>, dim3((nwin + 7) / 8), dim3(256), 0, 0, y, nwin); });
    const float t7 = time([&] { hipLaunchKernelGGL(p7, dim3(2048), dim3(256), 0, 0, (unsigned*)y, bytes / 4); });
    const float t8 = time([&] { hipLaunchKernelGGL(p8, dim3((unsigned)(bytes / 256 / 64)), dim3(256), 0, 0, (uint4*)y, bytes / 256); });
    const float t9 = time([&] { hipLaunchKernelGGL(p9, dim3((nwin + 1) / 2), dim3(512), 0, 0, y, nwin); });
    const size_t nl = bytes / 128;
    const float t10a = time([&] { hipLaunchKernelGGL(p10<32>, dim3((unsigned)(nl * 2 / 64)), dim3(256), 0, 0, (uint4*)y, nl); });
    const float t10b = time([&] { hipLaunchKernelGGL(p10<64>, dim3((unsigned)(nl / 64)), dim3(256), 0, 0, (uint4*)y, nl); });
    printf("P10 16-B chunks, workgroup-owned half lines %.1f us, whole lines %.1f us\n", t10a, t10b);
    printf("P9 pair: 16-B owned chunks + 2-B rest %.1f us (pairs within one row only: ~%.0f %% of the bytes)\n", t9,
           100.0 * 18 / 19);
    printf("P8 16-B, 64 lines per instruction (a line completed over 16 instructions of 4 waves) %.1f us\n", t8);
    printf("P4 b96+b16 rows, 1 window per WG %.1f us; P5 2 windows interleaved %.1f us; P6 8 windows interleaved %.1f us "
           "(interior windows only: ~%.0f %% of the bytes); P7 4-B streaming %.1f us\n", t4, t5, t6,
           100.0 * 17 * 17 / (19 * 19), t7);
    printf("B=%d y %.1f MB: P1 windowed 2-B pattern %.1f us (%.0f GB/s); P2 16-B streaming %.1f us (%.0f GB/s); "
           "P3 2-B lanes along x %.1f us (%.0f GB/s)\n", B, bytes / 1e6, t1, bytes / t1 / 1e3, t2, bytes / t2 / 1e3,
           t3, bytes / t3 / 1e3);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
