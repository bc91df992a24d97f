// membw.hip -- achievable-bandwidth ceilings on this MI355X for the sweep's access
// pattern: read 2 planes + write 1 plane of fp64 (24 B/cell), 16 B per lane.
//   (a) flat grid-stride stream (best case), (b) row-walking strips like k_sweep.
// hipcc --offload-arch=gfx950 -O3 -o tools/membw tools/membw.hip && ./tools/membw 4096
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

__global__ __launch_bounds__(256) void k_flat(const double2* __restrict__ a, const double2* __restrict__ b,
                                              double2* __restrict__ c, size_t n2) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
        double2 x = a[i], y = b[i];
        c[i] = make_double2(x.x + 0.5 * y.x, x.y + 0.5 * y.y);
    }
}

template <int SD>
__global__ __launch_bounds__(256) void k_strip(const double* __restrict__ a, const double* __restrict__ b,
                                               double* __restrict__ c, int nx, int ld, int L) {
    const int lane = threadIdx.x & 63, wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nsj = ld / 128, nsi = (nx + L - 1) / L;
    if (wid >= nsj * nsi) return;
    const int si = wid / nsj, sj = wid % nsj, jb = sj * 128, ib = si * L, ie = min(ib + L, nx);
    double2 Q[SD], QB[SD];
    auto load = [&](int r, double2& p, double2& q) {
        r = min(r, nx - 1);
        p = *reinterpret_cast<const double2*>(a + (size_t)r * ld + jb + 2 * lane);
        q = *reinterpret_cast<const double2*>(b + (size_t)r * ld + jb + 2 * lane);
    };
#pragma unroll
    for (int q = 0; q < SD; q++) load(ib + q, Q[q], QB[q]);
    for (int r = ib; r < ie; r += SD) {
#pragma unroll
        for (int q = 0; q < SD; q++) {
            if (r + q < ie)
                *reinterpret_cast<double2*>(c + (size_t)(r + q) * ld + jb + 2 * lane) =
                    make_double2(Q[q].x + 0.5 * QB[q].x, Q[q].y + 0.5 * QB[q].y);
            load(r + q + SD, Q[q], QB[q]);
        }
    }
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 4096;
    const size_t N = (size_t)n * n;
    double *a, *b, *c;
    hipMalloc(&a, N * 8); hipMalloc(&b, N * 8); hipMalloc(&c, N * 8);
    hipMemset(a, 0, N * 8); hipMemset(b, 0, N * 8); hipMemset(c, 0, N * 8);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto timeit = [&](auto launch, const char* name) {
        for (int w = 0; w < 5; w++) launch();
        std::vector<float> ts;
        for (int it = 0; it < 20; it++) {
            hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-28s median %8.1f us  %7.1f GB/s (24 B/cell)\n", name, ts[10] * 1e3, 24.0 * N / (ts[10] * 1e-3) / 1e9);
    };
    for (int g : {1024, 2048, 4096, 8192})
        timeit([&] { hipLaunchKernelGGL(k_flat, dim3(g), dim3(256), 0, 0, (const double2*)a, (const double2*)b, (double2*)c, N / 2); },
               (std::string("flat grid=") + std::to_string(g)).c_str());
    for (int L : {8, 16, 32, 64, 128}) {
        const int nw = (n / 128) * ((n + L - 1) / L);
        timeit([&] { hipLaunchKernelGGL(k_strip<4>, dim3((nw + 3) / 4), dim3(256), 0, 0, a, b, c, n, n, L); },
               (std::string("strip SD=4 L=") + std::to_string(L)).c_str());
        timeit([&] { hipLaunchKernelGGL(k_strip<8>, dim3((nw + 3) / 4), dim3(256), 0, 0, a, b, c, n, n, L); },
               (std::string("strip SD=8 L=") + std::to_string(L)).c_str());
    }
    return 0;
}
