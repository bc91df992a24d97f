// membw2.hip -- ceiling study for the 2-read + 1-write fp64 stream (24 B/cell) of the sweeps:
// unrolled grid-stride (U independent 16-B loads of each input in flight per lane), with and
// without non-temporal loads / stores, at 4096^2 (402 MB, partly Infinity-Cache resident) and
// 8192^2 (1.6 GB, HBM).  hipcc --offload-arch=gfx950 -O3 -o tools/membw2 tools/membw2.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_flat(const double2* __restrict__ a, const double2* __restrict__ b,
                                              double2* __restrict__ c, size_t n2) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i0 = blockIdx.x * 256 + threadIdx.x; i0 < n2; i0 += stride * U) {
        double2 x[U], y[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t i = i0 + k * stride;
            if (i < n2) {
                if (NTL) {
                    x[k].x = __builtin_nontemporal_load(&a[i].x); x[k].y = __builtin_nontemporal_load(&a[i].y);
                    y[k].x = __builtin_nontemporal_load(&b[i].x); y[k].y = __builtin_nontemporal_load(&b[i].y);
                } else { x[k] = a[i]; y[k] = b[i]; }
            }
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t i = i0 + k * stride;
            if (i < n2) {
                const double2 r = make_double2(x[k].x + 0.5 * y[k].x, x[k].y + 0.5 * y[k].y);
                if (NTS) { __builtin_nontemporal_store(r.x, &c[i].x); __builtin_nontemporal_store(r.y, &c[i].y); }
                else c[i] = r;
            }
        }
    }
}

// copy (1R + 1W) for reference against the guide's 6.3 TB/s
template <int U>
__global__ __launch_bounds__(256) void k_copy(const double2* __restrict__ a, double2* __restrict__ c, size_t n2) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i0 = blockIdx.x * 256 + threadIdx.x; i0 < n2; i0 += stride * U) {
        double2 x[U];
#pragma unroll
        for (int k = 0; k < U; k++) { const size_t i = i0 + k * stride; if (i < n2) x[k] = a[i]; }
#pragma unroll
        for (int k = 0; k < U; k++) { const size_t i = i0 + k * stride; if (i < n2) c[i] = x[k]; }
    }
}

// (r5) K1's stream mix: read u, v, cu0, cv0 and write cu, cv (in place), ru, rv -- 4 reads + 4 writes of 16 B
// per lane (64 B/cell), non-temporal stores like k_rhs_s: the ceiling of K1's own access pattern
template <int U>
__global__ __launch_bounds__(256) void k_4r4w(const double2* __restrict__ u, const double2* __restrict__ v,
                                              double2* cu, double2* cv, double2* __restrict__ ru,
                                              double2* __restrict__ rv, size_t n2) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i0 = blockIdx.x * 256 + threadIdx.x; i0 < n2; i0 += stride * U) {
        double2 a[U], b[U], c[U], d[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t i = i0 + k * stride;
            if (i < n2) { a[k] = u[i]; b[k] = v[i]; c[k] = cu[i]; d[k] = cv[i]; }
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t i = i0 + k * stride;
            if (i < n2) {
                auto st = [](double2* p, double x, double y) {
                    __builtin_nontemporal_store(x, &p->x); __builtin_nontemporal_store(y, &p->y);
                };
                st(&cu[i], a[k].x + c[k].x, a[k].y + c[k].y);
                st(&cv[i], b[k].x + d[k].x, b[k].y + d[k].y);
                st(&ru[i], a[k].x - d[k].x, a[k].y - d[k].y);
                st(&rv[i], b[k].x - c[k].x, b[k].y - c[k].y);
            }
        }
    }
}

// (r5) K5's stream mix: read phi, u*, v*, write u, v -- 3 reads + 2 writes of 16 B per lane (40 B/cell)
template <int U, bool NTS>
__global__ __launch_bounds__(256) void k_3r2w(const double2* __restrict__ p, const double2* __restrict__ us,
                                              const double2* __restrict__ vs, double2* __restrict__ u,
                                              double2* __restrict__ v, size_t n2) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i0 = blockIdx.x * 256 + threadIdx.x; i0 < n2; i0 += stride * U) {
        double2 a[U], b[U], c[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t i = i0 + k * stride;
            if (i < n2) { a[k] = p[i]; b[k] = us[i]; c[k] = vs[i]; }
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t i = i0 + k * stride;
            if (i < n2) {
                const double2 x = make_double2(b[k].x - 0.5 * a[k].x, b[k].y - 0.5 * a[k].y);
                const double2 y = make_double2(c[k].x - 0.5 * a[k].y, c[k].y - 0.5 * a[k].x);
                if (NTS) {
                    __builtin_nontemporal_store(x.x, &u[i].x); __builtin_nontemporal_store(x.y, &u[i].y);
                    __builtin_nontemporal_store(y.x, &v[i].x); __builtin_nontemporal_store(y.y, &v[i].y);
                } else { u[i] = x; v[i] = y; }
            }
        }
    }
}

// (r6) the guide's copy pattern (MI355X_MICROARCH.md: 6.29 TB/s "float4 copy"): one 16-B
// element per thread, a grid of n / 256 workgroups (no grid-stride loop), plain and non-temporal stores
template <bool NTS>
__global__ __launch_bounds__(256) void k_copy1(const double2* __restrict__ a, double2* __restrict__ c, size_t n2) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n2) {
        const double2 x = a[i];
        if (NTS) { __builtin_nontemporal_store(x.x, &c[i].x); __builtin_nontemporal_store(x.y, &c[i].y); }
        else c[i] = x;
    }
}
// (r6) K1 with K5 folded in (k_rhs_sc): read u*, v*, phi, cu, cv, write u, v, cu, cv, ru, rv -- 5 reads + 6 writes of
// 16 B per lane (88 B/cell), non-temporal stores like the kernel
template <int U>
__global__ __launch_bounds__(256) void k_5r6w(const double2* __restrict__ us, const double2* __restrict__ vs,
                                              const double2* __restrict__ ph, double2* cu, double2* cv,
                                              double2* __restrict__ u, double2* __restrict__ v, double2* __restrict__ ru,
                                              double2* __restrict__ rv, size_t n2) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i0 = blockIdx.x * 256 + threadIdx.x; i0 < n2; i0 += stride * U) {
        double2 a[U], b[U], c[U], d[U], e[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t i = i0 + k * stride;
            if (i < n2) { a[k] = us[i]; b[k] = vs[i]; c[k] = ph[i]; d[k] = cu[i]; e[k] = cv[i]; }
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t i = i0 + k * stride;
            if (i < n2) {
                auto st = [](double2* p, double x, double y) {
                    __builtin_nontemporal_store(x, &p->x); __builtin_nontemporal_store(y, &p->y);
                };
                st(&u[i], a[k].x - c[k].x, a[k].y - c[k].y);
                st(&v[i], b[k].x - c[k].y, b[k].y - c[k].x);
                st(&cu[i], a[k].x + d[k].x, a[k].y + d[k].y);
                st(&cv[i], b[k].x + e[k].x, b[k].y + e[k].y);
                st(&ru[i], a[k].x - e[k].x, a[k].y - e[k].y);
                st(&rv[i], b[k].x - d[k].x, b[k].y - d[k].y);
            }
        }
    }
}

// (r6) the strip walk of the streaming kernels (K1 / K5 / the sweeps): each wave owns a 64-lane x 16-B column strip
// (1 KiB of a row) and walks L rows with SK rows in flight; the workgroup's 4 waves take 4 adjacent strips (4 KiB of
// each row) -- a copy in that order, against the one-shot copy above
template <int SK>
__global__ __launch_bounds__(256) void k_strip_copy(const double2* __restrict__ a, double2* __restrict__ c, int ld2,
                                                    int nsj, int L, int rows) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nwj = nsj / 4;
    const int run = blockIdx.x / nwj, sj = (blockIdx.x % nwj) * 4 + wave;
    const size_t col = (size_t)sj * 64 + lane;
    const int r0 = run * L, r1 = min(r0 + L, rows);
    double2 q[SK];
#pragma unroll
    for (int k = 0; k < SK; k++) q[k] = r0 + k < r1 ? a[(size_t)(r0 + k) * ld2 + col] : make_double2(0, 0);
    for (int r = r0; r < r1; r += SK) {
#pragma unroll
        for (int k = 0; k < SK; k++) {
            if (r + k < r1) c[(size_t)(r + k) * ld2 + col] = q[k];
            if (r + k + SK < r1) q[k] = a[(size_t)(r + k + SK) * ld2 + col];
        }
    }
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "strip") {   // (r6) strip-walk copies at 4096^2 .. 16384^2
        for (int n : {4096, 8192, 16384}) {
            const size_t N = (size_t)n * n;
            double *a, *c;
            hipMalloc(&a, N * 8); hipMalloc(&c, N * 8);
            hipMemset(a, 0, N * 8); hipMemset(c, 0, N * 8);
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            auto timeit = [&](auto launch, const std::string& name) {
                for (int w = 0; w < 5; w++) launch();
                std::vector<float> ts;
                for (int it = 0; it < 20; it++) {
                    hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
                    float ms; hipEventElapsedTime(&ms, e0, e1); ts.push_back(ms);
                }
                std::sort(ts.begin(), ts.end());
                printf("n=%d %-34s median %8.1f us  %7.1f GB/s (16 B/cell)\n", n, name.c_str(), ts[10] * 1e3,
                       16.0 * N / (ts[10] * 1e-3) / 1e9);
            };
            const int ld2 = n / 2, nsj = ld2 / 64;
            const unsigned g1 = (unsigned)((N / 2 + 255) / 256);
            timeit([&] { hipLaunchKernelGGL((k_copy1<false>), dim3(g1), dim3(256), 0, 0, (const double2*)a, (double2*)c, N / 2); }, "copy one/thread");
            for (int L : {16, 64, 256}) {
                const int nb = (nsj / 4) * ((n + L - 1) / L);
                timeit([&] { hipLaunchKernelGGL((k_strip_copy<2>), dim3(nb), dim3(256), 0, 0, (const double2*)a, (double2*)c, ld2, nsj, L, n); }, "strip SK2 L=" + std::to_string(L));
                timeit([&] { hipLaunchKernelGGL((k_strip_copy<4>), dim3(nb), dim3(256), 0, 0, (const double2*)a, (double2*)c, ld2, nsj, L, n); }, "strip SK4 L=" + std::to_string(L));
            }
            hipFree(a); hipFree(c);
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "copy") {   // (r6) copy ceilings at 4096^2, 8192^2, 16384^2
        for (int n : {4096, 8192, 16384}) {
            const size_t N = (size_t)n * n;
            double *a, *c;
            hipMalloc(&a, N * 8); hipMalloc(&c, N * 8);
            hipMemset(a, 0, N * 8); hipMemset(c, 0, N * 8);
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            auto timeit = [&](auto launch, const std::string& name) {
                for (int w = 0; w < 5; w++) launch();
                std::vector<float> ts;
                for (int it = 0; it < 20; it++) {
                    hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
                    float ms; hipEventElapsedTime(&ms, e0, e1); ts.push_back(ms);
                }
                std::sort(ts.begin(), ts.end());
                printf("n=%d %-34s median %8.1f us  %7.1f GB/s (16 B/cell)\n", n, name.c_str(), ts[10] * 1e3,
                       16.0 * N / (ts[10] * 1e-3) / 1e9);
            };
            const unsigned g1 = (unsigned)((N / 2 + 255) / 256);
            timeit([&] { hipLaunchKernelGGL((k_copy1<false>), dim3(g1), dim3(256), 0, 0, (const double2*)a, (double2*)c, N / 2); }, "copy one/thread");
            timeit([&] { hipLaunchKernelGGL((k_copy1<true>), dim3(g1), dim3(256), 0, 0, (const double2*)a, (double2*)c, N / 2); }, "copy one/thread ntstore");
            for (int g : {2048, 8192, 32768}) {
                auto G = std::to_string(g);
                timeit([&] { hipLaunchKernelGGL((k_copy<1>), dim3(g), dim3(256), 0, 0, (const double2*)a, (double2*)c, N / 2); }, "copy U1 grid=" + G);
                timeit([&] { hipLaunchKernelGGL((k_copy<4>), dim3(g), dim3(256), 0, 0, (const double2*)a, (double2*)c, N / 2); }, "copy U4 grid=" + G);
            }
            hipFree(a); hipFree(c);
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "k1c") {   // (r6) K1 + K5's 5-read / 6-write mix
        for (int n : {4096, 8192}) {
            const size_t N = (size_t)n * n;
            double* f[9];
            for (auto& x : f) { hipMalloc(&x, N * 8); hipMemset(x, 0, N * 8); }
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            for (int g : {2048, 4096, 8192}) {
                auto launch = [&] {
                    hipLaunchKernelGGL((k_5r6w<2>), dim3(g), dim3(256), 0, 0, (const double2*)f[0], (const double2*)f[1],
                                       (const double2*)f[2], (double2*)f[3], (double2*)f[4], (double2*)f[5], (double2*)f[6],
                                       (double2*)f[7], (double2*)f[8], N / 2);
                };
                for (int w = 0; w < 5; w++) launch();
                std::vector<float> ts;
                for (int it = 0; it < 20; it++) {
                    hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
                    float ms; hipEventElapsedTime(&ms, e0, e1); ts.push_back(ms);
                }
                std::sort(ts.begin(), ts.end());
                printf("n=%d 5R6W (K1+K5 mix, nt stores) grid=%d median %8.1f us  %7.1f GB/s (88 B/cell)\n", n, g,
                       ts[10] * 1e3, 88.0 * N / (ts[10] * 1e-3) / 1e9);
            }
            for (auto x : f) hipFree(x);
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "k5") {   // K5's 3-read / 2-write mix at 4096^2 and 8192^2
        for (int n : {4096, 8192}) {
            const size_t N = (size_t)n * n;
            double* f[5];
            for (auto& x : f) { hipMalloc(&x, N * 8); hipMemset(x, 0, N * 8); }
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            auto timeit = [&](auto launch, const char* name, int g) {
                for (int w = 0; w < 5; w++) launch();
                std::vector<float> ts;
                for (int it = 0; it < 20; it++) {
                    hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
                    float ms; hipEventElapsedTime(&ms, e0, e1); ts.push_back(ms);
                }
                std::sort(ts.begin(), ts.end());
                printf("n=%d 3R2W %-10s grid=%d median %8.1f us  %7.1f GB/s (40 B/cell)\n", n, name, g, ts[10] * 1e3,
                       40.0 * N / (ts[10] * 1e-3) / 1e9);
            };
            for (int g : {2048, 4096, 8192}) {
                timeit([&] { hipLaunchKernelGGL((k_3r2w<2, false>), dim3(g), dim3(256), 0, 0, (const double2*)f[0], (const double2*)f[1], (const double2*)f[2], (double2*)f[3], (double2*)f[4], N / 2); }, "plain", g);
                timeit([&] { hipLaunchKernelGGL((k_3r2w<2, true>), dim3(g), dim3(256), 0, 0, (const double2*)f[0], (const double2*)f[1], (const double2*)f[2], (double2*)f[3], (double2*)f[4], N / 2); }, "ntstore", g);
            }
            for (auto x : f) hipFree(x);
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "k1") {   // K1's 4-read / 4-write mix at 4096^2 and 8192^2
        for (int n : {4096, 8192}) {
            const size_t N = (size_t)n * n;
            double* f[6];
            for (auto& x : f) { hipMalloc(&x, N * 8); hipMemset(x, 0, N * 8); }
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            for (int g : {2048, 4096, 8192}) {
                for (int w = 0; w < 5; w++)
                    hipLaunchKernelGGL((k_4r4w<2>), dim3(g), dim3(256), 0, 0, (const double2*)f[0], (const double2*)f[1],
                                       (double2*)f[2], (double2*)f[3], (double2*)f[4], (double2*)f[5], N / 2);
                std::vector<float> ts;
                for (int it = 0; it < 20; it++) {
                    hipEventRecord(e0);
                    hipLaunchKernelGGL((k_4r4w<2>), dim3(g), dim3(256), 0, 0, (const double2*)f[0], (const double2*)f[1],
                                       (double2*)f[2], (double2*)f[3], (double2*)f[4], (double2*)f[5], N / 2);
                    hipEventRecord(e1); hipEventSynchronize(e1);
                    float ms; hipEventElapsedTime(&ms, e0, e1); ts.push_back(ms);
                }
                std::sort(ts.begin(), ts.end());
                printf("n=%d 4R4W (K1 mix, nt stores) grid=%d median %8.1f us  %7.1f GB/s (64 B/cell)\n", n, g,
                       ts[10] * 1e3, 64.0 * N / (ts[10] * 1e-3) / 1e9);
            }
            for (auto x : f) hipFree(x);
        }
        return 0;
    }
    for (int n : {4096, 8192, 16384}) {
        const size_t N = (size_t)n * n;
        double *a, *b, *c;
        hipMalloc(&a, N * 8); hipMalloc(&b, N * 8); hipMalloc(&c, N * 8);
        hipMemset(a, 0, N * 8); hipMemset(b, 0, N * 8); hipMemset(c, 0, N * 8);
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        auto timeit = [&](auto launch, const std::string& name, double bytes_per_cell) {
            for (int w = 0; w < 5; w++) launch();
            std::vector<float> ts;
            for (int it = 0; it < 20; it++) {
                hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1); ts.push_back(ms);
            }
            std::sort(ts.begin(), ts.end());
            printf("n=%d %-34s median %8.1f us  %7.1f GB/s\n", n, name.c_str(), ts[10] * 1e3,
                   bytes_per_cell * N / (ts[10] * 1e-3) / 1e9);
        };
        for (int g : {1024, 2048, 4096}) {
            auto G = std::to_string(g);
            timeit([&] { hipLaunchKernelGGL((k_flat<1, false, false>), dim3(g), dim3(256), 0, 0, (const double2*)a, (const double2*)b, (double2*)c, N / 2); }, "2R1W U1 grid=" + G, 24);
            timeit([&] { hipLaunchKernelGGL((k_flat<4, false, false>), dim3(g), dim3(256), 0, 0, (const double2*)a, (const double2*)b, (double2*)c, N / 2); }, "2R1W U4 grid=" + G, 24);
            timeit([&] { hipLaunchKernelGGL((k_flat<4, false, true>), dim3(g), dim3(256), 0, 0, (const double2*)a, (const double2*)b, (double2*)c, N / 2); }, "2R1W U4 ntstore grid=" + G, 24);
            timeit([&] { hipLaunchKernelGGL((k_flat<4, true, true>), dim3(g), dim3(256), 0, 0, (const double2*)a, (const double2*)b, (double2*)c, N / 2); }, "2R1W U4 ntload+ntstore grid=" + G, 24);
            timeit([&] { hipLaunchKernelGGL((k_copy<4>), dim3(g), dim3(256), 0, 0, (const double2*)a, (double2*)c, N / 2); }, "copy U4 grid=" + G, 16);
        }
        hipFree(a); hipFree(b); hipFree(c);
    }
    return 0;
}
