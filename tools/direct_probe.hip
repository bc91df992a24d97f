// Phase timing of the coarsest-level direct solve kernel (k_direct, ns_kernels.hip) at 128^2:
// the same staging / MFMA / reduction structure with s_memtime stamps per phase (workgroup 0,
// thread 0), variants by template flag.  hipcc --offload-arch=gfx950 -O3 tools/direct_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double nsd4 __attribute__((ext_vector_type(4)));
constexpr int DM = 128;
__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
template <int MODE>   // 0 full, 1 staging only, 2 staging + step 1
__global__ __launch_bounds__(256) void kd(const double* __restrict__ P, const double* __restrict__ M,
                                          const double* __restrict__ Q, double* __restrict__ G, int n1p, int n2p,
                                          int ldm, unsigned long long* ts) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* Ms = sm;
    double* R2 = sm + n1p * n2p;
    unsigned long long t0 = stamp(), t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int bi = blockIdx.x, bj = blockIdx.y, r16 = lane & 15, k4 = lane >> 4;
    const int ps = n1p + 2, ts2 = n2p + 1;
    constexpr int QV = DM / 16;
    const int kq = n2p / 4, colq = 16 * bj + r16;
    double qv[QV];
#pragma unroll
    for (int q = 0; q < QV; q++) qv[q] = 4 * q < kq ? Q[(size_t)(w * kq + 4 * q + k4) * n2p + colq] : 0.0;
    {
        constexpr int NM = DM * DM / 256, NP = 16 * DM / 256;
        double mv[NM], pv[NP];
#pragma unroll
        for (int q = 0; q < NM; q++) { const int e = threadIdx.x + 256 * q; mv[q] = M[(size_t)(e / DM) * ldm + (e % DM)]; }
#pragma unroll
        for (int q = 0; q < NP; q++) { const int e = threadIdx.x + 256 * q; pv[q] = P[(size_t)16 * bi * n1p + e]; }
#pragma unroll
        for (int q = 0; q < NM; q++) { const int e = threadIdx.x + 256 * q, k = e / DM, c = e % DM; Ms[k * n2p + (c ^ ((k & 1) ? 16 : 0))] = mv[q]; }
#pragma unroll
        for (int q = 0; q < NP; q++) { const int e = threadIdx.x + 256 * q, r = e / DM, k = e % DM; R2[r * ps + k] = pv[q]; }
    }
    t1 = stamp();
    __syncthreads();
    t2 = stamp();
    if (MODE == 1) { if (threadIdx.x == 0 && bi == 0 && bj == 0) { ts[0] = t0; ts[1] = t1; ts[2] = t2; } G[threadIdx.x] = Ms[threadIdx.x] + qv[0]; return; }
    nsd4 acc[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    for (int k0 = 0; k0 < n1p; k0 += 4) {
        const int k = k0 + k4;
        const double av = R2[r16 * ps + k];
#pragma unroll
        for (int t = 0; t < 2; t++) {
            const int col = 16 * (w + 4 * t) + r16;
            acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, Ms[k * n2p + (col ^ ((k & 1) ? 16 : 0))], acc[t], 0, 0, 0);
        }
    }
    t3 = stamp();
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 2; t++) {
        const int col = 16 * (w + 4 * t) + r16;
#pragma unroll
        for (int r = 0; r < 4; r++) R2[(k4 + 4 * r) * ts2 + col] = acc[t][r];
    }
    __syncthreads();
    if (MODE == 2) { if (threadIdx.x == 0 && bi == 0 && bj == 0) { ts[0] = t0; ts[1] = t1; ts[2] = t2; ts[3] = t3; } G[threadIdx.x] = R2[threadIdx.x]; return; }
    nsd4 g4 = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < QV; q++) g4 = __builtin_amdgcn_mfma_f64_16x16x4f64(R2[r16 * ts2 + w * kq + 4 * q + k4], qv[q], g4, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; r++) Ms[w * 256 + (k4 + 4 * r) * 16 + r16] = g4[r];
    __syncthreads();
    t4 = stamp();
    const int t = threadIdx.x, gi = 16 * bi + (t >> 4), gj = 16 * bj + (t & 15);
    G[(size_t)gi * ldm + gj] = ((Ms[t] + Ms[256 + t]) + Ms[512 + t]) + Ms[768 + t];
    if (threadIdx.x == 0 && bi == 0 && bj == 0) { ts[0] = t0; ts[1] = t1; ts[2] = t2; ts[3] = t3; ts[4] = t4; ts[5] = stamp(); }
}
int main() {
    const int n = 128;
    double *P, *M, *Q, *G; unsigned long long* ts;
    hipMalloc(&P, n * n * 8); hipMalloc(&M, n * n * 8); hipMalloc(&Q, n * n * 8); hipMalloc(&G, n * n * 8);
    hipMalloc(&ts, 64);
    std::vector<double> h(n * n);
    for (int i = 0; i < n * n; i++) h[i] = 1.0 / (1 + i % 97);
    hipMemcpy(P, h.data(), n * n * 8, hipMemcpyHostToDevice); hipMemcpy(M, h.data(), n * n * 8, hipMemcpyHostToDevice);
    hipMemcpy(Q, h.data(), n * n * 8, hipMemcpyHostToDevice);
    const size_t bytes = (n * n + 16 * (n + 2)) * 8;
    hipFuncSetAttribute((const void*)kd<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)kd<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)kd<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int mode = 0; mode < 3; mode++) {
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(a);
            for (int k = 0; k < 20; k++) {
                if (mode == 0) kd<0><<<dim3(8, 8), 256, bytes>>>(P, M, Q, G, n, n, n, ts);
                if (mode == 1) kd<1><<<dim3(8, 8), 256, bytes>>>(P, M, Q, G, n, n, n, ts);
                if (mode == 2) kd<2><<<dim3(8, 8), 256, bytes>>>(P, M, Q, G, n, n, n, ts);
            }
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            unsigned long long t[6] = {}; hipMemcpy(t, ts, 48, hipMemcpyDeviceToHost);
            printf("mode %d: %.2f us/launch; stamps (100 MHz ticks? raw) issue %llu sync %llu step1 %llu step2 %llu end %llu\n", mode,
                   ms * 1000 / 20, t[1] - t[0], t[2] - t[1], t[3] ? t[3] - t[2] : 0, t[4] ? t[4] - t[3] : 0, t[5] ? t[5] - t[4] : 0);
        }
    }
    printf("err %s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
