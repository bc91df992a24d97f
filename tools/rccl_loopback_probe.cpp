// What a 1-rank RCCL communicator (the virtual slab's NSGPU_RCCL_LOOPBACK) launches per call:
// 10 x each of (a) ncclAllReduce of 4 doubles, (b) one group of send + recv to self of N bytes
// (a ghost-row exchange), (c) one group of 7 send / recv pairs to self (the agglomeration gather
// on 8 ranks), with a marker kernel between phases.  Run under rocprofv3 --kernel-trace to see
// which kernels / copies / fills each call costs.  Build:
//   hipcc --offload-arch=gfx950 -O2 tools/rccl_loopback_probe.cpp -lrccl -o tools/rccl_probe
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <cstdio>
#include <cstdlib>

__global__ void marker(int phase, double* d) { if (threadIdx.x == 0) d[0] += phase; }

#define CK(x) do { auto r_ = (x); if (r_ != 0) { printf("%s failed %d\n", #x, (int)r_); return 1; } } while (0)

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? (size_t)atol(argv[1]) : 20480;   // doubles per message (160 KB)
    ncclUniqueId id;
    ncclComm_t comm;
    CK(ncclGetUniqueId(&id));
    CK(ncclCommInitRank(&comm, 1, id, 0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    double *a, *b, *m;
    CK(hipMalloc(&a, 16 * n * sizeof(double)));
    CK(hipMalloc(&b, 16 * n * sizeof(double)));
    CK(hipMalloc(&m, 64));
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(marker, dim3(1), dim3(64), 0, st, 1, m);
        for (int k = 0; k < 10; k++) CK(ncclAllReduce(a, a, 4, ncclDouble, ncclSum, comm, st));
        hipLaunchKernelGGL(marker, dim3(1), dim3(64), 0, st, 2, m);
        for (int k = 0; k < 10; k++) {
            CK(ncclGroupStart());
            CK(ncclSend(a, n, ncclDouble, 0, comm, st));
            CK(ncclRecv(b, n, ncclDouble, 0, comm, st));
            CK(ncclGroupEnd());
        }
        hipLaunchKernelGGL(marker, dim3(1), dim3(64), 0, st, 3, m);
        for (int k = 0; k < 10; k++) {
            CK(ncclGroupStart());
            for (int q = 0; q < 7; q++) {
                CK(ncclSend(a + q * n, n, ncclDouble, 0, comm, st));
                CK(ncclRecv(b + q * n, n, ncclDouble, 0, comm, st));
            }
            CK(ncclGroupEnd());
        }
        hipLaunchKernelGGL(marker, dim3(1), dim3(64), 0, st, 4, m);
    }
    CK(hipStreamSynchronize(st));
    printf("rccl loopback probe done (%zu doubles per message)\n", n);
    ncclCommDestroy(comm);
    return 0;
}
