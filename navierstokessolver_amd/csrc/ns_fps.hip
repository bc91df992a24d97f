// ns_fps.hip -- the direct Poisson solve of rectangles with uniform spacing along y (r4).
//
// L phi = b - mean (FluidSolver.cpp:550-551) on a rectangle whose four sides are walls or inlets
// (zero-flux phi faces: ConstructLHS's 0 toward the boundary, FluidSolver.cpp:113-131) separates:
// L = Lx (x) I + I (x) Ly.  With hy uniform, Ly's eigenvectors are the DCT-II basis
// cos(pi k (2j+1) / 2N), eigenvalues mu_k = -(2 / hy^2)(1 - cos(pi k / N)); Lx (any hx) stays a
// tridiagonal matrix.  So the solve is
//   (1) a DCT-II of every row of b - shift            (k_fps_dct: one workgroup per row pair)
//   (2) for every mode k, the tridiagonal system (Lx + mu_k) x_k = f_k along x, by Thomas'
//       recurrences split into chunks of FPS_M rows: a chunk runs them from zero and a scan over
//       chunks (groups of FPS_G chunks, then groups) carries the true values in -- the forward
//       elimination (k_fps_t1 aggregates, k_fps_s1 scan, k_fps_t2 exact values) and the back
//       substitution (k_fps_t2 local, k_fps_s2 scan, k_fps_t3 fix-up)
//   (3) the inverse transform (DCT-III) of every row   (k_fps_idct)
// Mode 0 with walls on both x sides is singular (Lx 1 = 0): its last unknown is pinned to 0, a
// particular solution of the consistent system (phi is defined up to a constant, as the
// reference's MatNullSpace says).  Every step is a fixed sequence of arithmetic: deterministic,
// no iteration; its residual is ~1e-14 of ||b|| (checked by the solver, ns_solver.cpp).
//
// The transforms: Makhoul's DCT through an N-point complex FFT of the reordered row (v_n = x_2n,
// v_{N-1-n} = x_{2n+1}; X_k = Re(e^{-i pi k / 2N} V_k)), two real rows packed as the real and
// imaginary parts of one complex sequence.  The FFT is a Stockham radix-16 transform in LDS
// (N <= 8192 complex = 128 KiB), one workgroup of N/16 threads, one butterfly per thread and stage.
#include <hip/hip_runtime.h>

#include "ns_internal.h"

namespace nsg {

namespace {

struct cplx {
    double x, y;
};
__device__ inline cplx cadd(cplx a, cplx b) { return {a.x + b.x, a.y + b.y}; }
__device__ inline cplx csub(cplx a, cplx b) { return {a.x - b.x, a.y - b.y}; }
__device__ inline cplx cmul(cplx a, cplx b) { return {fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x)}; }

// cos / sin (2 pi k / 16), k < 8
__device__ constexpr double C16[8] = {1.0, 0.92387953251128675613, 0.70710678118654752440, 0.38268343236508977173,
                                      0.0, -0.38268343236508977173, -0.70710678118654752440, -0.92387953251128675613};
__device__ constexpr double S16[8] = {0.0, 0.38268343236508977173, 0.70710678118654752440, 0.92387953251128675613,
                                      1.0, 0.92387953251128675613, 0.70710678118654752440, 0.38268343236508977173};

// in-register DFT of R points, X_k = sum_n v_n e^{-2 pi i n k / R} (radix-2 decimation in time)
template <int R>
__device__ inline void dft(cplx* v) {
    if constexpr (R == 2) {
        const cplx a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    } else if constexpr (R > 2) {
        cplx e[R / 2], o[R / 2];
#pragma unroll
        for (int n = 0; n < R / 2; n++) {
            e[n] = v[2 * n];
            o[n] = v[2 * n + 1];
        }
        dft<R / 2>(e);
        dft<R / 2>(o);
#pragma unroll
        for (int k = 0; k < R / 2; k++) {
            const int q = k * (16 / R);   // w_R^k = w_16^q, q < 8
            cplx t;
            if (q == 0) t = o[k];
            else if (q == 4) t = {o[k].y, -o[k].x};   // * -i
            else t = cmul(o[k], cplx{C16[q], -S16[q]});
            v[k] = cadd(e[k], t);
            v[k + R / 2] = csub(e[k], t);
        }
    }
}

template <int LOGN>
struct Fft {
    static constexpr int N = 1 << LOGN;
    static constexpr int T = N / 16 < 64 ? 64 : (N / 16 > 512 ? 512 : N / 16);   // threads
};

// one Stockham stage of radix R over z[N] in LDS (sub-transform length Ns so far); every thread
// reads its butterflies' inputs, the block synchronises, then writes (in place)
template <int LOGN, int R>
__device__ inline void fft_stage(cplx* z, const cplx* __restrict__ tw, int tid, int Ns) {
    constexpr int N = Fft<LOGN>::N, T = Fft<LOGN>::T;
    constexpr int NB = N / R;
    constexpr int BPT = (NB + T - 1) / T;
    cplx v[BPT][R];
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        const int jb = tid + b * T;
        if (jb < NB) {
#pragma unroll
            for (int r = 0; r < R; r++) v[b][r] = z[jb + r * NB];
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        const int jb = tid + b * T;
        if (jb < NB) {
            const int k = jb & (Ns - 1);
            if (Ns > 1) {
                const int step = k * (N / (Ns * R));
#pragma unroll
                for (int r = 1; r < R; r++) v[b][r] = cmul(v[b][r], tw[(r * step) & (N - 1)]);
            }
            dft<R>(v[b]);
            const int d = (jb - k) * R + k;
#pragma unroll
            for (int r = 0; r < R; r++) z[d + r * Ns] = v[b][r];
        }
    }
    __syncthreads();
}

template <int LOGN>
__device__ inline void fft_lds(cplx* z, const cplx* __restrict__ tw, int tid) {
    int Ns = 1;
#pragma unroll
    for (int s = 0; s < LOGN / 4; s++) {
        fft_stage<LOGN, 16>(z, tw, tid, Ns);
        Ns *= 16;
    }
    if constexpr (LOGN % 4 != 0) fft_stage<LOGN, (1 << (LOGN % 4))>(z, tw, tid, Ns);
}

// (1) rows r0 = 2 blockIdx.x and r0 + 1 (the latter absent when nrows is odd) of in - shift ->
// their DCT-II coefficients in out.  tw[m] = e^{-2 pi i m / N}, wk[k] = e^{-i pi k / 2N}
template <int LOGN>
__global__ void __launch_bounds__(Fft<LOGN>::T) k_fps_dct(const double* __restrict__ in, const double* shiftp,
                                                           double* __restrict__ out, int nrows, int ld,
                                                           const cplx* __restrict__ tw, const cplx* __restrict__ wk) {
    constexpr int N = Fft<LOGN>::N, T = Fft<LOGN>::T;
    extern __shared__ cplx z[];
    const int tid = threadIdx.x;
    const int r0 = 2 * blockIdx.x;
    const bool two = r0 + 1 < nrows;
    const double sh = shiftp ? *shiftp : 0.0;
    const double* a = in + (size_t)r0 * ld;
    const double* b = a + ld;
    for (int j = tid; j < N; j += T) {
        const int n = (j & 1) ? N - 1 - (j >> 1) : (j >> 1);
        z[n] = cplx{a[j] - sh, two ? b[j] - sh : 0.0};
    }
    __syncthreads();
    fft_lds<LOGN>(z, tw, tid);
    double* oa = out + (size_t)r0 * ld;
    double* ob = oa + ld;
    for (int k = tid; k < N; k += T) {
        const cplx Zk = z[k], Zn = z[(N - k) & (N - 1)];
        const cplx Va{0.5 * (Zk.x + Zn.x), 0.5 * (Zk.y - Zn.y)};
        const cplx Vb{0.5 * (Zk.y + Zn.y), 0.5 * (Zn.x - Zk.x)};
        const cplx w = wk[k];
        oa[k] = fma(w.x, Va.x, -w.y * Va.y);
        if (two) ob[k] = fma(w.x, Vb.x, -w.y * Vb.y);
    }
}

// (3) the inverse: DCT-III with x_j = X_0 / N + (2 / N) sum_k>0 X_k cos(pi k (2j+1) / 2N), through
// V_k = e^{i pi k / 2N} (X_k - i X_{N-k}) (X_N = 0), v = IFFT(V) = conj(FFT(conj(V))) / N
template <int LOGN>
__global__ void __launch_bounds__(Fft<LOGN>::T) k_fps_idct(const double* __restrict__ in, double* __restrict__ out,
                                                            int nrows, int ld, const cplx* __restrict__ tw,
                                                            const cplx* __restrict__ wk) {
    constexpr int N = Fft<LOGN>::N, T = Fft<LOGN>::T;
    constexpr int PT = (N + T - 1) / T;
    extern __shared__ cplx z[];
    const int tid = threadIdx.x;
    const int r0 = 2 * blockIdx.x;
    const bool two = r0 + 1 < nrows;
    const double* a = in + (size_t)r0 * ld;
    const double* b = a + ld;
    for (int k = tid; k < N; k += T) z[k] = cplx{a[k], two ? b[k] : 0.0};
    __syncthreads();
    cplx v[PT];
#pragma unroll
    for (int p = 0; p < PT; p++) {
        const int k = tid + p * T;
        if (k < N) {
            const cplx Xk = z[k];
            const cplx Xn = k ? z[N - k] : cplx{0.0, 0.0};
            const cplx w = wk[k];   // e^{-i theta}: e^{i theta} = (w.x, -w.y)
            const double c = w.x, s = -w.y;
            // Va = e^{i theta} (A_k - i A_{N-k}), Vb likewise; V = Va + i Vb; store conj(V)
            const cplx Va{fma(c, Xk.x, s * Xn.x), fma(s, Xk.x, -c * Xn.x)};
            const cplx Vb{fma(c, Xk.y, s * Xn.y), fma(s, Xk.y, -c * Xn.y)};
            v[p] = cplx{Va.x - Vb.y, -(Va.y + Vb.x)};
        }
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < PT; p++) {
        const int k = tid + p * T;
        if (k < N) z[k] = v[p];
    }
    __syncthreads();
    fft_lds<LOGN>(z, tw, tid);
    const double rn = 1.0 / N;
    double* oa = out + (size_t)r0 * ld;
    double* ob = oa + ld;
    for (int j = tid; j < N; j += T) {
        const int n = (j & 1) ? N - 1 - (j >> 1) : (j >> 1);
        const cplx y = z[n];
        oa[j] = y.x * rn;
        if (two) ob[j] = -y.y * rn;
    }
}

// ---- (2) the tridiagonal systems along x, one per mode (column k of the transformed plane) ----
// Thomas on rows i (global gi): d_i = -(pw_i + pe_i) + mu_k, g_i = pw_i / p_{i-1},
// p_i = d_i - g_i pe_{i-1}, y_i = f_i - g_i y_{i-1}; back: x_i = y_i / p_i - (pe_i / p_i) x_{i+1}.
// Workgroup = FPS_G chunks (one wave each) x 64 modes.  rp0[c][k] = 1 / p of the row before chunk c.

// one row of the pivot recurrence: g = pw_i / p_{i-1} (from rprev = 1 / p_{i-1}); returns 1 / p_i
// (mode 0's pinned last global row: 0)
__device__ inline double piv_next(const FpsArgs& a, int gi, int k, double mu, double rprev, double& g) {
    const double pw = a.pw[gi], pe = a.pe[gi], pem = gi > 0 ? a.pe[gi - 1] : 0.0;
    g = pw * rprev;
    const double p = -(pw + pe) + mu - g * pem;
    return (a.pin && k == 0 && gi == a.nx - 1) ? 0.0 : 1.0 / p;
}

// T1: per chunk the forward recurrence from zero -> (E, Pi); the workgroup folds its chunks into
// the group's aggregate (y_out = E + Pi y_in)
__global__ void __launch_bounds__(64 * FPS_G) k_fps_t1(FpsArgs a, const double* __restrict__ f) {
    __shared__ double sE[FPS_G][64], sP[FPS_G][64];
    const int lane = threadIdx.x, w = threadIdx.y;
    const int k = blockIdx.x * 64 + lane;
    const int grp = blockIdx.y, c = grp * FPS_G + w;
    const int li0 = c * FPS_M;
    const int rows = k < a.ny ? min(FPS_M, a.nxl - li0) : 0;
    double E = 0.0, Pi = 1.0;
    if (rows > 0) {
        const double mu = a.mu[k];
        double r = a.rp0[(size_t)c * a.ld + k];
#pragma unroll
        for (int t = 0; t < FPS_M; t++) {
            if (t < rows) {
                double g;
                r = piv_next(a, a.i0 + li0 + t, k, mu, r, g);
                E = fma(-g, E, f[(size_t)(li0 + t) * a.ld + k]);
                Pi = -g * Pi;
            }
        }
    }
    sE[w][lane] = E;
    sP[w][lane] = Pi;
    __syncthreads();
    if (w == 0 && k < a.ny) {
        double GE = 0.0, GP = 1.0;
        for (int q = 0; q < FPS_G; q++) {
            GE = fma(sP[q][lane], GE, sE[q][lane]);
            GP = sP[q][lane] * GP;
        }
        a.ga[(size_t)grp * a.ld + k] = GE;
        a.ga[(size_t)(a.ngrp + grp) * a.ld + k] = GP;
    }
}

// S1 / S2: scan of the group aggregates per mode -> each group's carry-in (forward: ascending,
// backward: descending), from the carry-in of the ranks before / after (rin, null: 0); rout (if
// not null): this rank's aggregate (the fold of all its groups)
__global__ void k_fps_scan(int ngrp, int ld, int ny, const double* __restrict__ agg, double* __restrict__ carry,
                           const double* __restrict__ rin, double* __restrict__ rout, int backward) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= ny) return;
    double Y = rin ? rin[k] : 0.0, AE = 0.0, AP = 1.0;
    for (int q = 0; q < ngrp; q++) {
        const int grp = backward ? ngrp - 1 - q : q;
        const double E = agg[(size_t)grp * ld + k], P = agg[(size_t)(ngrp + grp) * ld + k];
        carry[(size_t)grp * ld + k] = Y;
        Y = fma(P, Y, E);
        AE = fma(P, AE, E);
        AP = P * AP;
    }
    if (rout) {
        rout[k] = AE;
        rout[ld + k] = AP;
    }
}

// T2: the chunk's exact forward values (its carry-in: the group's, through the group's earlier
// chunks), then the back substitution from zero -> xl (in place over f) and the chunk's backward
// aggregate (x_s = BX + BR x_e) into cb; the workgroup folds its chunks into gb
__global__ void __launch_bounds__(64 * FPS_G) k_fps_t2(FpsArgs a, double* __restrict__ f) {
    __shared__ double sE[FPS_G][64], sP[FPS_G][64];
    const int lane = threadIdx.x, w = threadIdx.y;
    const int k = blockIdx.x * 64 + lane;
    const int grp = blockIdx.y, c = grp * FPS_G + w;
    const int li0 = c * FPS_M;
    const int rows = k < a.ny ? min(FPS_M, a.nxl - li0) : 0;
    double y[FPS_M], pi[FPS_M], rp[FPS_M];
    double E = 0.0, Pi = 1.0;
    if (rows > 0) {
        const double mu = a.mu[k];
        double r = a.rp0[(size_t)c * a.ld + k];
#pragma unroll
        for (int t = 0; t < FPS_M; t++) {
            if (t < rows) {
                double g;
                r = piv_next(a, a.i0 + li0 + t, k, mu, r, g);
                E = fma(-g, E, f[(size_t)(li0 + t) * a.ld + k]);
                Pi = -g * Pi;
                y[t] = E;
                pi[t] = Pi;
                rp[t] = r;
            }
        }
    }
    sE[w][lane] = E;
    sP[w][lane] = Pi;
    __syncthreads();
    double Y = k < a.ny ? a.gc[(size_t)grp * a.ld + k] : 0.0;
    for (int q = 0; q < w; q++) Y = fma(sP[q][lane], Y, sE[q][lane]);
    double BX = 0.0, BR = 1.0;
    if (rows > 0) {
        double xl = 0.0, rho = 1.0;
#pragma unroll
        for (int t = FPS_M - 1; t >= 0; t--) {
            if (t < rows) {
                const int gi = a.i0 + li0 + t;
                const double yt = fma(pi[t], Y, y[t]);
                const double q = -a.pe[gi] * rp[t];
                xl = fma(yt, rp[t], q * xl);
                rho = q * rho;
                f[(size_t)(li0 + t) * a.ld + k] = xl;
            }
        }
        BX = xl;
        BR = rho;
        a.cb[(size_t)c * a.ld + k] = BX;
        a.cb[(size_t)(a.nch + c) * a.ld + k] = BR;
    }
    __syncthreads();   // (sE / sP reused)
    sE[w][lane] = BX;
    sP[w][lane] = BR;
    __syncthreads();
    if (w == 0 && k < a.ny) {
        double GX = 0.0, GR = 1.0;
        for (int q = FPS_G - 1; q >= 0; q--) {
            GX = fma(sP[q][lane], GX, sE[q][lane]);
            GR = sP[q][lane] * GR;
        }
        a.gb[(size_t)grp * a.ld + k] = GX;
        a.gb[(size_t)(a.ngrp + grp) * a.ld + k] = GR;
    }
}

// T3: the chunk's carry-in from the next chunk (the group's carry through its later chunks), then
// x_i = xl_i + rho_i x_e (in place)
__global__ void __launch_bounds__(64 * FPS_G) k_fps_t3(FpsArgs a, double* __restrict__ f) {
    __shared__ double sX[FPS_G][64], sR[FPS_G][64];
    const int lane = threadIdx.x, w = threadIdx.y;
    const int k = blockIdx.x * 64 + lane;
    const int grp = blockIdx.y, c = grp * FPS_G + w;
    const int li0 = c * FPS_M;
    const int rows = k < a.ny ? min(FPS_M, a.nxl - li0) : 0;
    double BX = 0.0, BR = 1.0;
    if (rows > 0) {
        BX = a.cb[(size_t)c * a.ld + k];
        BR = a.cb[(size_t)(a.nch + c) * a.ld + k];
    }
    sX[w][lane] = BX;
    sR[w][lane] = BR;
    __syncthreads();
    if (rows <= 0) return;
    double X = a.gx[(size_t)grp * a.ld + k];
    for (int q = FPS_G - 1; q > w; q--) X = fma(sR[q][lane], X, sX[q][lane]);
    const double mu = a.mu[k];
    double rp[FPS_M];
    double r = a.rp0[(size_t)c * a.ld + k];
#pragma unroll
    for (int t = 0; t < FPS_M; t++) {
        if (t < rows) {
            double g;
            r = piv_next(a, a.i0 + li0 + t, k, mu, r, g);
            rp[t] = r;
        }
    }
    double rho = 1.0;
#pragma unroll
    for (int t = FPS_M - 1; t >= 0; t--) {
        if (t < rows) {
            const int gi = a.i0 + li0 + t;
            rho = -a.pe[gi] * rp[t] * rho;
            double* p = f + (size_t)(li0 + t) * a.ld + k;
            *p = fma(rho, X, *p);
        }
    }
}

template <int LOGN>
void dct_pair(bool inverse, const double* in, const double* shift, double* out, int nrows, int ld, const void* tw,
              const void* wk, hipStream_t st) {
    constexpr int T = Fft<LOGN>::T;
    const size_t lds = sizeof(cplx) * (size_t)Fft<LOGN>::N;
    const dim3 grid((nrows + 1) / 2);
    if (inverse) {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void*)k_fps_idct<LOGN>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            attr = true;
        }
        hipLaunchKernelGGL(k_fps_idct<LOGN>, grid, dim3(T), lds, st, in, out, nrows, ld, (const cplx*)tw,
                           (const cplx*)wk);
    } else {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void*)k_fps_dct<LOGN>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            attr = true;
        }
        hipLaunchKernelGGL(k_fps_dct<LOGN>, grid, dim3(T), lds, st, in, shift, out, nrows, ld, (const cplx*)tw,
                           (const cplx*)wk);
    }
}

}  // namespace

int fps_log2(int ny) {
    int l = 0;
    while ((1 << l) < ny) l++;
    return (1 << l) == ny && l >= FPS_LOGN_MIN && l <= FPS_LOGN_MAX ? l : -1;
}

int launch_fps_dct(bool inverse, const double* in, const double* shift, double* out, int nrows, int ny, int ld,
                   const double* tw, const double* wk, hipStream_t st) {
    switch (fps_log2(ny)) {
    case 4: dct_pair<4>(inverse, in, shift, out, nrows, ld, tw, wk, st); break;
    case 5: dct_pair<5>(inverse, in, shift, out, nrows, ld, tw, wk, st); break;
    case 6: dct_pair<6>(inverse, in, shift, out, nrows, ld, tw, wk, st); break;
    case 7: dct_pair<7>(inverse, in, shift, out, nrows, ld, tw, wk, st); break;
    case 8: dct_pair<8>(inverse, in, shift, out, nrows, ld, tw, wk, st); break;
    case 9: dct_pair<9>(inverse, in, shift, out, nrows, ld, tw, wk, st); break;
    case 10: dct_pair<10>(inverse, in, shift, out, nrows, ld, tw, wk, st); break;
    case 11: dct_pair<11>(inverse, in, shift, out, nrows, ld, tw, wk, st); break;
    case 12: dct_pair<12>(inverse, in, shift, out, nrows, ld, tw, wk, st); break;
    case 13: dct_pair<13>(inverse, in, shift, out, nrows, ld, tw, wk, st); break;
    default: return -1;
    }
    return 0;
}

void launch_fps_t1(const FpsArgs& a, const double* f, hipStream_t st) {
    hipLaunchKernelGGL(k_fps_t1, dim3((a.ny + 63) / 64, a.ngrp), dim3(64, FPS_G), 0, st, a, f);
}
void launch_fps_t2(const FpsArgs& a, double* f, hipStream_t st) {
    hipLaunchKernelGGL(k_fps_t2, dim3((a.ny + 63) / 64, a.ngrp), dim3(64, FPS_G), 0, st, a, f);
}
void launch_fps_t3(const FpsArgs& a, double* f, hipStream_t st) {
    hipLaunchKernelGGL(k_fps_t3, dim3((a.ny + 63) / 64, a.ngrp), dim3(64, FPS_G), 0, st, a, f);
}
void launch_fps_scan(const FpsArgs& a, bool backward, const double* rin, double* rout, hipStream_t st) {
    hipLaunchKernelGGL(k_fps_scan, dim3((a.ny + 255) / 256), dim3(256), 0, st, a.ngrp, a.ld, a.ny,
                       backward ? a.gb : a.ga, backward ? a.gx : a.gc, rin, rout, backward ? 1 : 0);
}

}  // namespace nsg
