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
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>

#include "ns_internal.h"

namespace nsg {

namespace {

struct cplx {
    double x, y;
};
__device__ inline cplx cadd(cplx a, cplx b) { return {a.x + b.x, a.y + b.y}; }
__device__ inline cplx csub(cplx a, cplx b) { return {a.x - b.x, a.y - b.y}; }
__device__ inline cplx cmul(cplx a, cplx b) { return {fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x)}; }

__device__ inline double2 ld2(const double* p) { return *reinterpret_cast<const double2*>(p); }
__device__ inline void st2(double* p, double x, double y) { *reinterpret_cast<double2*>(p) = double2{x, y}; }

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

// radix 2^FPS_LR stages (A/B: 3 = radix 8, N/8 threads per row pair, more waves per CU)
#ifndef FPS_LR
#define FPS_LR 4
#endif
#ifndef FPS_PREF
#define FPS_PREF 0   // 1: the persistent transforms load the next row pair during this one (A/B, r4: 365 vs 343 us per solve -- its registers cost more than the overlap gains)
#endif
// (radix 8: two workgroups of N/8 threads per CU need <= 128 VGPRs)
// (radix 16: the register-fed stages (FPS_REGIO, N = 1024 ... 8192) need 134-210 VGPRs with the LDS indices
// formed per row pair (fps_remat); hoisted, they took 256 VGPRs + up to 123 AGPRs -- one workgroup per CU)
#if FPS_LR == 3
#define FPS_WAVES __attribute__((amdgpu_waves_per_eu(4)))
#else
#define FPS_WAVES
#endif
template <int LOGN>
struct Fft {
    static constexpr int N = 1 << LOGN;
    static constexpr int R = 1 << FPS_LR;
    static constexpr int T = (N >> FPS_LR) < 64 ? 64 : ((N >> FPS_LR) > 1024 ? 1024 : (N >> FPS_LR));   // threads
};

// LDS slot of element i (16 B each).  FPS_SWZ = 1 (default): the low three bits of i XOR-ed with bits
// 4-6 -- the first stage's writes of stride 16 elements land on 8 distinct slots of a 128-B bank row
// (ds_write_b128 banks), and contiguous ds_read_b128 runs stay conflict-free for its lane groups
// {0-3,12-15,20-27}, {4-11,16-19,28-31} (MI355X_MICROARCH.md LDS).  The padded layout (FPS_SWZ = 0:
// one slot every 16 and 256 elements) made every contiguous read 2-way (rocprofv3: SQ_LDS_BANK_CONFLICT
// = half of SQ_LDS_IDX_ACTIVE in k_fps_dct_div and k_fps_idct).  Only the transform's mirror read
// (X_{N-k}) stays 2-way.
#ifndef FPS_SWZ
#define FPS_SWZ 1
#endif
__device__ inline int pz(int i) {
#if FPS_SWZ
    return i ^ ((i >> 4) & 7);
#else
    return i + (i >> 4) + (i >> 8);
#endif
}
template <int LOGN>
struct FftLds {
    static constexpr int n = FPS_SWZ ? (1 << LOGN)
                                     : (1 << LOGN) - 1 + (((1 << LOGN) - 1) >> 4) + (((1 << LOGN) - 1) >> 8) + 1;
};

// one Stockham stage of radix R over z[N] in LDS (sub-transform length Ns so far); every thread
// reads its butterflies' inputs, the block synchronises, then writes (in place).  Twiddles
// w^r = e^{-2 pi i r k / (Ns R)}: w from the table, its powers by repeated products (r <= 15 roundings)
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
            for (int r = 0; r < R; r++) v[b][r] = z[pz(jb + r * NB)];
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        const int jb = tid + b * T;
        if (jb < NB) {
            const int k = jb & (Ns - 1);
            if (Ns > 1) {
                const cplx w = tw[k * (N / (Ns * R))];
                cplx wr = w;
#pragma unroll
                for (int r = 1; r < R; r++) {
                    v[b][r] = cmul(v[b][r], wr);
                    if (r + 1 < R) wr = cmul(wr, w);
                }
            }
            dft<R>(v[b]);
            const int d = (jb - k) * R + k;
#pragma unroll
            for (int r = 0; r < R; r++) z[pz(d + r * Ns)] = v[b][r];
        }
    }
    __syncthreads();
}

template <int LOGN>
__device__ inline void fft_lds(cplx* z, const cplx* __restrict__ tw, int tid) {
    int Ns = 1;
#pragma unroll
    for (int s = 0; s < LOGN / FPS_LR; s++) {
        fft_stage<LOGN, (1 << FPS_LR)>(z, tw, tid, Ns);
        Ns *= 1 << FPS_LR;
    }
    if constexpr (LOGN % FPS_LR != 0) fft_stage<LOGN, (1 << (LOGN % FPS_LR))>(z, tw, tid, Ns);
}

// The same transform with its first stage fed from registers and its last stage left in registers
// (N = 1024 ... 8192, N/16 threads): thread t holds the points t + (N/16) r, r < 16, on entry --
// exactly the first Stockham stage's inputs -- and Z[t + (N/16) r] on exit, the last stage's outputs
// (a radix-2/4/8 last stage: 16/R butterflies per thread).  At N = 4096 two LDS write passes and two
// read passes instead of four and four.
#ifndef FPS_REGIO
#define FPS_REGIO 1
#endif
#ifndef FPS_ISTAGE
#define FPS_ISTAGE 1   // the register-fed inverse transform's output staged through LDS (A/B: 0)
#endif
#ifndef FPS_NT
#define FPS_NT 0   // A/B: non-temporal stores of the inverse transform's phi
#endif
template <int LOGN>
__device__ inline void fft_regs(cplx* z, const cplx* __restrict__ tw, int tid, cplx* v) {
    constexpr int N = 1 << LOGN, T = N / 16, S16 = LOGN / 4, RL = 1 << (LOGN % 4);
    static_assert(Fft<LOGN>::T == T && S16 >= 2, "fft_regs: N / 16 threads, at least two radix-16 stages");
    dft<16>(v);   // stage 1 (Ns = 1: no twiddles), outputs to 16 tid + r
#pragma unroll
    for (int r = 0; r < 16; r++) z[pz(16 * tid + r)] = v[r];
    __syncthreads();
    int Ns = 16;
    constexpr int MID = RL == 1 ? S16 - 2 : S16 - 1;   // LDS-to-LDS radix-16 stages
#pragma unroll
    for (int st = 0; st < MID; st++) {
        fft_stage<LOGN, 16>(z, tw, tid, Ns);
        Ns *= 16;
    }
    // last stage: radix R (16, or the remainder 2 / 4 / 8), Ns = N / R; butterfly jb = tid + b T has
    // k = jb and outputs Z[jb + Ns r] = Z[tid + T (b + (16 / R) r)]: slot b + (16 / R) r of v
    constexpr int R = RL == 1 ? 16 : RL, BPT = 16 / R, NB = N / R;
#pragma unroll
    for (int bb = 0; bb < BPT; bb++) {
        const int jb = tid + bb * T;
        cplx u[R];
#pragma unroll
        for (int r = 0; r < R; r++) u[r] = z[pz(jb + r * NB)];
        const cplx w = tw[jb];   // e^{-2 pi i jb / N}: k (N / (Ns R)) with Ns R = N
        cplx wr = w;
#pragma unroll
        for (int r = 1; r < R; r++) {
            u[r] = cmul(u[r], wr);
            if (r + 1 < R) wr = cmul(wr, w);
        }
        dft<R>(u);
#pragma unroll
        for (int r = 0; r < R; r++) v[bb + BPT * r] = u[r];
    }
}

// the persistent transforms: tid made opaque at every row pair, so that the LDS slot and twiddle indices
// of every stage are formed per pair instead of hoisted out of the loop into ~100 live registers (they
// pushed the kernels past 256 VGPRs, one workgroup per CU).  FPS_REMAT=0: hoisted (A/B)
// pass orders alternating up / down the slab between the direct solve's passes (A/B: 0)
#ifndef FPS_SNAKE
#define FPS_SNAKE 1
#endif
#ifndef FPS_REMAT
#define FPS_REMAT 1
#endif
__device__ inline void fps_remat(int& t) {
#if FPS_REMAT
    asm volatile("" : "+v"(t));
#endif
}

// (1) DCT-II of row pairs (r0 = 2 p, r0 + 1; the latter absent when nrows is odd) of in - shift
// -> their coefficients in out.  tw[m] = e^{-2 pi i m / N}, wk[k] = e^{-i pi k / 2N}.  Persistent:
// a workgroup walks pairs p = blockIdx.x, + gridDim.x, ...; the next pair's rows are loaded into
// registers while this pair's coefficients are formed and stored (the LDS allows two workgroups
// per CU, so without that overlap the CU idles through every load)
// (r5) oe_pair: the row pair whose second row is the NEUMANN outflow row -- it transforms b_{n-1} - b_{n-2} / 2
// (the elimination of piv_next); -1: none
template <int LOGN>
__global__ void __launch_bounds__(Fft<LOGN>::T) FPS_WAVES k_fps_dct(const double* __restrict__ in, const double* shiftp,
                                                           double* __restrict__ out, int nrows, int ld,
                                                           const cplx* __restrict__ tw, const cplx* __restrict__ wk,
                                                           int oe_pair) {
    constexpr int N = Fft<LOGN>::N, T = Fft<LOGN>::T;
    constexpr int PT = (N + T - 1) / T;
    extern __shared__ cplx z[];
    int tid = threadIdx.x;
    const int npairs = (nrows + 1) / 2;
    const double sh = shiftp ? *shiftp : 0.0;
    double ra[PT], rb[PT];
    auto load = [&](int p) {
        const int r0 = 2 * p;
        const bool two = r0 + 1 < nrows;
        const double* a = in + (size_t)r0 * ld;
#pragma unroll
        for (int q = 0; q < PT; q++) {
            const int j = tid + q * T;
            if (j < N) {
                ra[q] = a[j];
                rb[q] = two ? a[ld + j] : sh;
            }
        }
    };
    // (N = 8192: the prefetch registers would spill -- load each pair when it starts)
    constexpr bool PREF = FPS_PREF && LOGN <= 12;
    int p = blockIdx.x;
    constexpr bool REGIO = FPS_REGIO && FPS_LR == 4 && LOGN >= 10 && LOGN <= 13;
    if constexpr (REGIO) {
        // thread t holds v_n, n = t + 256 r: v_n = x_2n (n < N/2), x_{2(N-1-n)+1} (n >= N/2)
        for (; p < npairs; p += gridDim.x) {
            fps_remat(tid);
            const int r0 = 2 * p;
            const bool two = r0 + 1 < nrows;
            const double* a = in + (size_t)r0 * ld;
            cplx v[16];
            const double lam = p == oe_pair ? 0.5 : 0.0;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int n = tid + r * T;
                const int j = n < N / 2 ? 2 * n : 2 * (N - 1 - n) + 1;
                const double xa = a[j] - sh;
                v[r] = cplx{xa, two ? a[ld + j] - sh - lam * xa : 0.0};
            }
            fft_regs<LOGN>(z, tw, tid, v);
            __syncthreads();   // (every thread has read its last stage's inputs)
#pragma unroll
            for (int r = 0; r < 16; r++) z[pz(tid + r * T)] = v[r];
            __syncthreads();
            double* oa = out + (size_t)r0 * ld;
            double* ob = oa + ld;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int k = tid + r * T;
                const cplx Zk = v[r], Zn = z[pz((N - k) & (N - 1))];
                const cplx Va{0.5 * (Zk.x + Zn.x), 0.5 * (Zk.y - Zn.y)};
                const cplx Vb{0.5 * (Zk.y + Zn.y), 0.5 * (Zn.x - Zk.x)};
                const cplx w = wk[k];
                oa[k] = fma(w.x, Va.x, -w.y * Va.y);
                if (two) ob[k] = fma(w.x, Vb.x, -w.y * Vb.y);
            }
            __syncthreads();   // (z is rewritten by the next pair)
        }
        return;
    }
    if (PREF && p < npairs) load(p);
    for (; p < npairs; p += gridDim.x) {
        fps_remat(tid);
        const int r0 = 2 * p;
        const bool two = r0 + 1 < nrows;
        if (!PREF) load(p);
        const double lam = p == oe_pair ? 0.5 : 0.0;
#pragma unroll
        for (int q = 0; q < PT; q++) {
            const int j = tid + q * T;
            if (j < N) {
                const int n = (j & 1) ? N - 1 - (j >> 1) : (j >> 1);
                z[pz(n)] = cplx{ra[q] - sh, rb[q] - sh - lam * (ra[q] - sh)};
            }
        }
        __syncthreads();
        fft_lds<LOGN>(z, tw, tid);
        if (PREF && p + (int)gridDim.x < npairs) load(p + gridDim.x);
        double* oa = out + (size_t)r0 * ld;
        double* ob = oa + ld;
#pragma unroll
        for (int q = 0; q < PT; q++) {
            const int k = tid + q * T;
            if (k < N) {
                const cplx Zk = z[pz(k)], Zn = z[pz((N - k) & (N - 1))];
                const cplx Va{0.5 * (Zk.x + Zn.x), 0.5 * (Zk.y - Zn.y)};
                const cplx Vb{0.5 * (Zk.y + Zn.y), 0.5 * (Zn.x - Zk.x)};
                const cplx w = wk[k];
                oa[k] = fma(w.x, Va.x, -w.y * Va.y);
                if (two) ob[k] = fma(w.x, Vb.x, -w.y * Vb.y);
            }
        }
        __syncthreads();   // (z is rewritten by the next pair)
    }
}

// (1') K3 fused into the transform (r4): the row pair's b = Div_V(u*, v*) / dt (FluidSolver.cpp:380-418,
// k_cell_s<3>'s arithmetic) formed in the transform's LDS, its sums (sum, sum^2: the mean and
// ||b - mean|| of MatNullSpaceRemove, :550) as workgroup partials, b itself stored only when asked
// (the checked solves' residual).  The mean is not known yet: the coefficients are those of b, and the
// recurrences take N mean off mode 0 (FpsArgs::sh0) -- the DCT of a constant.  One HBM pass less per
// step (K3's b written and read back).  Pairs p = plo + q pstep, q < cnt (slabs: the interior pairs,
// then the two edge pairs after the u*, v* ghost-row exchange); consecutive pairs on one XCD (their
// shared u* rows in its L2).  The sums go out per row pair (deterministic under any split).
__device__ inline double fv_ghost(const Geo& g, double q, int side, int d) {
    return g.neu[side] ? q : (-q + (d == 0 ? g.c0[side] : g.c1[side]));
}
__device__ inline double dpp_up1(double x) {   // lane l <- lane l - 1
    const int lo = __double2loint(x), hi = __double2hiint(x);
    return __hiloint2double(__builtin_amdgcn_update_dpp(hi, hi, 0x138, 0xf, 0xf, false),
                            __builtin_amdgcn_update_dpp(lo, lo, 0x138, 0xf, 0xf, false));
}
__device__ inline double dpp_dn1(double x) {   // lane l <- lane l + 1
    const int lo = __double2loint(x), hi = __double2hiint(x);
    return __hiloint2double(__builtin_amdgcn_update_dpp(hi, hi, 0x130, 0xf, 0xf, false),
                            __builtin_amdgcn_update_dpp(lo, lo, 0x130, 0xf, 0xf, false));
}

#ifndef FPS_DB
#define FPS_DB 4   // column pairs whose loads k_fps_dct_div issues before their arithmetic (A/B: 8)
#endif
struct FpsDivArgs {
    Geo g;
    Coef c;
    double rdt;            // 1 / dt
    const double *u, *v;   // u*, v* (local row 0; one ghost row each side read)
    double* b;             // null, or rhs_phi is stored too
    double* out;           // coefficients
    double* part;          // (sum, sum^2) per row pair p at part + 2 p
    int nrows, ld, plo, cnt, pstep;
    const cplx *tw, *wk;
    int outE;              // (r5) NEUMANN outflow E side: the last row pair's second row transforms b_{n-1} - b_{n-2} / 2
};

template <int LOGN>
__global__ void __launch_bounds__(Fft<LOGN>::T) FPS_WAVES k_fps_dct_div(FpsDivArgs A) {
    constexpr int N = Fft<LOGN>::N, T = Fft<LOGN>::T, NC = N / 2;   // column pairs per row
    extern __shared__ cplx z[];
    __shared__ double red[T / 64][2];
    const Geo& g = A.g;
    int tid = threadIdx.x;
    const int lane = tid & 63;
    const int ld = A.ld;
    double acc[2] = {0.0, 0.0};
    constexpr bool REGIO = FPS_REGIO && FPS_LR == 4 && LOGN >= 10 && LOGN <= 13;
    const int G = gridDim.x;
    const int q0 = G % 8 == 0 ? (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8 : blockIdx.x;
    for (int q = q0; q < A.cnt; q += G) {
        fps_remat(tid);
        const int p = A.plo + q * A.pstep;
        const int r0 = 2 * p;
        const bool two = r0 + 1 < A.nrows;
        const int gi = g.i0 + r0;
        const bool hWa = gi > 0, hEa = gi < g.nx - 1, hWb = gi + 1 > 0, hEb = gi + 1 < g.nx - 1;
        const double* u0 = A.u + (ptrdiff_t)(r0 - 1) * ld;
        const double* va = A.v + (ptrdiff_t)r0 * ld;
        // (uniform spacing -- the direct solve's premise: one interior column's 1 / hy; 1 / h and 1 / dt
        // as products instead of K3's divisions)
        const double rhy = A.c.rhy[1], hrdt = 0.5 * A.rdt;
        const double rhxa = A.c.rhx[gi], rhxb = two ? A.c.rhx[gi + 1] : 0.0;
        // column pair cb (columns j = 2 cb, j + 1): u* rows r0 - 1 .. r0 + 2, v* rows r0, r0 + 1; v* at
        // columns j - 1 / j + 2 from the neighbouring lanes, loaded by the wave's edge lanes (E)
        auto load = [&](int cb, double2(&U)[4], double2(&Vv)[2], double(&E)[4]) {
            const int j = 2 * cb;
#pragma unroll
            for (int k = 0; k < 4; k++) U[k] = ld2(u0 + k * ld + j);
            Vv[0] = ld2(va + j);
            Vv[1] = ld2(va + ld + j);
            if (lane == 0) {
                const int js = max(j - 1, 0);
                E[0] = va[js];
                E[1] = va[ld + js];
            }
            if (lane == 63 || cb + 1 >= NC) {
                const int jn = min(j + 2, g.ny - 1);
                E[2] = va[jn];
                E[3] = va[ld + jn];
            }
        };
        auto cell = [&](int cb, const double2(&U)[4], const double2(&Vv)[2], const double(&E)[4]) {
            const int j = 2 * cb;
            double vsA = dpp_up1(Vv[0].y), vsB = dpp_up1(Vv[1].y), vnA = dpp_dn1(Vv[0].x), vnB = dpp_dn1(Vv[1].x);
            if (lane == 0) {
                vsA = E[0];
                vsB = E[1];
            }
            if (lane == 63 || cb + 1 >= NC) {
                vnA = E[2];
                vnB = E[3];
            }
            // (uniform spacing: every interior face weight is 1/2, so V1 - V0 = (X - Y) / 2 with X, Y the
            // east / west neighbours or, across a wall / inlet face, the ghost -- the same divergence as
            // k_cell_s<3>'s four face values, ~1 ulp apart, in a third of the arithmetic)
            double d[2][2];
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const int jj = j + e;
                const bool s = jj > 0, n = jj < g.ny - 1;
#pragma unroll
                for (int rr = 0; rr < 2; rr++) {
                    const double2 uc2 = U[rr + 1], uw2 = U[rr], ue2 = U[rr + 2], vv = Vv[rr];
                    const double uc = e ? uc2.y : uc2.x, uwv = e ? uw2.y : uw2.x, uev = e ? ue2.y : ue2.x;
                    const double vc = e ? vv.y : vv.x;
                    const double vs = e ? vv.x : (rr ? vsB : vsA), vn = e ? (rr ? vnB : vnA) : vv.y;
                    const bool hW = rr ? hWb : hWa, hE = rr ? hEb : hEa;
                    const double X = hE ? uev : fv_ghost(g, uc, 1, 0), Y = hW ? uwv : fv_ghost(g, uc, 0, 0);
                    const double Xn = n ? vn : fv_ghost(g, vc, 3, 1), Ys = s ? vs : fv_ghost(g, vc, 2, 1);
                    d[rr][e] = fma(X - Y, rr ? rhxb : rhxa, (Xn - Ys) * rhy) * hrdt;
                }
            }
            if (!two) d[1][0] = d[1][1] = 0.0;
            acc[0] += d[0][0] + d[0][1];
            acc[1] += d[0][0] * d[0][0] + d[0][1] * d[0][1];
            if (two) {
                acc[0] += d[1][0] + d[1][1];
                acc[1] += d[1][0] * d[1][0] + d[1][1] * d[1][1];
            }
            if (A.b) {
                st2(A.b + (ptrdiff_t)r0 * ld + j, d[0][0], d[0][1]);
                if (two) st2(A.b + (ptrdiff_t)(r0 + 1) * ld + j, d[1][0], d[1][1]);
            }
            if (A.outE && two && gi + 1 == g.nx - 1) {   // (the outflow row's elimination, piv_next)
                d[1][0] -= 0.5 * d[0][0];
                d[1][1] -= 0.5 * d[0][1];
            }
            // v_n = x_2n, v_{N-1-n} = x_{2n+1}
            z[pz(cb)] = cplx{d[0][0], d[1][0]};
            z[pz(N - 1 - cb)] = cplx{d[0][1], d[1][1]};
        };
        if constexpr (NC % T == 0) {
            // (N >= 128: every lane has NC / T column pairs; their loads issued in batches of 4 before the
            // arithmetic -- one HBM latency per batch instead of two per column pair)
            constexpr int NCT = NC / T, B = NCT < FPS_DB ? NCT : FPS_DB;
#pragma unroll
            for (int c0 = 0; c0 < NCT; c0 += B) {
                double2 U[B][4], Vv[B][2];
                double E[B][4];
#pragma unroll
                for (int q = 0; q < B; q++) load(tid + (c0 + q) * T, U[q], Vv[q], E[q]);
#pragma unroll
                for (int q = 0; q < B; q++) cell(tid + (c0 + q) * T, U[q], Vv[q], E[q]);
            }
        } else {
            for (int cb = tid; cb < NC; cb += T) {
                double2 U[4], Vv[2];
                double E[4];
                load(cb, U, Vv, E);
                cell(cb, U, Vv, E);
            }
        }
        // the pair's (sum, sum^2) -> part[2 p]: one fixed order per pair, whatever the launches' split
#pragma unroll
        for (int k = 0; k < 2; k++)
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) acc[k] += __shfl_xor(acc[k], off, 64);
        if (lane == 0) {
            red[tid >> 6][0] = acc[0];
            red[tid >> 6][1] = acc[1];
        }
        acc[0] = acc[1] = 0.0;
        __syncthreads();
        if (tid == 0) {
            double s0 = 0.0, s1 = 0.0;
            for (int w = 0; w < T / 64; w++) {
                s0 += red[w][0];
                s1 += red[w][1];
            }
            A.part[2 * p] = s0;
            A.part[2 * p + 1] = s1;
        }
        double* oa = A.out + (size_t)r0 * ld;
        double* ob = oa + ld;
        if constexpr (REGIO) {
            cplx v[16];
#pragma unroll
            for (int r = 0; r < 16; r++) v[r] = z[pz(tid + r * T)];
            __syncthreads();
            fft_regs<LOGN>(z, A.tw, tid, v);
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 16; r++) z[pz(tid + r * T)] = v[r];
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int k = tid + r * T;
                const cplx Zk = v[r], Zn = z[pz((N - k) & (N - 1))];
                const cplx Va{0.5 * (Zk.x + Zn.x), 0.5 * (Zk.y - Zn.y)};
                const cplx Vb{0.5 * (Zk.y + Zn.y), 0.5 * (Zn.x - Zk.x)};
                const cplx w = A.wk[k];
                oa[k] = fma(w.x, Va.x, -w.y * Va.y);
                if (two) ob[k] = fma(w.x, Vb.x, -w.y * Vb.y);
            }
        } else {
            constexpr int PT = (N + T - 1) / T;
            fft_lds<LOGN>(z, A.tw, tid);
#pragma unroll
            for (int qq = 0; qq < PT; qq++) {
                const int k = tid + qq * T;
                if (k < N) {
                    const cplx Zk = z[pz(k)], Zn = z[pz((N - k) & (N - 1))];
                    const cplx Va{0.5 * (Zk.x + Zn.x), 0.5 * (Zk.y - Zn.y)};
                    const cplx Vb{0.5 * (Zk.y + Zn.y), 0.5 * (Zn.x - Zk.x)};
                    const cplx w = A.wk[k];
                    oa[k] = fma(w.x, Va.x, -w.y * Va.y);
                    if (two) ob[k] = fma(w.x, Vb.x, -w.y * Vb.y);
                }
            }
        }
        __syncthreads();   // (z is rewritten by the next pair)
    }
}

// (1'') (r6) the same forward transform with K3 fused, ONE row per workgroup: the row's N reals
// in Makhoul's order v as the N/2-point complex sequence y_m = v_2m + i v_2m+1, Y = FFT_{N/2}(y) by radix-8
// Stockham stages (N/16 threads), then V_k = E_k + e^{-2 pi i k / N} O_k and V_{k+N/2} = E_k - e^{-2 pi i k / N} O_k
// with E_k = (Y_k + conj Y_{N/2-k}) / 2, O_k = (Y_k - conj Y_{N/2-k}) / 2i the even / odd samples' spectra, and
// X_k = Re(e^{-i pi k / 2N} V_k) as before.  Half the LDS of the row pair's transform (32 KiB at N = 4096) and
// half its registers per thread: 4 workgroups of 4 waves per CU instead of 2.  The divergence arithmetic is
// k_fps_dct_div's (b identical); the sums go out per row (slot 2 p + h: 2 np partials).  Not for a NEUMANN
// outflow E side (its last row is transformed against the row above: k_fps_dct_div keeps it)
template <int LOGN>
struct RFft {
    static constexpr int N = 1 << LOGN, M = N / 2, T = M / 8;
};
#ifndef FPS_RB
#define FPS_RB 4   // k_fps_dct_div_r: column pairs whose loads are issued before their arithmetic (A/B: 8)
#endif
#ifndef FPS_RE
#define FPS_RE 0   // k_fps_dct_div_r: the wave-edge neighbours loaded by the edge lanes only (A/B: 1)
#endif
#ifndef FPS_RTW
#define FPS_RTW 1   // the row transforms' stage twiddles loaded up front (RTw), the split's formed by products (A/B: 0)
// (N <= 8192; at 16384 -- 1024 threads, one workgroup per CU -- they measured slower: 2346 vs 2219 us forward)
#endif
// every radix-8 stage's twiddle of this thread's butterfly and the last (radix 2 / 4) stage's, loaded before the row:
// their latency behind its loads instead of one global round trip per stage between two barriers
template <int LOGN>
struct RTw {
    static constexpr int N = 1 << LOGN, M = N / 2, T = RFft<LOGN>::T, LOGM = LOGN - 1, NS8 = LOGM / 3,
                         RL = 1 << (LOGM % 3), BL = RL > 1 ? (M / RL) / T : 1;
    cplx w8[NS8], wl[BL];
    __device__ inline void load(const cplx* __restrict__ tw, int tid) {
        int Ns = 1;
#pragma unroll
        for (int st = 0; st < NS8; st++) {
            w8[st] = tw[(tid & (Ns - 1)) * (N / (Ns * 8))];
            Ns *= 8;
        }
        if constexpr (RL > 1) {
#pragma unroll
            for (int b = 0; b < BL; b++) wl[b] = tw[((tid + b * T) & (Ns - 1)) * (N / (Ns * RL))];
        }
    }
};
template <int LOGN, int R>
__device__ inline void rfft_stage(cplx* z, const cplx* __restrict__ tw, int tid, int Ns, const cplx* wp = nullptr) {
    constexpr int N = 1 << LOGN, M = N / 2, T = RFft<LOGN>::T, NB = M / R, BPT = NB / T;
    static_assert(NB % T == 0, "rfft stage layout");
    cplx v[BPT][R];
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        const int jb = tid + b * T;
#pragma unroll
        for (int r = 0; r < R; r++) v[b][r] = z[pz(jb + r * NB)];
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BPT; b++) {
        const int jb = tid + b * T;
        const int k = jb & (Ns - 1);
        if (Ns > 1) {
            const cplx w = wp ? wp[b] : tw[k * (N / (Ns * R))];   // e^{-2 pi i k / (Ns R)}: the N-point table
            cplx wr = w;
#pragma unroll
            for (int r = 1; r < R; r++) {
                v[b][r] = cmul(v[b][r], wr);
                if (r + 1 < R) wr = cmul(wr, w);
            }
        }
        dft<R>(v[b]);
        const int d = (jb - k) * R + k;
#pragma unroll
        for (int r = 0; r < R; r++) z[pz(d + r * Ns)] = v[b][r];
    }
    __syncthreads();
}

template <int LOGN>
__global__ void __launch_bounds__(RFft<LOGN>::T) k_fps_dct_div_r(FpsDivArgs A) {
    constexpr int N = 1 << LOGN, M = N / 2, T = RFft<LOGN>::T, LOGM = LOGN - 1;
    constexpr int NCT = M / T, B = NCT < FPS_RB ? NCT : FPS_RB;   // column pairs per thread (8), loads batched by 4
    extern __shared__ cplx z[];
    __shared__ double red[T / 64][2];
    const Geo& g = A.g;
    const int tid = threadIdx.x, lane = tid & 63;
    const int ld = A.ld;
    // workgroup -> (pair q, its row h); consecutive rows on one XCD (their shared u* rows in its L2)
    const int G = gridDim.x, bx = blockIdx.x;
    const int un = G % 8 == 0 ? (bx % 8) * (G / 8) + bx / 8 : bx;
    const int p = A.plo + (un >> 1) * A.pstep, r = 2 * p + (un & 1);
    if (r >= A.nrows) {   // (an odd slab's last pair has one row: zero sums for the other)
        if (tid == 0) A.part[2 * r] = A.part[2 * r + 1] = 0.0;
        return;
    }
    const int gi = g.i0 + r;
    const bool hW = gi > 0, hE = gi < g.nx - 1;
    const double* u0 = A.u + (ptrdiff_t)(r - 1) * ld;
    const double* va = A.v + (ptrdiff_t)r * ld;
    const double rhy = A.c.rhy[1], hrdt = 0.5 * A.rdt, rhx = A.c.rhx[gi];
    double* zd = reinterpret_cast<double*>(z);
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
    for (int c0 = 0; c0 < NCT; c0 += B) {
        double2 U[B][3], V[B];
        double E[B][2];
#pragma unroll
        for (int q = 0; q < B; q++) {
            const int j = 2 * (tid + (c0 + q) * T);
#pragma unroll
            for (int k = 0; k < 3; k++) U[q][k] = ld2(u0 + k * ld + j);
            V[q] = ld2(va + j);
            if (FPS_RE == 0 || lane == 0) E[q][0] = va[max(j - 1, 0)];                      // (lane 0's west neighbour)
            if (FPS_RE == 0 || lane == 63 || j + 2 >= N) E[q][1] = va[min(j + 2, g.ny - 1)];   // (lane 63's east one)
        }
#pragma unroll
        for (int q = 0; q < B; q++) {
            const int cb = tid + (c0 + q) * T, j = 2 * cb;
            double vs = dpp_up1(V[q].y), vn = dpp_dn1(V[q].x);
            if (lane == 0) vs = E[q][0];
            if (lane == 63 || cb + 1 >= M) vn = E[q][1];
            double d[2];
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const int jj = j + e;
                const bool sa = jj > 0, na = jj < g.ny - 1;
                const double uc = e ? U[q][1].y : U[q][1].x, uwv = e ? U[q][0].y : U[q][0].x,
                             uev = e ? U[q][2].y : U[q][2].x;
                const double vc = e ? V[q].y : V[q].x;
                const double vsv = e ? V[q].x : vs, vnv = e ? vn : V[q].y;
                const double X = hE ? uev : fv_ghost(g, uc, 1, 0), Y = hW ? uwv : fv_ghost(g, uc, 0, 0);
                const double Xn = na ? vnv : fv_ghost(g, vc, 3, 1), Ys = sa ? vsv : fv_ghost(g, vc, 2, 1);
                d[e] = fma(X - Y, rhx, (Xn - Ys) * rhy) * hrdt;
            }
            acc0 += d[0] + d[1];
            acc1 += d[0] * d[0] + d[1] * d[1];
            if (A.b) st2(A.b + (ptrdiff_t)r * ld + j, d[0], d[1]);
            // x_2cb = v_cb -> y_{cb/2} (re / im by cb's parity); x_{2cb+1} = v_{N-1-cb} -> y_{(N-1-cb)/2}
            const int n1 = N - 1 - cb;
            zd[2 * pz(cb >> 1) + (cb & 1)] = d[0];
            zd[2 * pz(n1 >> 1) + (n1 & 1)] = d[1];
        }
    }
    // (the transform's twiddles now, after the row's registers are free: all stages' in one round trip, behind the
    // partial sums' barrier)
    RTw<LOGN> W;
    cplx t0{1.0, 0.0}, w0s{1.0, 0.0};
    if constexpr (FPS_RTW && LOGN <= 13) {
        W.load(A.tw, tid);
        t0 = A.tw[tid];    // the split's e^{-2 pi i k / N}, e^{-i pi k / 2N} at k = tid; k = tid + q T by products
        w0s = A.wk[tid];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        acc0 += __shfl_xor(acc0, off, 64);
        acc1 += __shfl_xor(acc1, off, 64);
    }
    if (lane == 0) {
        red[tid >> 6][0] = acc0;
        red[tid >> 6][1] = acc1;
    }
    __syncthreads();
    if (tid == 0) {
        double s0 = 0.0, s1 = 0.0;
        for (int w = 0; w < T / 64; w++) {
            s0 += red[w][0];
            s1 += red[w][1];
        }
        A.part[2 * r] = s0;
        A.part[2 * r + 1] = s1;
    }
    int Ns = 1;
#pragma unroll
    for (int st = 0; st < LOGM / 3; st++) {
        rfft_stage<LOGN, 8>(z, A.tw, tid, Ns, (FPS_RTW && LOGN <= 13) ? &W.w8[st] : nullptr);
        Ns *= 8;
    }
    if constexpr (LOGM % 3 != 0) rfft_stage<LOGN, (1 << (LOGM % 3))>(z, A.tw, tid, Ns, (FPS_RTW && LOGN <= 13) ? W.wl : nullptr);
    double* oa = A.out + (size_t)r * ld;
#pragma unroll
    for (int q = 0; q < M / T; q++) {
        const int k = tid + q * T;
        const cplx Yk = z[pz(k)], Ym = z[pz((M - k) & (M - 1))];
        const cplx Ek{0.5 * (Yk.x + Ym.x), 0.5 * (Yk.y - Ym.y)};
        const cplx Ok{0.5 * (Yk.y + Ym.y), 0.5 * (Ym.x - Yk.x)};
        // (FPS_RTW: e^{-2 pi i k / N} = tw[tid] tw[q T], e^{-i pi k / 2N} = wk[tid] wk[q T], e^{-i pi (k + M) / 2N} =
        // that times wk[M] -- the uniform factors are scalar loads; one rounding more than the table)
        const cplx tk = (FPS_RTW && LOGN <= 13) ? (q ? cmul(t0, A.tw[q * T]) : t0) : A.tw[k];
        const cplx tO = cmul(tk, Ok);
        const cplx V0 = cadd(Ek, tO), V1 = csub(Ek, tO);
        const cplx w0 = (FPS_RTW && LOGN <= 13) ? (q ? cmul(w0s, A.wk[q * T]) : w0s) : A.wk[k];
        const cplx w1 = (FPS_RTW && LOGN <= 13) ? cmul(w0, A.wk[M]) : A.wk[k + M];
        oa[k] = fma(w0.x, V0.x, -w0.y * V0.y);
        oa[k + M] = fma(w1.x, V1.x, -w1.y * V1.y);
    }
}

// (3'') (r6) the inverse of ONE row per workgroup (k_fps_dct_div_r's layout backwards): V is Hermitian (v real), so
// with V_k = e^{i pi k / 2N} (X_k - i X_{N-k}), E_k = (V_k + V_{k+N/2}) / 2, O_k = (V_k - V_{k+N/2}) e^{2 pi i k / N} / 2
// (the even / odd samples' spectra), y = IFFT_{N/2}(E + i O) holds v_2m + i v_2m+1 -- one N/2-point transform
// (conj(FFT(conj .)) / (N/2)) instead of a row pair's N-point one; each lane stores columns 2 cb, 2 cb + 1
template <int LOGN>
__global__ void __launch_bounds__(RFft<LOGN>::T) k_fps_idct_r(const double* __restrict__ in, double* __restrict__ out,
                                                              int nrows, int ld, const cplx* __restrict__ tw,
                                                              const cplx* __restrict__ wk) {
    constexpr int N = 1 << LOGN, M = N / 2, T = RFft<LOGN>::T, LOGM = LOGN - 1;
    extern __shared__ cplx z[];
    const int tid = threadIdx.x;
    const int r = nrows - 1 - (int)blockIdx.x;   // (as k_fps_idct's pass order: up the slab)
    const double* a = in + (size_t)r * ld;
    RTw<LOGN> W;
    if constexpr (FPS_RTW && LOGN <= 13) W.load(tw, tid);
#pragma unroll
    for (int q = 0; q < M / T; q++) {
        const int k = tid + q * T;
        const double xa = a[k], ya = k ? a[N - k] : 0.0, xb = a[k + M], yb = a[M - k];
        const cplx w0 = wk[k], w1 = wk[k + M], t = tw[k];   // e^{-i pi k / 2N}, e^{-i pi (k + M) / 2N}, e^{-2 pi i k / N}
        const double c0 = w0.x, s0 = -w0.y, c1 = w1.x, s1 = -w1.y;
        const cplx Va{fma(c0, xa, s0 * ya), fma(s0, xa, -c0 * ya)};
        const cplx Vb{fma(c1, xb, s1 * yb), fma(s1, xb, -c1 * yb)};
        const cplx Ek{0.5 * (Va.x + Vb.x), 0.5 * (Va.y + Vb.y)};
        const cplx Ok = cmul(cplx{0.5 * (Va.x - Vb.x), 0.5 * (Va.y - Vb.y)}, cplx{t.x, -t.y});
        z[pz(k)] = cplx{Ek.x - Ok.y, -(Ek.y + Ok.x)};   // conj(E + i O)
    }
    __syncthreads();
    int Ns = 1;
#pragma unroll
    for (int st = 0; st < LOGM / 3; st++) {
        rfft_stage<LOGN, 8>(z, tw, tid, Ns, (FPS_RTW && LOGN <= 13) ? &W.w8[st] : nullptr);
        Ns *= 8;
    }
    if constexpr (LOGM % 3 != 0) rfft_stage<LOGN, (1 << (LOGM % 3))>(z, tw, tid, Ns, (FPS_RTW && LOGN <= 13) ? W.wl : nullptr);
    constexpr double rm = 1.0 / M;
    double* o = out + (size_t)r * ld;
    const double* zd = reinterpret_cast<const double*>(z);
#pragma unroll
    for (int q = 0; q < M / T; q++) {
        const int cb = tid + q * T, n1 = N - 1 - cb;
        // y_m = conj(Z_m) / M: v_2m = Z_m.x / M, v_2m+1 = -Z_m.y / M; x_2cb = v_cb, x_2cb+1 = v_{N-1-cb}
        const double e0 = zd[2 * pz(cb >> 1) + (cb & 1)], e1 = zd[2 * pz(n1 >> 1) + (n1 & 1)];
        st2(o + 2 * cb, (cb & 1) ? -e0 * rm : e0 * rm, (n1 & 1) ? -e1 * rm : e1 * rm);
    }
}

// (3) the inverse: DCT-III with x_j = X_0 / N + (2 / N) sum_k>0 X_k cos(pi k (2j+1) / 2N), through
// V_k = e^{i pi k / 2N} (X_k - i X_{N-k}) (X_N = 0), v = IFFT(V) = conj(FFT(conj(V))) / N.
// Persistent like k_fps_dct
template <int LOGN>
__global__ void __launch_bounds__(Fft<LOGN>::T) FPS_WAVES k_fps_idct(const double* __restrict__ in, double* __restrict__ out,
                                                            int nrows, int ld, const cplx* __restrict__ tw,
                                                            const cplx* __restrict__ wk,
                                                            const int32_t* __restrict__ fcm) {
    constexpr int N = Fft<LOGN>::N, T = Fft<LOGN>::T;
    constexpr int PT = (N + T - 1) / T;
    extern __shared__ cplx z[];
    int tid = threadIdx.x;
    const int npairs = (nrows + 1) / 2;
    const double rn = 1.0 / N;
    // (each thread loads its coefficients X_k and their mirrors X_{N-k} itself -- the mirrors are
    // the same cache lines, read in reverse -- so conj(V) goes to LDS in one pass.  N = 8192: the
    // mirrors' registers would spill; they come through LDS, one pass more)
    constexpr bool MIRROR = LOGN <= 12;
    constexpr int PM = MIRROR ? PT : 1;
    double ra[PT], rb[PT], na[PM], nb[PM];
    auto load = [&](int p) {
        const int r0 = 2 * p;
        const bool two = r0 + 1 < nrows;
        const double* a = in + (size_t)r0 * ld;
#pragma unroll
        for (int q = 0; q < PT; q++) {
            const int k = tid + q * T;
            if (k < N) {
                ra[q] = a[k];
                rb[q] = two ? a[ld + k] : 0.0;
                if constexpr (MIRROR) {
                    na[q] = k ? a[N - k] : 0.0;
                    nb[q] = two && k ? a[ld + N - k] : 0.0;
                }
            }
        }
    };
    constexpr bool PREF = FPS_PREF && LOGN <= 12;
    int p = blockIdx.x;
    constexpr bool REGIO = FPS_REGIO && FPS_LR == 4 && LOGN >= 10 && LOGN <= 13;
    if constexpr (REGIO) {
        // thread t forms conj(V_n), n = t + 256 r, from X_n and X_{N-n} of both rows, and writes
        // x_2n = Re z_n (n < N/2), x_{2(N-1-n)+1} (n >= N/2) straight from its last stage
        for (; p < npairs; p += gridDim.x) {
            fps_remat(tid);
            const int r0 = 2 * (FPS_SNAKE ? npairs - 1 - p : p);
            const bool two = r0 + 1 < nrows;
            const double* a = in + (size_t)r0 * ld;
            cplx v[16];
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int k = tid + r * T;
                const double xa = a[k], xb = two ? a[ld + k] : 0.0;
                const double ya = k ? a[N - k] : 0.0, yb = two && k ? a[ld + N - k] : 0.0;
                const cplx w = wk[k];   // e^{-i theta}: e^{i theta} = (w.x, -w.y)
                const double c = w.x, s = -w.y;
                const cplx Va{fma(c, xa, s * ya), fma(s, xa, -c * ya)};
                const cplx Vb{fma(c, xb, s * yb), fma(s, xb, -c * yb)};
                v[r] = cplx{Va.x - Vb.y, -(Va.y + Vb.x)};
            }
            fft_regs<LOGN>(z, tw, tid, v);
            double* oa = out + (size_t)r0 * ld;
            double* ob = oa + ld;
            if constexpr (FPS_ISTAGE) {
                // (staged through LDS: each lane then stores columns 2m, 2m + 1 of both rows as 16 B --
                // the direct stores of x_2n / x_{2n+1} from the registers left every line half-written
                // at a time: rocprofv3 WRITE_SIZE 1.34x of phi's bytes)
                __syncthreads();   // (every thread has read its last stage's inputs)
#pragma unroll
                for (int r = 0; r < 16; r++) z[pz(tid + r * T)] = v[r];
                __syncthreads();
                if (fcm) {   // (r6, a masked domain's solution: its cells only, the rest of `out` kept; codes loaded first)
                    int2 ca[8], cb[8];
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const int m = tid + q * T;
                        ca[q] = *reinterpret_cast<const int2*>(fcm + (size_t)r0 * ld + 2 * m);
                        cb[q] = *reinterpret_cast<const int2*>(fcm + (size_t)(two ? r0 + 1 : r0) * ld + 2 * m);
                    }
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const int m = tid + q * T;
                        const cplx e = z[pz(m)], o = z[pz(N - 1 - m)];
                        if (ca[q].x & FC_IN) oa[2 * m] = e.x * rn;
                        if (ca[q].y & FC_IN) oa[2 * m + 1] = o.x * rn;
                        if (two && (cb[q].x & FC_IN)) ob[2 * m] = -e.y * rn;
                        if (two && (cb[q].y & FC_IN)) ob[2 * m + 1] = -o.y * rn;
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const int m = tid + q * T;   // columns 2m (v_m) and 2m + 1 (v_{N-1-m})
                        const cplx e = z[pz(m)], o = z[pz(N - 1 - m)];
                        st2(oa + 2 * m, e.x * rn, o.x * rn);
                        if (two) st2(ob + 2 * m, -e.y * rn, -o.y * rn);
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int n = tid + r * T;
                    const int j = n < N / 2 ? 2 * n : 2 * (N - 1 - n) + 1;
                    if constexpr (FPS_NT) {   // (phi goes to HBM, not into the Infinity Cache as dirty lines)
                        __builtin_nontemporal_store(v[r].x * rn, oa + j);
                        if (two) __builtin_nontemporal_store(-v[r].y * rn, ob + j);
                    } else {
                        oa[j] = v[r].x * rn;
                        if (two) ob[j] = -v[r].y * rn;
                    }
                }
            }
            __syncthreads();   // (z is rewritten by the next pair)
        }
        return;
    }
    if (PREF && p < npairs) load(p);
    for (; p < npairs; p += gridDim.x) {
        fps_remat(tid);
        const int r0 = 2 * p;
        const bool two = r0 + 1 < nrows;
        if (!PREF) load(p);
        // Va = e^{i theta} (A_k - i A_{N-k}), Vb likewise; V = Va + i Vb; z <- conj(V)
        auto conjv = [&](int k, double xa, double xb, double ya, double yb) {
            const cplx w = wk[k];   // e^{-i theta}: e^{i theta} = (w.x, -w.y)
            const double c = w.x, s = -w.y;
            const cplx Va{fma(c, xa, s * ya), fma(s, xa, -c * ya)};
            const cplx Vb{fma(c, xb, s * yb), fma(s, xb, -c * yb)};
            return cplx{Va.x - Vb.y, -(Va.y + Vb.x)};
        };
        if constexpr (MIRROR) {
#pragma unroll
            for (int q = 0; q < PT; q++) {
                const int k = tid + q * T;
                if (k < N) z[pz(k)] = conjv(k, ra[q], rb[q], na[q], nb[q]);
            }
        } else {
#pragma unroll
            for (int q = 0; q < PT; q++) {
                const int k = tid + q * T;
                if (k < N) z[pz(k)] = cplx{ra[q], rb[q]};
            }
            __syncthreads();
            cplx v[PT];
#pragma unroll
            for (int q = 0; q < PT; q++) {
                const int k = tid + q * T;
                if (k < N) {
                    const cplx Xk = z[pz(k)];
                    const cplx Xn = k ? z[pz(N - k)] : cplx{0.0, 0.0};
                    v[q] = conjv(k, Xk.x, Xk.y, Xn.x, Xn.y);
                }
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < PT; q++) {
                const int k = tid + q * T;
                if (k < N) z[pz(k)] = v[q];
            }
        }
        __syncthreads();
        fft_lds<LOGN>(z, tw, tid);
        if (PREF && p + (int)gridDim.x < npairs) load(p + gridDim.x);
        double* oa = out + (size_t)r0 * ld;
        double* ob = oa + ld;
#pragma unroll
        for (int q = 0; q < PT; q++) {
            const int j = tid + q * T;
            if (j < N) {
                const int n = (j & 1) ? N - 1 - (j >> 1) : (j >> 1);
                const cplx y = z[pz(n)];
                oa[j] = y.x * rn;
                if (two) ob[j] = -y.y * rn;
            }
        }
        __syncthreads();
    }
}

// ---- (2) the tridiagonal systems along x, one per mode (column k of the transformed plane) ----
// Thomas on rows i (global gi): d_i = -(pw_i + pe_i) + mu_k, g_i = pw_i / p_{i-1},
// p_i = d_i - g_i pe_{i-1}, y_i = f_i - g_i y_{i-1}; back: x_i = y_i / p_i - (pe_i / p_i) x_{i+1}.
// Workgroup = FPS_G chunks (one wave each) x 128 modes (two per lane: 16-B loads, 1 KiB per wave
// and row).  rp0[c][k] = 1 / p of the row before chunk c.

// one row of the pivot recurrence: g = pw_i / p_{i-1} (from rprev = 1 / p_{i-1}); returns 1 / p_i
// (mode 0's pinned last global row: 0).  pw, pe, pem: the row's coefficients pw_i, pe_i, pe_{i-1}
// (r5) a NEUMANN outflow E side (a.outE, uniform hx): the last row 0.5 x_{n-3} - x_{n-2} + (0.5 + mu h^2) x_{n-1}
// (AddGhostStencils' 2.5 / -2 / 0.5 ghost, FluidSolver.cpp:98-101, 147-163) minus half the row above it is
// tridiagonal again: (-mu / 2) x_{n-2} + mu x_{n-1} = f_{n-1} - f_{n-2} / 2 (the transform of that rhs row is
// formed by k_fps_dct / k_fps_dct_div)
__device__ inline double piv_next(const FpsArgs& a, int gi, int k, double mu, double rprev, double pw, double pe,
                                  double pem, double& g) {
    const bool oe = a.outE && gi == a.nx - 1;
    g = (oe ? -0.5 * mu : pw) * rprev;
    // (r5: an explicit fma -- fps_setup's host recurrences use the same one, so host and device pivots are the
    // same bits and the block fixed points of FpsArgs::prowb are exact)
    const double p = fma(-g, pem, oe ? mu : -(pw + pe) + mu);
    return (a.pin && k == 0 && gi == a.nx - 1) ? 0.0 : 1.0 / p;
}


// a raw coefficient pair of row li, modes k0, k0 + 1; with the transform fused into K3 (sh0) mode 0
// takes N mean off here (the DCT of the constant; x - 0.0 is exact for every other mode)
// (branch-free: a branch per row would keep the chunk's row loads from being issued together)
// (r5) the pivots of a mode pair's row without the fp64 division chain where they are tabled (FpsArgs::ptab):
// a wave whose modes all converge (k >= kfast) reads 1 / p of rows < prow from the table and the converged
// 1 / p after (pinf); the last global row (no east neighbour) and the slow modes keep piv_next
// (pb: the first global row of this mode block's fixed point -- 0 with the table, prowb's entry without)
__device__ inline int fps_prow_block(const FpsArgs& a) {
    if (a.prowb) return a.prowb[blockIdx.x];
    return a.ptab && (int)(blockIdx.x * 128) >= a.kfast ? 0 : (1 << 30);
}
__device__ inline void piv_pair(const FpsArgs& a, bool fast, double2 pinf, int gi, int k0, const double (&mu)[2],
                                double (&r)[2], double pw, double pe, double pem, double& g0, double& g1, int pb) {
    if (fast && gi >= pb && gi != a.nx - 1) {
        g0 = pw * r[0];
        g1 = pw * r[1];
        const double2 t = a.ptab && gi < a.prow ? ld2(a.ptab + (size_t)gi * a.ld + k0) : pinf;
        r[0] = t.x;
        r[1] = t.y;
    } else {
        r[0] = piv_next(a, gi, k0, mu[0], r[0], pw, pe, pem, g0);
        r[1] = piv_next(a, gi, k0 + 1, mu[1], r[1], pw, pe, pem, g1);
    }
}

// (r5) with an outflow side mode 0 is solved in the projected sense of the BiCGStab path (P A x = P b: A x =
// b + C 1 for the C that makes it consistent).  Its eliminated last row is 0 = f'_{n-1} + C / 2, so
// C = -2 f'_{n-1}, known from the transform alone: every row's mode 0 takes it as this shift (the pinned
// last row ignores its own).  t1b reads it from the plane f (not yet overwritten), k_fps_mid stores it in
// *a.s0 for t2b (which overwrites the plane)
__device__ inline double mode0_shift(const FpsArgs& a, int k0, const double* f = nullptr) {
    if (k0 != 0) return 0.0;
    if (a.outE) return f && !a.s0_given ? 2.0 * f[(size_t)(a.nxl - 1) * a.ld] : *a.s0;
    return a.sh0 ? (a.sh0s != 0.0 ? a.sh0s : (double)a.ny) * *a.sh0 : 0.0;
}
__device__ inline double2 ldf0(const FpsArgs& a, const double* f, int li, int k0, double s0) {
    double2 x = ld2(f + (size_t)li * a.ld + k0);
    x.x -= s0;
    return x;
}

// a chunk's rows: every load issued before the recurrence consumes the first (the recurrence is a
// dependent chain of divisions; one row in flight at a time left the passes at 3 TB/s)
struct ChunkRows {
    double pw[FPS_M], pe[FPS_M], pem[FPS_M];
    // (r6) branch-free, rows past the chunk's end clamped onto its last (their values unused): a per-row
    // `t < rows` branch serialised the loads -- one scalar round trip per row
    __device__ inline void load(const FpsArgs& a, int li0, int rows) {
        (void)rows;
#pragma unroll
        for (int t = 0; t < FPS_M; t++) {
            const int gi = a.i0 + min(li0 + t, a.nxl - 1);
            pw[t] = a.pw[gi];
            pe[t] = a.pe[gi];
            const double pm = a.pe[max(gi - 1, 0)];
            pem[t] = gi > 0 ? pm : 0.0;
        }
    }
    // (r6) the same values by ONE vector load per wave -- lanes 0-15 pw, 16-31 pe, 32-47 the row before's pe --
    // and lane reads into scalars: 48 scalar loads waited in small groups cost k_fps_t1b ~9 us.  Every lane of
    // the wave must run it (call before any divergent branch)
    __device__ inline void load_wave(const FpsArgs& a, int li0) {
        if constexpr (3 * FPS_M > 64) {   // (a taller chunk, FPS_ROWS A/B builds: the scalar loads)
            load(a, li0, FPS_M);
            return;
        }
        const int lane = threadIdx.x & 63, t = lane % FPS_M, kind = lane / FPS_M;
        const int gi = a.i0 + min(li0 + t, a.nxl - 1);
        const int gk = kind == 2 ? max(gi - 1, 0) : gi;
        const double* src = kind == 0 ? a.pw : a.pe;
        double v = kind < 3 ? src[gk] : 0.0;
        if (kind == 2 && gi == 0) v = 0.0;
        const int lo = __double2loint(v), hi = __double2hiint(v);
        auto rd = [&](int l) {
            return __hiloint2double(__builtin_amdgcn_readlane(hi, l), __builtin_amdgcn_readlane(lo, l));
        };
#pragma unroll
        for (int q = 0; q < FPS_M; q++) {
            pw[q] = rd(q);
            pe[q] = rd(FPS_M + q);
            pem[q] = rd(2 * FPS_M + q);
        }
    }
};

// T1: per chunk the forward recurrence from zero -> (E, Pi) into ca; the workgroup folds its chunks
// into the group's aggregate ga (y_out = E + Pi y_in)
__global__ void __launch_bounds__(64 * FPS_G) k_fps_t1(FpsArgs a, const double* __restrict__ f) {
    __shared__ double2 sE[FPS_G][64], sP[FPS_G][64];
    const int lane = threadIdx.x, w = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const int k0 = 2 * (blockIdx.x * 64 + lane);
    const int grp = blockIdx.y, c = grp * FPS_G + w;
    const int li0 = c * FPS_M;
    const int rows = k0 < a.ny ? min(FPS_M, a.nxl - li0) : 0;
    double E[2] = {0.0, 0.0}, P[2] = {1.0, 1.0};
    if (rows > 0) {
        const double mu[2] = {a.mu[k0], a.mu[k0 + 1]};
        const double2 r0 = ld2(a.rp0 + (size_t)c * a.ld + k0);
        const double s0 = mode0_shift(a, k0);
        ChunkRows cr;
        cr.load(a, li0, rows);
        double2 fv[FPS_M];
#pragma unroll
        for (int t = 0; t < FPS_M; t++)
            if (t < rows) fv[t] = ldf0(a, f, li0 + t, k0, s0);
        double r[2] = {r0.x, r0.y};
#pragma unroll
        for (int t = 0; t < FPS_M; t++) {
            if (t < rows) {
                const int gi = a.i0 + li0 + t;
                const double fm[2] = {fv[t].x, fv[t].y};
#pragma unroll
                for (int m = 0; m < 2; m++) {
                    double g;
                    r[m] = piv_next(a, gi, k0 + m, mu[m], r[m], cr.pw[t], cr.pe[t], cr.pem[t], g);
                    E[m] = fma(-g, E[m], fm[m]);
                    P[m] = -g * P[m];
                }
            }
        }
        st2(a.ca + (size_t)c * a.ld + k0, E[0], E[1]);
        st2(a.ca + (size_t)(a.nch + c) * a.ld + k0, P[0], P[1]);
    }
    sE[w][lane] = double2{E[0], E[1]};
    sP[w][lane] = double2{P[0], P[1]};
    __syncthreads();
    if (w == 0 && k0 < a.ny) {
        double GE[2] = {0.0, 0.0}, GP[2] = {1.0, 1.0};
        for (int q = 0; q < FPS_G; q++) {
            const double2 e = sE[q][lane], pp = sP[q][lane];
            GE[0] = fma(pp.x, GE[0], e.x);
            GE[1] = fma(pp.y, GE[1], e.y);
            GP[0] = pp.x * GP[0];
            GP[1] = pp.y * GP[1];
        }
        st2(a.ga + (size_t)grp * a.ld + k0, GE[0], GE[1]);
        st2(a.ga + (size_t)(a.ngrp + grp) * a.ld + k0, GP[0], GP[1]);
    }
}

// multi-rank: this rank's carry-in of mode k from every rank's gathered aggregate (R.gath: P slots of
// R.stride doubles, rank q's (E, Pi) or (X, R) in slot q) -- forward the fold of ranks 0 .. r-1 in order,
// backward of P-1 .. r+1 (r4's k_fps_rank_carry, now inside the scan: two launches less per solve).
// Deferred mean (r5, forward, R.a1): the aggregates were formed from b's raw mode-0 coefficients; the
// gathered (sum b, sum b^2) of every rank (at 2 ld of its slot) give the mean, and mode 0's aggregates are
// corrected by the linear response to the constant ny mean (a1: every rank's aggregate of the constant 1;
// the group aggregates through sft0 in the scan).  Returns the carry-in; *sft0 = ny mean (0 without)
__device__ inline double fps_rank_in(const FpsRank& R, int k, int ld, int ny, bool backward, double* sft0) {
    double sft = 0.0;
    if (R.a1) {
        double S = 0.0, S2 = 0.0;
        for (int q = 0; q < R.P; q++) {
            S += R.gath[(size_t)q * R.stride + 2 * (size_t)ld];
            S2 += R.gath[(size_t)q * R.stride + 2 * (size_t)ld + 1];
        }
        const double mean = S / R.ncells;
        sft = ny * mean;
        if (k == 0 && R.shift) {   // MatNullSpaceRemove's mean and ||b - mean||^2 (k_finish_mean's arithmetic)
            R.shift[0] = mean;
            R.shift[1] = fmax(S2 - S * S / R.ncells, 0.0);
        }
    }
    *sft0 = k == 0 ? sft : 0.0;
    double Y = 0.0;
    if (!R.gath) return Y;
    if (backward && R.bq) {
        // (r5, one allgather) every rank's forward carry-in, then the backward fold of the ranks after this one
        constexpr int PMAX = 64;
        double yin[PMAX];
        double Yf = 0.0;
        for (int q = 0; q < R.P && q < PMAX; q++) {
            yin[q] = Yf;
            const double E = R.gath[(size_t)q * R.stride + k] - (R.a1 ? *sft0 * R.a1[q] : 0.0);
            Yf = fma(R.gath[(size_t)q * R.stride + ld + k], Yf, E);
        }
        const size_t ox = 2 * (size_t)ld + 8;
        for (int q = R.P - 1; q > R.r; q--) {
            const double* sl = R.gath + (size_t)q * R.stride;
            const double X0 = sl[ox + k] - (R.x1 ? *sft0 * R.x1[q] : 0.0);
            Y = fma(sl[ox + ld + k], Y, fma(R.bq[(size_t)q * ld + k], yin[q], X0));
        }
        return Y;
    }
    if (!backward) {
        for (int q = 0; q < R.r; q++) {
            const double E = R.gath[(size_t)q * R.stride + k] - (R.a1 ? *sft0 * R.a1[q] : 0.0);
            Y = fma(R.gath[(size_t)q * R.stride + ld + k], Y, E);
        }
    } else {
        for (int q = R.P - 1; q > R.r; q--)
            Y = fma(R.gath[(size_t)q * R.stride + ld + k], Y, R.gath[(size_t)q * R.stride + k]);
    }
    return Y;
}

// S1 / S2: scan of the group aggregates per mode -> each group's carry-in (forward: ascending,
// backward: descending), from the carry-in of the ranks before / after (R, fps_rank_in; one rank: 0);
// rout (if not null): this rank's aggregate (the fold of all its groups)
__global__ void k_fps_scan(int ngrp, int ld, int ny, const double* __restrict__ agg, double* __restrict__ carry,
                           FpsRank R, double* __restrict__ rout, int backward) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= ny) return;
    double sft0 = 0.0;
    double Y = fps_rank_in(R, k, ld, ny, backward, &sft0), AE = 0.0, AP = 1.0;
    constexpr int B = 8;   // (the loads of B groups in flight together: the fold is a dependent chain)
    for (int q0 = 0; q0 < ngrp; q0 += B) {
        double E[B], P[B];
#pragma unroll
        for (int t = 0; t < B; t++) {
            const int q = q0 + t;
            const int grp = backward ? ngrp - 1 - q : q;
            E[t] = q < ngrp ? agg[(size_t)grp * ld + k] - (R.ge1 ? sft0 * R.ge1[grp] : 0.0) : 0.0;
            P[t] = q < ngrp ? agg[(size_t)(ngrp + grp) * ld + k] : 1.0;
        }
#pragma unroll
        for (int t = 0; t < B; t++) {
            const int q = q0 + t;
            if (q < ngrp) {
                const int grp = backward ? ngrp - 1 - q : q;
                carry[(size_t)grp * ld + k] = Y;
                Y = fma(P[t], Y, E[t]);
                AE = fma(P[t], AE, E[t]);
                AP = P[t] * AP;
            }
        }
    }
    if (rout) {
        rout[k] = AE;
        rout[ld + k] = AP;
    }
}

// The same scan with the groups cut into FPS_SSEG segments per mode (one wave each, modes across the
// lanes): every wave folds its segment from zero, the first wave folds the segments' aggregates in
// order into their carry-ins (and the rank's aggregate), then every wave walks its segment again from
// its carry-in -- a chain of ngrp / S + S dependent steps instead of ngrp (the single-thread-per-mode
// scan's 64 groups at 4096^2 took 9 us a direction).  The same affine maps composed in another
// grouping (~1 ulp apart).  FPS_SSEG = 1: k_fps_scan (A/B)
#ifndef FPS_SSEG
#define FPS_SSEG 8
#endif
template <int S>
__global__ void __launch_bounds__(64 * S) k_fps_scan_seg(int ngrp, int ld, int ny, const double* __restrict__ agg,
                                                         double* __restrict__ carry, FpsRank R,
                                                         double* __restrict__ rout, int backward) {
    __shared__ double sE[S][64], sP[S][64], sY[S][64];
    const int lane = threadIdx.x, s = threadIdx.y;
    const int k = blockIdx.x * 64 + lane;
    const int per = (ngrp + S - 1) / S, q0 = s * per, q1 = min(ngrp, q0 + per);
    constexpr int B = 8;
    auto gq = [&](int q) { return backward ? ngrp - 1 - q : q; };
    // (the rank carry-in and the deferred mean's mode-0 shift: every segment needs the shift, wave 0 the carry)
    double sft0 = 0.0, Yin = 0.0;
    if (k < ny) Yin = fps_rank_in(s == 0 ? R : FpsRank{R.gath, R.P, R.r, R.stride, R.a1, R.ge1, R.ncells, nullptr},
                                  k, ld, ny, backward, &sft0);
    auto ge = [&](int q) { return agg[(size_t)gq(q) * ld + k] - (R.ge1 ? sft0 * R.ge1[gq(q)] : 0.0); };
    double AE = 0.0, AP = 1.0;
    if (k < ny) {
        for (int qb = q0; qb < q1; qb += B) {
            double E[B], P[B];
#pragma unroll
            for (int t = 0; t < B; t++) {   // (r6: clamped loads, then the select -- no branch around them)
                const int q = qb + t, qc = min(q, q1 - 1);
                const double e = ge(qc), pv = agg[(size_t)(ngrp + gq(qc)) * ld + k];
                E[t] = q < q1 ? e : 0.0;
                P[t] = q < q1 ? pv : 1.0;
            }
#pragma unroll
            for (int t = 0; t < B; t++) {
                AE = fma(P[t], AE, E[t]);
                AP = P[t] * AP;
            }
        }
    }
    sE[s][lane] = AE;
    sP[s][lane] = AP;
    __syncthreads();
    if (s == 0 && k < ny) {
        double Y = Yin, TE = 0.0, TP = 1.0;
        for (int t = 0; t < S; t++) {
            sY[t][lane] = Y;
            Y = fma(sP[t][lane], Y, sE[t][lane]);
            TE = fma(sP[t][lane], TE, sE[t][lane]);
            TP = sP[t][lane] * TP;
        }
        if (rout) {
            rout[k] = TE;
            rout[ld + k] = TP;
        }
    }
    __syncthreads();
    if (k < ny) {
        double Y = sY[s][lane];
        for (int qb = q0; qb < q1; qb += B) {
            double E[B], P[B];
#pragma unroll
            for (int t = 0; t < B; t++) {   // (r6: clamped loads, then the select -- no branch around them)
                const int q = qb + t, qc = min(q, q1 - 1);
                const double e = ge(qc), pv = agg[(size_t)(ngrp + gq(qc)) * ld + k];
                E[t] = q < q1 ? e : 0.0;
                P[t] = q < q1 ? pv : 1.0;
            }
#pragma unroll
            for (int t = 0; t < B; t++) {
                const int q = qb + t;
                if (q < q1) {
                    carry[(size_t)gq(q) * ld + k] = Y;
                    Y = fma(P[t], Y, E[t]);
                }
            }
        }
    }
}

// T2: the chunk's carry-in (the group's, through the group's earlier chunks: T1's aggregates), the
// exact forward values from it, then the back substitution from zero -> xl (in place over f) and the
// chunk's backward aggregate (x_s = BX + BR x_e) into cb; the workgroup folds its chunks into gb
__global__ void __launch_bounds__(64 * FPS_G) k_fps_t2(FpsArgs a, double* __restrict__ f) {
    __shared__ double2 sX[FPS_G][64], sR[FPS_G][64];
    const int lane = threadIdx.x, w = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const int k0 = 2 * (blockIdx.x * 64 + lane);
    const int grp = blockIdx.y, c = grp * FPS_G + w;
    const int li0 = c * FPS_M;
    const int rows = k0 < a.ny ? min(FPS_M, a.nxl - li0) : 0;
    double BX[2] = {0.0, 0.0}, BR[2] = {1.0, 1.0};
    if (rows > 0) {
        const double s0 = mode0_shift(a, k0);
        ChunkRows cr;
        cr.load(a, li0, rows);
        double2 yv[FPS_M];   // f, then the exact forward values in place
#pragma unroll
        for (int t = 0; t < FPS_M; t++)
            yv[t] = ldf0(a, f, min(li0 + t, a.nxl - 1), k0, s0);   // (r6: unconditional, clamped: pipelined)
        const double2 y0 = ld2(a.gc + (size_t)grp * a.ld + k0);
        double y[2] = {y0.x, y0.y};
        for (int q = grp * FPS_G; q < c; q++) {
            const double2 e = ld2(a.ca + (size_t)q * a.ld + k0), pp = ld2(a.ca + (size_t)(a.nch + q) * a.ld + k0);
            y[0] = fma(pp.x, y[0], e.x);
            y[1] = fma(pp.y, y[1], e.y);
        }
        const double mu[2] = {a.mu[k0], a.mu[k0 + 1]};
        const double2 r0 = ld2(a.rp0 + (size_t)c * a.ld + k0);
        double r[2] = {r0.x, r0.y};
        double2 rv[FPS_M];
#pragma unroll
        for (int t = 0; t < FPS_M; t++) {
            if (t < rows) {
                const int gi = a.i0 + li0 + t;
                double g0, g1;
                r[0] = piv_next(a, gi, k0, mu[0], r[0], cr.pw[t], cr.pe[t], cr.pem[t], g0);
                r[1] = piv_next(a, gi, k0 + 1, mu[1], r[1], cr.pw[t], cr.pe[t], cr.pem[t], g1);
                y[0] = fma(-g0, y[0], yv[t].x);
                y[1] = fma(-g1, y[1], yv[t].y);
                yv[t] = double2{y[0], y[1]};
                rv[t] = double2{r[0], r[1]};
            }
        }
        double xl[2] = {0.0, 0.0};
#pragma unroll
        for (int t = FPS_M - 1; t >= 0; t--) {
            if (t < rows) {
                const double q0 = -cr.pe[t] * rv[t].x, q1 = -cr.pe[t] * rv[t].y;
                xl[0] = fma(yv[t].x, rv[t].x, q0 * xl[0]);
                xl[1] = fma(yv[t].y, rv[t].y, q1 * xl[1]);
                BR[0] = q0 * BR[0];
                BR[1] = q1 * BR[1];
                st2(f + (size_t)(li0 + t) * a.ld + k0, xl[0], xl[1]);
            }
        }
        BX[0] = xl[0];
        BX[1] = xl[1];
        st2(a.cb + (size_t)c * a.ld + k0, BX[0], BX[1]);
        st2(a.cb + (size_t)(a.nch + c) * a.ld + k0, BR[0], BR[1]);
    }
    sX[w][lane] = double2{BX[0], BX[1]};
    sR[w][lane] = double2{BR[0], BR[1]};
    __syncthreads();
    if (w == 0 && k0 < a.ny) {
        double GX[2] = {0.0, 0.0}, GR[2] = {1.0, 1.0};
        for (int q = FPS_G - 1; q >= 0; q--) {
            const double2 x = sX[q][lane], rr = sR[q][lane];
            GX[0] = fma(rr.x, GX[0], x.x);
            GX[1] = fma(rr.y, GX[1], x.y);
            GR[0] = rr.x * GR[0];
            GR[1] = rr.y * GR[1];
        }
        st2(a.gb + (size_t)grp * a.ld + k0, GX[0], GX[1]);
        st2(a.gb + (size_t)(a.ngrp + grp) * a.ld + k0, GR[0], GR[1]);
    }
}

// T3: the chunk's carry-in from the next chunk (the group's carry through its later chunks), then
// x_i = xl_i + rho_i x_e (in place)
__global__ void __launch_bounds__(64 * FPS_G) k_fps_t3(FpsArgs a, double* __restrict__ f) {
    __shared__ double2 sX[FPS_G][64], sR[FPS_G][64];
    const int lane = threadIdx.x, w = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const int k0 = 2 * (blockIdx.x * 64 + lane);
    const int grp = blockIdx.y, c = grp * FPS_G + w;
    const int li0 = c * FPS_M;
    const int rows = k0 < a.ny ? min(FPS_M, a.nxl - li0) : 0;
    double2 bx{0.0, 0.0}, br{1.0, 1.0};
    if (rows > 0) {
        bx = ld2(a.cb + (size_t)c * a.ld + k0);
        br = ld2(a.cb + (size_t)(a.nch + c) * a.ld + k0);
    }
    sX[w][lane] = bx;
    sR[w][lane] = br;
    __syncthreads();
    if (rows <= 0) return;
    ChunkRows cr;
    cr.load(a, li0, rows);
    double2 xv[FPS_M];
#pragma unroll
    for (int t = 0; t < FPS_M; t++)
        if (t < rows) xv[t] = ld2(f + (size_t)(li0 + t) * a.ld + k0);
    const double2 x0 = ld2(a.gx + (size_t)grp * a.ld + k0);
    double X[2] = {x0.x, x0.y};
    for (int q = FPS_G - 1; q > w; q--) {
        const double2 x = sX[q][lane], rr = sR[q][lane];
        X[0] = fma(rr.x, X[0], x.x);
        X[1] = fma(rr.y, X[1], x.y);
    }
    const double mu[2] = {a.mu[k0], a.mu[k0 + 1]};
    const double2 r0 = ld2(a.rp0 + (size_t)c * a.ld + k0);
    double r[2] = {r0.x, r0.y};
    double2 rv[FPS_M];
#pragma unroll
    for (int t = 0; t < FPS_M; t++) {
        if (t < rows) {
            const int gi = a.i0 + li0 + t;
            double g;
            r[0] = piv_next(a, gi, k0, mu[0], r[0], cr.pw[t], cr.pe[t], cr.pem[t], g);
            r[1] = piv_next(a, gi, k0 + 1, mu[1], r[1], cr.pw[t], cr.pe[t], cr.pem[t], g);
            rv[t] = double2{r[0], r[1]};
        }
    }
    double rho[2] = {1.0, 1.0};
#pragma unroll
    for (int t = FPS_M - 1; t >= 0; t--) {
        if (t < rows) {
            rho[0] = -cr.pe[t] * rv[t].x * rho[0];
            rho[1] = -cr.pe[t] * rv[t].y * rho[1];
            st2(f + (size_t)(li0 + t) * a.ld + k0, fma(rho[0], X[0], xv[t].x), fma(rho[1], X[1], xv[t].y));
        }
    }
}

// ---- the same recurrences in two full passes (r4, default; NSGPU_FPS_PASSES=3: t1 / t2 / t3 above) ----
// A chunk's back substitution from zero over its exact forward values y' = y_loc + pi Y_in is linear in
// the carry-in: its start value is BXl + beta Y_in, where BXl runs the back substitution over y_loc
// and beta = the same recurrence over pi -- with BR (the product of the back multipliers) a property
// of the operator alone, tabulated by the host (bt).  So T1b forms (E, Pi) and BXl from f, the
// forward scan gives the carries, k_fps_mid forms every chunk's carry-in and final (BX, BR) and the
// groups' backward aggregates, the backward scan gives their carries, and T2b writes the exact values:
// f is read twice and written once (24 B/cell) instead of read three times and written twice (40).

// T1b: t1 + the chunk's back substitution from zero over its local forward values -> BXl into cb.
// (FPS_SNAKE: the groups walk down the slab -- the transform's last rows first, while the Infinity Cache
// still holds them; t2b then walks up, and the inverse transform down again)
__global__ void __launch_bounds__(64 * FPS_G) k_fps_t1b(FpsArgs a, const double* __restrict__ f) {
    __shared__ double2 sE[FPS_G][64], sP[FPS_G][64];
    const int lane = threadIdx.x, w = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const int k0 = 2 * (blockIdx.x * 64 + lane);
    const int grp = FPS_SNAKE ? (int)gridDim.y - 1 - (int)blockIdx.y : (int)blockIdx.y, c = grp * FPS_G + w;
    const int li0 = c * FPS_M;
    const int rows = k0 < a.ny ? min(FPS_M, a.nxl - li0) : 0;
    double E[2] = {0.0, 0.0}, P[2] = {1.0, 1.0};
    ChunkRows cr;
    cr.load_wave(a, li0);   // (every lane, before the divergent branch)
    if (rows > 0) {
        const double mu[2] = {a.mu[k0], a.mu[k0 + 1]};
        const double2 r0 = ld2(a.rp0 + (size_t)c * a.ld + k0);
        const double s0 = mode0_shift(a, k0, f);
        double2 yv[FPS_M], rv[FPS_M];
#pragma unroll
        for (int t = 0; t < FPS_M; t++)
            yv[t] = ldf0(a, f, min(li0 + t, a.nxl - 1), k0, s0);   // (r6: unconditional, clamped: pipelined)
        double r[2] = {r0.x, r0.y};
        const int pb = fps_prow_block(a);
        const bool fast = pb < a.nx;
        const double2 pinf = fast ? ld2(a.pinf + k0) : double2{0.0, 0.0};
#pragma unroll
        for (int t = 0; t < FPS_M; t++) {
            if (t < rows) {
                const int gi = a.i0 + li0 + t;
                double g0, g1;
                piv_pair(a, fast, pinf, gi, k0, mu, r, cr.pw[t], cr.pe[t], cr.pem[t], g0, g1, pb);
                E[0] = fma(-g0, E[0], yv[t].x);
                E[1] = fma(-g1, E[1], yv[t].y);
                P[0] = -g0 * P[0];
                P[1] = -g1 * P[1];
                yv[t] = double2{E[0], E[1]};
                rv[t] = double2{r[0], r[1]};
            }
        }
        double xl[2] = {0.0, 0.0};
#pragma unroll
        for (int t = FPS_M - 1; t >= 0; t--) {
            if (t < rows) {
                xl[0] = fma(yv[t].x, rv[t].x, -cr.pe[t] * rv[t].x * xl[0]);
                xl[1] = fma(yv[t].y, rv[t].y, -cr.pe[t] * rv[t].y * xl[1]);
            }
        }
        st2(a.ca + (size_t)c * a.ld + k0, E[0], E[1]);
        st2(a.ca + (size_t)(a.nch + c) * a.ld + k0, P[0], P[1]);
        st2(a.cb + (size_t)c * a.ld + k0, xl[0], xl[1]);
    }
    sE[w][lane] = double2{E[0], E[1]};
    sP[w][lane] = double2{P[0], P[1]};
    __syncthreads();
    if (w == 0 && k0 < a.ny) {
        double GE[2] = {0.0, 0.0}, GP[2] = {1.0, 1.0};
        for (int q = 0; q < FPS_G; q++) {
            const double2 e = sE[q][lane], pp = sP[q][lane];
            GE[0] = fma(pp.x, GE[0], e.x);
            GE[1] = fma(pp.y, GE[1], e.y);
            GP[0] = pp.x * GP[0];
            GP[1] = pp.y * GP[1];
        }
        st2(a.ga + (size_t)grp * a.ld + k0, GE[0], GE[1]);
        st2(a.ga + (size_t)(a.ngrp + grp) * a.ld + k0, GP[0], GP[1]);
    }
}

// every chunk's forward carry-in (ya) and final backward aggregate (cb <- BXl + beta Y_in; BR from bt),
// and the group's backward aggregate gb; one thread per group and mode pair
__global__ void __launch_bounds__(64) k_fps_mid(FpsArgs a, const double* __restrict__ f) {
    const int k0 = 2 * (blockIdx.x * 64 + threadIdx.x);
    const int grp = blockIdx.y;
    if (k0 >= a.ny) return;
    if (a.outE && !a.s0_given && k0 == 0 && grp == 0) *a.s0 = mode0_shift(a, 0, f);   // (t2b overwrites the plane)
    const double2 y0 = ld2(a.gc + (size_t)grp * a.ld + k0);
    double Y[2] = {y0.x, y0.y};
    double BX[FPS_G][2], BR[FPS_G][2];
    // (r6) every chunk's loads first (clamped chunk index): inside the uniform `c < nch` branch below they were
    // issued chunk by chunk behind the carry's dependent chain
    double2 le[FPS_G], lp[FPS_G], lb[FPS_G], lbe[FPS_G], lbr[FPS_G];
#pragma unroll
    for (int w = 0; w < FPS_G; w++) {
        const int c = min(grp * FPS_G + w, a.nch - 1);
        le[w] = ld2(a.ca + (size_t)c * a.ld + k0);
        lp[w] = ld2(a.ca + (size_t)(a.nch + c) * a.ld + k0);
        lb[w] = ld2(a.cb + (size_t)c * a.ld + k0);
        lbe[w] = ld2(a.bt + (size_t)c * a.ld + k0);
        lbr[w] = ld2(a.bt + (size_t)(a.nch + c) * a.ld + k0);
    }
#pragma unroll
    for (int w = 0; w < FPS_G; w++) {
        const int c = grp * FPS_G + w;
        BX[w][0] = BX[w][1] = 0.0;
        BR[w][0] = BR[w][1] = 1.0;
        if (c < a.nch) {
            double2 e = le[w];
            const double2 pp = lp[w];
            double2 bl = lb[w];
            if (a.m0e && k0 == 0) {   // (r5, the deferred mean: t1b's mode 0 saw b's raw coefficients)
                const double sft = a.ny * *a.m0s;
                e.x -= sft * a.m0e[c];
                bl.x -= sft * a.m0b[c];
            }
            const double2 be = lbe[w], br = lbr[w];
            if (!a.mid_local) st2(a.ya + (size_t)c * a.ld + k0, Y[0], Y[1]);
            BX[w][0] = fma(be.x, Y[0], bl.x);
            BX[w][1] = fma(be.y, Y[1], bl.y);
            BR[w][0] = br.x;
            BR[w][1] = br.y;
            if (!a.mid_local) st2(a.cb + (size_t)c * a.ld + k0, BX[w][0], BX[w][1]);
            Y[0] = fma(pp.x, Y[0], e.x);
            Y[1] = fma(pp.y, Y[1], e.y);
        }
    }
    double GX[2] = {0.0, 0.0}, GR[2] = {1.0, 1.0};
#pragma unroll
    for (int w = FPS_G - 1; w >= 0; w--) {
        GX[0] = fma(BR[w][0], GX[0], BX[w][0]);
        GX[1] = fma(BR[w][1], GX[1], BX[w][1]);
        GR[0] = BR[w][0] * GR[0];
        GR[1] = BR[w][1] * GR[1];
    }
    st2(a.gb + (size_t)grp * a.ld + k0, GX[0], GX[1]);
    st2(a.gb + (size_t)(a.ngrp + grp) * a.ld + k0, GR[0], GR[1]);
}

// T2b: the chunk's exact values -- the forward recurrence from its carry-in Y_in (ya), the back
// substitution from its carry-in X_in (the group's, through the later chunks' (BX, BR)) -- in place
// (GHOST: the deep slabs' variant with a.ghost's two extra rows -- a separate build, since keeping the carries live
// to the end of the kernel cost the plain one 52 -> 63 us at 4096^2)
template <bool GHOST>
__global__ void __launch_bounds__(64 * FPS_G) k_fps_t2b(FpsArgs a, double* __restrict__ f) {
    const int lane = threadIdx.x, w = __builtin_amdgcn_readfirstlane(threadIdx.y);
    const int k0 = 2 * (blockIdx.x * 64 + lane);
    const int grp = blockIdx.y, c = grp * FPS_G + w;
    const int li0 = c * FPS_M;
    const int rows = k0 < a.ny ? min(FPS_M, a.nxl - li0) : 0;
    ChunkRows cr;
    cr.load_wave(a, li0);   // (every lane, before the divergent return)
    if (rows <= 0) return;
    const double s0 = mode0_shift(a, k0);
    double2 yv[FPS_M];
#pragma unroll
    for (int t = 0; t < FPS_M; t++)
        yv[t] = ldf0(a, f, min(li0 + t, a.nxl - 1), k0, s0);   // (r6: unconditional, clamped: pipelined)
    const double2 yin = ld2(a.ya + (size_t)c * a.ld + k0);
    const double2 x0 = ld2(a.gx + (size_t)grp * a.ld + k0);
    double X[2] = {x0.x, x0.y};
    for (int q = FPS_G - 1; q > w; q--) {
        const int cq = grp * FPS_G + q;
        if (cq >= a.nch) continue;
        const double2 bx = ld2(a.cb + (size_t)cq * a.ld + k0), br = ld2(a.bt + (size_t)(a.nch + cq) * a.ld + k0);
        X[0] = fma(br.x, X[0], bx.x);
        X[1] = fma(br.y, X[1], bx.y);
    }
    // (r5, a.ghost) the slab's last chunk: X is now the solution at the next slab's first row (the backward carry)
    if (GHOST && c == a.nch - 1 && a.i0 + a.nxl < a.nx) st2(f + (size_t)a.nxl * a.ld + k0, X[0], X[1]);
    const double mu[2] = {a.mu[k0], a.mu[k0 + 1]};
    const double2 r0 = ld2(a.rp0 + (size_t)c * a.ld + k0);
    double r[2] = {r0.x, r0.y}, y[2] = {yin.x, yin.y};
    double2 rv[FPS_M];
    const int pb = fps_prow_block(a);
    const bool fast = pb < a.nx;
    const double2 pinf = fast ? ld2(a.pinf + k0) : double2{0.0, 0.0};
#pragma unroll
    for (int t = 0; t < FPS_M; t++) {
        if (t < rows) {
            const int gi = a.i0 + li0 + t;
            double g0, g1;
            piv_pair(a, fast, pinf, gi, k0, mu, r, cr.pw[t], cr.pe[t], cr.pem[t], g0, g1, pb);
            y[0] = fma(-g0, y[0], yv[t].x);
            y[1] = fma(-g1, y[1], yv[t].y);
            yv[t] = double2{y[0], y[1]};
            rv[t] = double2{r[0], r[1]};
        }
    }
#pragma unroll
    for (int t = FPS_M - 1; t >= 0; t--) {
        if (t < rows) {
            X[0] = fma(yv[t].x, rv[t].x, -cr.pe[t] * rv[t].x * X[0]);
            X[1] = fma(yv[t].y, rv[t].y, -cr.pe[t] * rv[t].y * X[1]);
            st2(f + (size_t)(li0 + t) * a.ld + k0, X[0], X[1]);
        }
    }
    // (r5, a.ghost) the slab's first chunk: the previous slab's last row, one more back-substitution step from
    // its forward value (the forward carry yin) and pivot (r0: 1 / p of the row before the chunk)
    if (GHOST && c == 0 && a.i0 > 0) {
        // (the carries loaded again -- kept live through the loop they cost the kernel 10 VGPRs)
        const double2 yi = ld2(a.ya + k0), rq = ld2(a.rp0 + k0);
        const double pe = a.pe[a.i0 - 1];
        st2(f - (ptrdiff_t)a.ld + k0, fma(yi.x, rq.x, -pe * rq.x * X[0]), fma(yi.y, rq.y, -pe * rq.y * X[1]));
    }
}

bool fps_div_real(int logn, int outE);
template <int LOGN>
void idct_row(const double* in, double* out, int nrows, int ld, const void* tw, const void* wk, hipStream_t st) {
    const size_t lr = sizeof(cplx) * (size_t)RFft<LOGN>::M;
    lds_attr_once((const void*)k_fps_idct_r<LOGN>, (int)lr);
    hipEvent_t a, b;
    if (take_launch_timing(a, b))
        hipExtLaunchKernelGGL(k_fps_idct_r<LOGN>, dim3(nrows), dim3(RFft<LOGN>::T), lr, st, a, b, 0, in, out, nrows,
                              ld, (const cplx*)tw, (const cplx*)wk);
    else
        hipLaunchKernelGGL(k_fps_idct_r<LOGN>, dim3(nrows), dim3(RFft<LOGN>::T), lr, st, in, out, nrows, ld,
                           (const cplx*)tw, (const cplx*)wk);
}
template <int LOGN>
void dct_pair(bool inverse, const double* in, const double* shift, double* out, int nrows, int ld, const void* tw,
              const void* wk, hipStream_t st, int oe_pair, const int32_t* fcm = nullptr) {
    constexpr int T = Fft<LOGN>::T;
    const size_t lds = sizeof(cplx) * (size_t)FftLds<LOGN>::n;
    // (r6) one workgroup per row pair: 106.5 / 64.6 us at 4096^2 against 110.7 / 65.6 with r4-r5's one persistent
    // round of two per CU (profiles/r06/ab/fpsg_summary.txt); NSGPU_FPS_GRID=n: at most n workgroups (A/B)
    static const int fg = getenv("NSGPU_FPS_GRID") ? std::atoi(getenv("NSGPU_FPS_GRID")) : 0;
    const dim3 grid(std::min((nrows + 1) / 2, fg > 0 ? fg : 1 << 30));
    if constexpr (LOGN >= 10 && LOGN <= 13) {
        if (inverse && !fcm && fps_div_real(LOGN, 0)) {   // (r6: one row per workgroup, k_fps_idct_r)
            idct_row<LOGN>(in, out, nrows, ld, tw, wk, st);
            return;
        }
    }
    if (inverse) {
        lds_attr_once((const void*)k_fps_idct<LOGN>, (int)lds);
        hipEvent_t a, b;
        if (take_launch_timing(a, b))
            hipExtLaunchKernelGGL(k_fps_idct<LOGN>, grid, dim3(T), lds, st, a, b, 0, in, out, nrows, ld,
                                  (const cplx*)tw, (const cplx*)wk, fcm);
        else
            hipLaunchKernelGGL(k_fps_idct<LOGN>, grid, dim3(T), lds, st, in, out, nrows, ld, (const cplx*)tw,
                               (const cplx*)wk, fcm);
    } else {
        lds_attr_once((const void*)k_fps_dct<LOGN>, (int)lds);
        hipEvent_t a, b;
        if (take_launch_timing(a, b))
            hipExtLaunchKernelGGL(k_fps_dct<LOGN>, grid, dim3(T), lds, st, a, b, 0, in, shift, out, nrows, ld,
                                  (const cplx*)tw, (const cplx*)wk, oe_pair);
        else
            hipLaunchKernelGGL(k_fps_dct<LOGN>, grid, dim3(T), lds, st, in, shift, out, nrows, ld, (const cplx*)tw,
                               (const cplx*)wk, oe_pair);
    }
}

// (r6) the one-row-per-workgroup transform (k_fps_dct_div_r): 2 cnt workgroups; NSGPU_FPS_REAL=0: the pairs (A/B)
bool fps_div_real(int logn, int outE) {
    const char* e = getenv("NSGPU_FPS_REAL");   // (read per launch: the parity test switches it)
    return (!e || std::atoi(e) != 0) && !outE && logn >= 10 && logn <= 14;
}
template <int LOGN>
int div_row(const FpsDivArgs& a0, hipStream_t st) {
    if constexpr (LOGN >= 10 && LOGN <= 14) {
        constexpr int T = RFft<LOGN>::T;
        const size_t lds = sizeof(cplx) * (size_t)RFft<LOGN>::M;
        lds_attr_once((const void*)k_fps_dct_div_r<LOGN>, (int)lds);
        const dim3 grid(2 * a0.cnt);
        hipEvent_t a, b;
        if (take_launch_timing(a, b)) hipExtLaunchKernelGGL(k_fps_dct_div_r<LOGN>, grid, dim3(T), lds, st, a, b, 0, a0);
        else hipLaunchKernelGGL(k_fps_dct_div_r<LOGN>, grid, dim3(T), lds, st, a0);
        return (int)grid.x;
    }
    return -1;
}

template <int LOGN>
int div_pair(const FpsDivArgs& a0, hipStream_t st) {
    constexpr int T = Fft<LOGN>::T;
    const size_t lds = sizeof(cplx) * (size_t)FftLds<LOGN>::n;
    lds_attr_once((const void*)k_fps_dct_div<LOGN>, (int)lds);
    static const int fg = getenv("NSGPU_FPS_GRID") ? std::atoi(getenv("NSGPU_FPS_GRID")) : 0;   // (as dct_pair)
    const dim3 grid(std::min(a0.cnt, fg > 0 ? fg : 1 << 30));
    hipEvent_t a, b;
    if (take_launch_timing(a, b)) hipExtLaunchKernelGGL(k_fps_dct_div<LOGN>, grid, dim3(T), lds, st, a, b, 0, a0);
    else hipLaunchKernelGGL(k_fps_dct_div<LOGN>, grid, dim3(T), lds, st, a0);
    return (int)grid.x;
}

// ---- (r5) N = 16384 (configs[4]'s grid): the row pair's 16384-point FFT does not fit the LDS (256 KiB), so each
// row pair runs as two 8192-point transforms (fft_regs<13>, 128 KiB) in ONE persistent launch, one workgroup per CU:
//   forward, decimation in frequency: a_n = z_n + z_{n+N/2}, b_n = (z_n - z_{n+N/2}) W^n (n < N/2, W = e^{-2 pi i/N})
//     give Z_{2k} = FFT_{N/2}(a)_k and Z_{2k+1} = FFT_{N/2}(b)_k; the DCT's post-step pairs Z_k with Z_{N-k}, of the
//     same parity, so each half finishes on its own (its mirror through the LDS) and thread t stores
//     (X_{2k}, X_{2k+1}) of both rows as 16 B;
//   inverse, decimation in time: E = FFT_{N/2}(y_{2m}), O = FFT_{N/2}(y_{2m+1}), Y_n = E_n + W^n O_n,
//     Y_{n+N/2} = E_n - W^n O_n -- thread t holds E_n, O_n for the same n; the second half goes through the LDS
//     so that columns 2n, 2n + 1 leave as 16 B.
// HBM: the row pair read once and written once (16 B/cell), as the one-pass transforms of N <= 8192.
constexpr int N14 = 1 << 14, NH14 = N14 / 2, TH14 = NH14 / 16;

// forward: z_n = (x_a[j(n)], x_b[j(n)]) - shift, j(n) = 2n (n < N/2), 2(N-1-n)+1 after (Makhoul's order);
// oe_pair as k_fps_dct.  tw: e^{-2 pi i m/N} (m < N), tw8: e^{-2 pi i m/(N/2)}, wk[k] = e^{-i pi k/2N}
__global__ void __launch_bounds__(TH14) k_fps_dct14(const double* __restrict__ in, const double* shiftp,
                                                   double* __restrict__ out, int nrows, int ld,
                                                   const cplx* __restrict__ tw, const cplx* __restrict__ tw8,
                                                   const cplx* __restrict__ wk, int oe_pair) {
    extern __shared__ cplx z[];
    int tid = threadIdx.x;
    const int npairs = (nrows + 1) / 2;
    const double sh = shiftp ? *shiftp : 0.0;
    for (int p = blockIdx.x; p < npairs; p += gridDim.x) {
        const int r0 = 2 * p;
        const bool two = r0 + 1 < nrows;
        const double* a = in + (size_t)r0 * ld;
        double* oa = out + (size_t)r0 * ld;
        const double lam = p == oe_pair ? 0.5 : 0.0;
        double xe[2][16];   // X_{2k} of both rows, stored with X_{2k+1}
        // (one loop body for both halves: the two transforms' index arithmetic is not kept live together)
#pragma unroll 1
        for (int h = 0; h < 2; h++) {
            fps_remat(tid);
            // z_n (n < N/2) = x_{2n}, z_{n+N/2} = x_{N-1-2n}; h = 0: a_n = z_n + z_{n+N/2}, 1: b_n = (z_n - z_{n+N/2}) W^n
            cplx v[16];
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int n = tid + r * TH14;
                const int j0 = 2 * n, j1 = N14 - 1 - 2 * n;
                const double x0 = a[j0] - sh, x1 = a[j1] - sh;
                const cplx z0{x0, two ? a[ld + j0] - sh - lam * x0 : 0.0}, z1{x1, two ? a[ld + j1] - sh - lam * x1 : 0.0};
                v[r] = h ? cmul(csub(z0, z1), tw[n]) : cadd(z0, z1);
            }
            fft_regs<13>(z, tw8, tid, v);   // Z_{2k + h}, k = tid + r TH14
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 16; r++) z[pz(tid + r * TH14)] = v[r];
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int k = tid + r * TH14;
                // the mirror Z_{N-2k-h}: Z_{2(N/2-k)} (h = 0), Z_{2(N/2-1-k)+1} (h = 1)
                const cplx Zk = v[r], Zn = z[pz((NH14 - k - h) & (NH14 - 1))];
                const cplx Va{0.5 * (Zk.x + Zn.x), 0.5 * (Zk.y - Zn.y)};
                const cplx Vb{0.5 * (Zk.y + Zn.y), 0.5 * (Zn.x - Zk.x)};
                const cplx w = wk[2 * k + h];
                const double ya = fma(w.x, Va.x, -w.y * Va.y), yb = fma(w.x, Vb.x, -w.y * Vb.y);
                if (!h) {
                    xe[0][r] = ya;
                    xe[1][r] = yb;
                } else {
                    st2(oa + 2 * k, xe[0][r], ya);
                    if (two) st2(oa + ld + 2 * k, xe[1][r], yb);
                }
            }
            __syncthreads();   // (z is rewritten by the next transform)
        }
    }
}

// inverse: y_k = conj(V_k), V_k = e^{i pi k/2N} (X_k - i X_{N-k}) packed over the two rows (k_fps_idct's input
// step); E from the even k, O from the odd; x_{2n} = Re Y_n / N, x_{2n+1} = Re Y_{N-1-n} / N (row b: -Im)
__global__ void __launch_bounds__(TH14) k_fps_idct14(const double* __restrict__ in, double* __restrict__ out,
                                                    int nrows, int ld, const cplx* __restrict__ tw,
                                                    const cplx* __restrict__ tw8, const cplx* __restrict__ wk) {
    extern __shared__ cplx z[];
    int tid = threadIdx.x;
    const int npairs = (nrows + 1) / 2;
    const double rn = 1.0 / N14;
    for (int p = blockIdx.x; p < npairs; p += gridDim.x) {
        const int r0 = 2 * (FPS_SNAKE ? npairs - 1 - p : p);
        const bool two = r0 + 1 < nrows;
        const double* a = in + (size_t)r0 * ld;
        cplx e[16];   // E_n, then Y_n
#pragma unroll 1
        for (int h = 0; h < 2; h++) {
            fps_remat(tid);
            cplx v[16];
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int k = 2 * (tid + r * TH14) + h;
                const double xa = a[k], xb = two ? a[ld + k] : 0.0;
                const double ya = k ? a[N14 - k] : 0.0, yb = two && k ? a[ld + N14 - k] : 0.0;
                const cplx w = wk[k];   // e^{-i theta}: e^{i theta} = (w.x, -w.y)
                const double c = w.x, s = -w.y;
                const cplx Va{fma(c, xa, s * ya), fma(s, xa, -c * ya)};
                const cplx Vb{fma(c, xb, s * yb), fma(s, xb, -c * yb)};
                v[r] = cplx{Va.x - Vb.y, -(Va.y + Vb.x)};
            }
            fft_regs<13>(z, tw8, tid, v);   // E_n (h = 0), O_n (h = 1), n = tid + r TH14
            __syncthreads();   // (every thread has read its last stage's inputs)
            if (!h) {
#pragma unroll
                for (int r = 0; r < 16; r++) e[r] = v[r];
                continue;
            }
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const cplx t = cmul(v[r], tw[tid + r * TH14]);
                z[pz(tid + r * TH14)] = csub(e[r], t);   // Y_{n+N/2}
                e[r] = cadd(e[r], t);                    // Y_n
            }
            __syncthreads();
            double* oa = out + (size_t)r0 * ld;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int n = tid + r * TH14;
                const cplx o = z[pz(NH14 - 1 - n)];   // Y_{N-1-n} = Y_{(N/2-1-n)+N/2}
                st2(oa + 2 * n, e[r].x * rn, o.x * rn);
                if (two) st2(oa + ld + 2 * n, -e[r].y * rn, -o.y * rn);
            }
            __syncthreads();   // (z is rewritten by the next pair)
        }
    }
}

void dct14(bool inverse, const double* in, const double* shift, double* out, int nrows, int ld, const double* tw,
           const double* tw8, const double* wk, hipStream_t st, int oe_pair) {
    const size_t lds = sizeof(cplx) * (size_t)FftLds<13>::n;
    const dim3 grid(std::min((nrows + 1) / 2, device_cus()));   // (128 KiB of LDS: one workgroup per CU)
    hipEvent_t a, b;
    const bool tm = take_launch_timing(a, b);
    if (!inverse) {
        lds_attr_once((const void*)k_fps_dct14, (int)lds);
        if (tm) hipExtLaunchKernelGGL(k_fps_dct14, grid, dim3(TH14), lds, st, a, b, 0, in, shift, out, nrows, ld,
                                      (const cplx*)tw, (const cplx*)tw8, (const cplx*)wk, oe_pair);
        else hipLaunchKernelGGL(k_fps_dct14, grid, dim3(TH14), lds, st, in, shift, out, nrows, ld, (const cplx*)tw,
                                (const cplx*)tw8, (const cplx*)wk, oe_pair);
    } else {
        lds_attr_once((const void*)k_fps_idct14, (int)lds);
        if (tm) hipExtLaunchKernelGGL(k_fps_idct14, grid, dim3(TH14), lds, st, a, b, 0, in, out, nrows, ld,
                                      (const cplx*)tw, (const cplx*)tw8, (const cplx*)wk);
        else hipLaunchKernelGGL(k_fps_idct14, grid, dim3(TH14), lds, st, in, out, nrows, ld, (const cplx*)tw,
                                (const cplx*)tw8, (const cplx*)wk);
    }
}

}  // namespace

// ---- (r6) any even ny in [16, 8192] whose prime factors are 2, 3, 5, 7 (3072, 3000, 1000, ...):
// the same two transforms -- two rows per complex N-point FFT, Makhoul's reordering, the k_fps_dct / k_fps_idct
// pre- and post-processing -- through a mixed-radix Stockham FFT in LDS (radices 8, 4, 2 for the power of two,
// then 3, 5, 7), one stage per barrier pair: each thread reads its butterflies' R inputs, the block synchronises,
// then writes.  Twiddles w^r = e^{-2 pi i r k / (Ns R)} from the N-entry table (Ns R divides N); the odd radices'
// DFTs by their constant tables (O(R^2), R <= 7).  Not the power-of-two kernels' register-fed fast path: the
// general grids' direct solve, not the headline's
namespace {
constexpr int GT = 512;   // threads per workgroup: at most 8 butterflies of radix 2 per thread at N = 8192
struct GenFft {
    int N, nst;
    int rad[24];
};
__device__ constexpr double C3[3] = {1.0, -0.5, -0.5};
__device__ constexpr double S3[3] = {0.0, 0.86602540378443864676, -0.86602540378443864676};
__device__ constexpr double C5[5] = {1.0, 0.30901699437494742410, -0.80901699437494742410, -0.80901699437494742410,
                                     0.30901699437494742410};
__device__ constexpr double S5[5] = {0.0, 0.95105651629515357212, 0.58778525229247312917, -0.58778525229247312917,
                                     -0.95105651629515357212};
__device__ constexpr double C7[7] = {1.0, 0.62348980185873353053, -0.22252093395631440429, -0.90096886790241912624,
                                     -0.90096886790241912624, -0.22252093395631440429, 0.62348980185873353053};
__device__ constexpr double S7[7] = {0.0, 0.78183148246802980871, 0.97492791218182360702, 0.43388373911755812048,
                                     -0.43388373911755812048, -0.97492791218182360702, -0.78183148246802980871};
// X_k = sum_n v_n e^{-2 pi i n k / R}
template <int R>
__device__ inline void dftg(cplx* v) {
    if constexpr (R == 2 || R == 4 || R == 8) {
        dft<R>(v);
    } else {
        const double* C = R == 3 ? C3 : R == 5 ? C5 : C7;
        const double* S = R == 3 ? S3 : R == 5 ? S5 : S7;
        cplx x[R];
#pragma unroll
        for (int k = 0; k < R; k++) {
            cplx a = v[0];
#pragma unroll
            for (int n = 1; n < R; n++) {
                const int m = (n * k) % R;
                a = cadd(a, cmul(v[n], cplx{C[m], -S[m]}));
            }
            x[k] = a;
        }
#pragma unroll
        for (int k = 0; k < R; k++) v[k] = x[k];
    }
}
template <int R>
__device__ inline void stage_g(cplx* z, const cplx* __restrict__ tw, int N, int Ns) {
    constexpr int MB = (8192 / R + GT - 1) / GT;
    const int NB = N / R, tid = threadIdx.x;
    cplx v[MB][R];
#pragma unroll
    for (int b = 0; b < MB; b++) {
        const int jb = tid + b * GT;
        if (jb < NB)
#pragma unroll
            for (int r = 0; r < R; r++) v[b][r] = z[jb + r * NB];
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < MB; b++) {
        const int jb = tid + b * GT;
        if (jb < NB) {
            const int k = jb % Ns;
            if (Ns > 1) {
                const cplx w = tw[k * (N / (Ns * R))];
                cplx wr = w;
#pragma unroll
                for (int r = 1; r < R; r++) {
                    v[b][r] = cmul(v[b][r], wr);
                    if (r + 1 < R) wr = cmul(wr, w);
                }
            }
            dftg<R>(v[b]);
            const int d = (jb - k) * R + k;
#pragma unroll
            for (int r = 0; r < R; r++) z[d + r * Ns] = v[b][r];
        }
    }
    __syncthreads();
}
__device__ inline void fft_g(cplx* z, const cplx* __restrict__ tw, const GenFft& P) {
    int Ns = 1;
    for (int s = 0; s < P.nst; s++) {
        switch (P.rad[s]) {
        case 8: stage_g<8>(z, tw, P.N, Ns); break;
        case 4: stage_g<4>(z, tw, P.N, Ns); break;
        case 2: stage_g<2>(z, tw, P.N, Ns); break;
        case 3: stage_g<3>(z, tw, P.N, Ns); break;
        case 5: stage_g<5>(z, tw, P.N, Ns); break;
        default: stage_g<7>(z, tw, P.N, Ns); break;
        }
        Ns *= P.rad[s];
    }
}
// DCT-II of row pairs (k_fps_dct's arithmetic, any N of the plan)
__global__ void __launch_bounds__(GT) k_fps_dctg(const double* __restrict__ in, const double* shiftp,
                                                 double* __restrict__ out, int nrows, int ld, const cplx* __restrict__ tw,
                                                 const cplx* __restrict__ wk, int oe_pair, GenFft P) {
    extern __shared__ cplx z[];
    const int N = P.N, tid = threadIdx.x, npairs = (nrows + 1) / 2;
    const double sh = shiftp ? *shiftp : 0.0;
    for (int p = blockIdx.x; p < npairs; p += gridDim.x) {
        const int r0 = 2 * p;
        const bool two = r0 + 1 < nrows;
        const double* a = in + (size_t)r0 * ld;
        const double lam = p == oe_pair ? 0.5 : 0.0;
        for (int j = tid; j < N; j += GT) {
            const int n = (j & 1) ? N - 1 - (j >> 1) : (j >> 1);
            const double xa = a[j] - sh;
            z[n] = cplx{xa, two ? a[ld + j] - sh - lam * xa : 0.0};
        }
        __syncthreads();
        fft_g(z, tw, P);
        double* oa = out + (size_t)r0 * ld;
        double* ob = oa + ld;
        for (int k = tid; k < N; k += GT) {
            const cplx Zk = z[k], Zn = z[k ? N - k : 0];
            const cplx Va{0.5 * (Zk.x + Zn.x), 0.5 * (Zk.y - Zn.y)};
            const cplx Vb{0.5 * (Zk.y + Zn.y), 0.5 * (Zn.x - Zk.x)};
            const cplx w = wk[k];
            oa[k] = fma(w.x, Va.x, -w.y * Va.y);
            if (two) ob[k] = fma(w.x, Vb.x, -w.y * Vb.y);
        }
        __syncthreads();
    }
}
// DCT-III of row pairs (k_fps_idct's arithmetic)
__global__ void __launch_bounds__(GT) k_fps_idctg(const double* __restrict__ in, double* __restrict__ out, int nrows,
                                                  int ld, const cplx* __restrict__ tw, const cplx* __restrict__ wk,
                                                  GenFft P) {
    extern __shared__ cplx z[];
    const int N = P.N, tid = threadIdx.x, npairs = (nrows + 1) / 2;
    const double rn = 1.0 / N;
    for (int p = blockIdx.x; p < npairs; p += gridDim.x) {
        const int r0 = 2 * p;
        const bool two = r0 + 1 < nrows;
        const double* a = in + (size_t)r0 * ld;
        for (int k = tid; k < N; k += GT) {
            const double xa = a[k], xb = two ? a[ld + k] : 0.0;
            const double ya = k ? a[N - k] : 0.0, yb = two && k ? a[ld + N - k] : 0.0;
            const cplx w = wk[k];
            const double c = w.x, sn = -w.y;
            const cplx Va{fma(c, xa, sn * ya), fma(sn, xa, -c * ya)};
            const cplx Vb{fma(c, xb, sn * yb), fma(sn, xb, -c * yb)};
            z[k] = cplx{Va.x - Vb.y, -(Va.y + Vb.x)};
        }
        __syncthreads();
        fft_g(z, tw, P);
        double* oa = out + (size_t)r0 * ld;
        double* ob = oa + ld;
        for (int j = tid; j < N; j += GT) {
            const int n = (j & 1) ? N - 1 - (j >> 1) : (j >> 1);
            const cplx y = z[n];
            oa[j] = y.x * rn;
            if (two) ob[j] = -y.y * rn;
        }
        __syncthreads();
    }
}
// the radix plan of N (radices 8 / 4 / 2 first, then 3, 5, 7); false if N has another prime factor
bool gen_plan(int N, GenFft& P) {
    P.N = N;
    P.nst = 0;
    int m = N;
    while (m % 8 == 0) { P.rad[P.nst++] = 8; m /= 8; }
    if (m % 4 == 0) { P.rad[P.nst++] = 4; m /= 4; }
    if (m % 2 == 0) { P.rad[P.nst++] = 2; m /= 2; }
    for (int q : {3, 5, 7})
        while (m % q == 0 && P.nst < 24) { P.rad[P.nst++] = q; m /= q; }
    return m == 1;
}
}  // namespace

namespace {
__global__ __launch_bounds__(256) void k_dense_mats(const double* __restrict__ C, const double* __restrict__ shy,
                                                    double rsum, int N, double* __restrict__ F, double* __restrict__ G) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (size_t)N * N) return;
    const int j = (int)(t % N), k = (int)(t / N);   // column k of F^T / G: element (j, k)
    const double sq = shy[j];
    double f, gv;
    if (k == 0) {
        f = sq * sq * rsum;
        gv = rsum;
    } else {
        const double q = C[(size_t)(N - 1 - k) * N + j];
        f = q * sq;
        gv = q / sq;
    }
    F[(size_t)j * N + k] = f;     // F(k, j), column-major
    G[(size_t)k * N + j] = gv;    // G(j, k)
}
}  // namespace
void launch_dense_mats(const double* C, const double* shy, double rsum, int N, double* F, double* G, hipStream_t st) {
    const size_t n = (size_t)N * N;
    hipLaunchKernelGGL(k_dense_mats, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, C, shy, rsum, N, F, G);
}

bool fps_gen_ok(int ny) {
    GenFft P;
    return ny >= 16 && ny <= 8192 && ny % 2 == 0 && fps_log2(ny) < 0 && gen_plan(ny, P);
}

int fps_log2(int ny) {
    int l = 0;
    while ((1 << l) < ny) l++;
    return (1 << l) == ny && l >= FPS_LOGN_MIN && l <= FPS_LOGN_MAX ? l : -1;
}
int fps_log2x(int ny) { return ny == N14 ? 14 : fps_log2(ny); }

// (r6) the inverse transform storing only a masked domain's cells (the register-fed transforms: 1024 <= ny <= 8192,
// a power of two); false where that build is not there
bool fps_idct_mask_ok(int ny) {
    const int l = fps_log2(ny);
    return FPS_REGIO && FPS_LR == 4 && FPS_ISTAGE && l >= 10 && l <= 13;
}
int launch_fps_idct_masked(const double* in, double* out, int nrows, int ny, int ld, const double* tw, const double* wk,
                           hipStream_t st, const int32_t* fcm) {
    if (!fps_idct_mask_ok(ny)) return -1;
    switch (fps_log2(ny)) {
    case 10: dct_pair<10>(true, in, nullptr, out, nrows, ld, tw, wk, st, -1, fcm); break;
    case 11: dct_pair<11>(true, in, nullptr, out, nrows, ld, tw, wk, st, -1, fcm); break;
    case 12: dct_pair<12>(true, in, nullptr, out, nrows, ld, tw, wk, st, -1, fcm); break;
    case 13: dct_pair<13>(true, in, nullptr, out, nrows, ld, tw, wk, st, -1, fcm); break;
    default: return -1;
    }
    return 0;
}

int launch_fps_dct(bool inverse, const double* in, const double* shift, double* out, int nrows, int ny, int ld,
                   const double* tw, const double* wk, hipStream_t st, int oe_pair, const double* tw8) {
    if (ny == N14 && inverse && fps_div_real(14, 0)) {   // (r6: one row per workgroup, 1024 threads)
        idct_row<14>(in, out, nrows, ld, tw, wk, st);
        return 0;
    }
    if (ny == N14) {   // (r5: two 8192-point transforms per row pair)
        if (!tw8) return -1;
        dct14(inverse, in, shift, out, nrows, ld, tw, tw8, wk, st, oe_pair);
        return 0;
    }
    if (fps_gen_ok(ny)) {   // (r6) the mixed-radix transforms
        GenFft P;
        gen_plan(ny, P);
        const int npairs = (nrows + 1) / 2, lds = ny * (int)sizeof(cplx);
        const int nb = std::max(1, std::min(npairs, 1024));
        hipEvent_t ea, eb;
        const bool tm = take_launch_timing(ea, eb);   // (the solve's dispatch-stamped transform timing)
        if (inverse) {
            lds_attr_once((const void*)k_fps_idctg, lds);
            if (tm)
                hipExtLaunchKernelGGL(k_fps_idctg, dim3(nb), dim3(GT), lds, st, ea, eb, 0, in, out, nrows, ld,
                                      (const cplx*)tw, (const cplx*)wk, P);
            else
                hipLaunchKernelGGL(k_fps_idctg, dim3(nb), dim3(GT), lds, st, in, out, nrows, ld, (const cplx*)tw,
                                   (const cplx*)wk, P);
        } else {
            lds_attr_once((const void*)k_fps_dctg, lds);
            if (tm)
                hipExtLaunchKernelGGL(k_fps_dctg, dim3(nb), dim3(GT), lds, st, ea, eb, 0, in, shift, out, nrows, ld,
                                      (const cplx*)tw, (const cplx*)wk, oe_pair, P);
            else
                hipLaunchKernelGGL(k_fps_dctg, dim3(nb), dim3(GT), lds, st, in, shift, out, nrows, ld, (const cplx*)tw,
                                   (const cplx*)wk, oe_pair, P);
        }
        return 0;
    }
    switch (fps_log2(ny)) {
    case 4: dct_pair<4>(inverse, in, shift, out, nrows, ld, tw, wk, st, oe_pair); break;
    case 5: dct_pair<5>(inverse, in, shift, out, nrows, ld, tw, wk, st, oe_pair); break;
    case 6: dct_pair<6>(inverse, in, shift, out, nrows, ld, tw, wk, st, oe_pair); break;
    case 7: dct_pair<7>(inverse, in, shift, out, nrows, ld, tw, wk, st, oe_pair); break;
    case 8: dct_pair<8>(inverse, in, shift, out, nrows, ld, tw, wk, st, oe_pair); break;
    case 9: dct_pair<9>(inverse, in, shift, out, nrows, ld, tw, wk, st, oe_pair); break;
    case 10: dct_pair<10>(inverse, in, shift, out, nrows, ld, tw, wk, st, oe_pair); break;
    case 11: dct_pair<11>(inverse, in, shift, out, nrows, ld, tw, wk, st, oe_pair); break;
    case 12: dct_pair<12>(inverse, in, shift, out, nrows, ld, tw, wk, st, oe_pair); break;
    case 13: dct_pair<13>(inverse, in, shift, out, nrows, ld, tw, wk, st, oe_pair); break;
    default: return -1;
    }
    return 0;
}

int launch_fps_div(const Geo& g, const Coef& c, double dt, const double* u, const double* v, double* b, double* out,
                   double* part, int phase, const double* tw, const double* wk, hipStream_t st, int outE) {
    const int np = (g.nxl + 1) / 2;
    FpsDivArgs a{g, c, 1.0 / dt, u, v, b, out, part, g.nxl, g.ld, 0, np, 1, (const cplx*)tw, (const cplx*)wk, outE};
    if (phase == 1) {
        a.plo = 1;
        a.cnt = std::max(np - 2, 0);
    } else if (phase == 2) {
        a.cnt = std::min(np, 2);
        a.pstep = std::max(np - 1, 1);
    }
    const int lg = g.ny == (1 << 14) ? 14 : fps_log2(g.ny);
    if (fps_div_real(lg, outE)) {   // (per-row sums: 2 np partials)
        if (a.cnt <= 0) return 2 * np;
        int n = -1;
        switch (lg) {
        case 10: n = div_row<10>(a, st); break;
        case 11: n = div_row<11>(a, st); break;
        case 12: n = div_row<12>(a, st); break;
        case 13: n = div_row<13>(a, st); break;
        case 14: n = div_row<14>(a, st); break;   // (ny = 16384: 128 KiB, one workgroup of 1024 threads per CU)
        default: return -1;
        }
        return n < 0 ? -1 : 2 * np;
    }
    if (a.cnt <= 0) return np;
    int n = -1;
    switch (lg) {
    case 4: n = div_pair<4>(a, st); break;
    case 5: n = div_pair<5>(a, st); break;
    case 6: n = div_pair<6>(a, st); break;
    case 7: n = div_pair<7>(a, st); break;
    case 8: n = div_pair<8>(a, st); break;
    case 9: n = div_pair<9>(a, st); break;
    case 10: n = div_pair<10>(a, st); break;
    case 11: n = div_pair<11>(a, st); break;
    case 12: n = div_pair<12>(a, st); break;
    case 13: n = div_pair<13>(a, st); break;
    default: return -1;
    }
    return n < 0 ? -1 : np;
}

// whether the step's divergence can go into the forward transform (launch_fps_div): the row pairs for ny = 2^p <= 8192,
// the one-row transforms (r6) up to 16384
bool fps_fuse_ok(int ny, int outE) { return ny == (1 << 14) ? fps_div_real(14, outE) : fps_log2(ny) >= 0; }

void launch_fps_t1(const FpsArgs& a, const double* f, hipStream_t st) {
    hipLaunchKernelGGL(k_fps_t1, dim3((a.ny + 127) / 128, a.ngrp), dim3(64, FPS_G), 0, st, a, f);
}
void launch_fps_t2(const FpsArgs& a, double* f, hipStream_t st) {
    hipLaunchKernelGGL(k_fps_t2, dim3((a.ny + 127) / 128, a.ngrp), dim3(64, FPS_G), 0, st, a, f);
}
void launch_fps_t1b(const FpsArgs& a, const double* f, hipStream_t st) {
    hipLaunchKernelGGL(k_fps_t1b, dim3((a.ny + 127) / 128, a.ngrp), dim3(64, FPS_G), 0, st, a, f);
}
void launch_fps_mid(const FpsArgs& a, const double* f, hipStream_t st) {
    hipLaunchKernelGGL(k_fps_mid, dim3((a.ny + 127) / 128, a.ngrp), dim3(64), 0, st, a, f);
}
namespace {
__global__ void k_fps_oe_s0(const double* __restrict__ f, int row, int ld, int last, double* __restrict__ out) {
    if (threadIdx.x == 0) out[0] = last ? 2.0 * f[(size_t)row * ld] : 0.0;
}
}  // namespace
void launch_fps_oe_s0(const double* f, int row, int ld, int last, double* out, hipStream_t st) {
    hipLaunchKernelGGL(k_fps_oe_s0, dim3(1), dim3(64), 0, st, f, row, ld, last, out);
}
void launch_fps_t2b(const FpsArgs& a, double* f, hipStream_t st) {
    if (a.ghost) hipLaunchKernelGGL(k_fps_t2b<true>, dim3((a.ny + 127) / 128, a.ngrp), dim3(64, FPS_G), 0, st, a, f);
    else hipLaunchKernelGGL(k_fps_t2b<false>, dim3((a.ny + 127) / 128, a.ngrp), dim3(64, FPS_G), 0, st, a, f);
}
void launch_fps_t3(const FpsArgs& a, double* f, hipStream_t st) {
    hipLaunchKernelGGL(k_fps_t3, dim3((a.ny + 127) / 128, a.ngrp), dim3(64, FPS_G), 0, st, a, f);
}
// ------------------------------------------------ (r5) masked domains: the capacitance solve
// L_ext (the masked operator on the domain, zero-flux at its inner walls) differs from the bounding box's L_box
// only across the m interface faces f = (i in the domain, j outside): L_box = L_ext - D_w D^T, d_f = e_i - e_j,
// D_w's columns w_f d_f.  L_ext x = q is then x = L_box^+ (q - D_w y) with (I + D^T L_box^+ D_w) y = D^T L_box^+ q;
// the capacitance matrix C is singular along y0 = 1 (the domain's constant), C + 1 1^T / m is not (CapArgs)
namespace {

// y = Cinv (D^T z): one row per wave; every workgroup gathers the m interface differences into LDS first
__global__ __launch_bounds__(256) void k_cap_gemv(CapArgs a, const double* __restrict__ z) {
    extern __shared__ double gl[];
    const int M = a.m + a.border;
    for (int f = threadIdx.x; f < M; f += 256) gl[f] = f < a.m ? z[a.fi[f]] - z[a.fj[f]] : 0.0;
    __syncthreads();
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    const double* cr = a.cinv + (size_t)row * M;
    double acc = 0.0;
    for (int k = lane; k < M; k += 64) acc = fma(cr[k], gl[k], acc);
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) a.y[row] = acc;
}

// q -= D_w y at the interface cells (mode 0), or q = 0 at those outside the domain (mode 1: the Krylov planes'
// invariant -- 0 outside -- restored after the second box solve)
__global__ __launch_bounds__(256) void k_cap_scatter(CapArgs a, double* __restrict__ q, int mode) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= a.ncell) return;
    const int4 f4 = a.cf[c];
    const int fs[4] = {f4.x, f4.y, f4.z, f4.w};
    if (mode == 1) {
        if (fs[0] < 0) q[a.co[c]] = 0.0;   // (a cell outside holds only negative references)
        return;
    }
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int v = fs[k];
        if (v == 0) continue;
        const int f = (v > 0 ? v : -v) - 1;
        acc += (v > 0 ? 1.0 : -1.0) * a.w[f] * a.y[f];
    }
    q[a.co[c]] -= acc;
}

// x += z (+ lambda e1, bordered) on the domain's cells (set: x = ...)
__global__ __launch_bounds__(256) void k_cap_axpy(Geo g, CapArgs a, double* __restrict__ x, const double* __restrict__ z,
                                                  int set) {
    const int j = blockIdx.x * 64 + threadIdx.x, li = blockIdx.y * 4 + threadIdx.y;
    if (j >= g.ny || li >= g.nxl) return;
    const ptrdiff_t o = (ptrdiff_t)li * g.ld + j;
    if (!(g.fc[o] & FC_IN)) return;
    double d = z[o];
    if (a.border) d = fma(a.y[a.m], a.e1[o], d);
    x[o] = set ? d : x[o] + d;
}

// set-up: q = val on the domain's cells
__global__ __launch_bounds__(256) void k_cap_fill(Geo g, double* __restrict__ q, double val) {
    const int j = blockIdx.x * 64 + threadIdx.x, li = blockIdx.y * 4 + threadIdx.y;
    if (j >= g.ny || li >= g.nxl) return;
    const ptrdiff_t o = (ptrdiff_t)li * g.ld + j;
    if (g.fc[o] & FC_IN) q[o] = val;
}

// r = b - *shift on the domain's cells (the first capacitance solve's right-hand side, from x = 0)
__global__ __launch_bounds__(256) void k_cap_rhs(Geo g, const double* __restrict__ b, const double* __restrict__ shift,
                                                 double* __restrict__ r) {
    const int j = blockIdx.x * 64 + threadIdx.x, li = blockIdx.y * 4 + threadIdx.y;
    if (j >= g.ny || li >= g.nxl) return;
    const ptrdiff_t o = (ptrdiff_t)li * g.ld + j;
    if (!g.fc || (g.fc[o] & FC_IN)) r[o] = b[o] - (shift ? shift[0] : 0.0);   // (r6: rectangles too)
}

// set-up: the source w_f d_f of column f in the zeroed plane q (the previous column's cleared; f < 0: only that)
__global__ void k_cap_src(CapArgs a, double* __restrict__ q, int fprev, int f) {
    if (fprev >= 0) { q[a.fi[fprev]] = 0.0; q[a.fj[fprev]] = 0.0; }
    if (f >= 0) { q[a.fi[f]] = a.w[f]; q[a.fj[f]] = -a.w[f]; }
}

// set-up: column f of C + 1 1^T / m from z = L_box^+ (w_f d_f) (row-major in cmat); bordered, its row m = 1
// (y0^T y = 0), and column f = m from z = L_box^+ 1_domain: -D^T z, 0
__global__ __launch_bounds__(256) void k_cap_col(CapArgs a, const double* __restrict__ z, int f,
                                                 double* __restrict__ cmat) {
    const int r = blockIdx.x * 256 + threadIdx.x, M = a.m + a.border;
    if (r >= M) return;
    double val;
    if (r == a.m) val = f < a.m ? 1.0 : 0.0;
    else if (f == a.m) val = -(z[a.fi[r]] - z[a.fj[r]]);
    else val = (r == f ? 1.0 : 0.0) + (z[a.fi[r]] - z[a.fj[r]]) + 1.0 / a.m;
    cmat[(size_t)r * M + f] = val;
}

// set-up: Gauss-Jordan inversion in place without pivoting (C + 1 1^T / m is symmetric positive definite for
// uniform face weights, a diagonal similarity of one otherwise): pivot k's scaled row t and column u ...
// (r6) flagged -- the caller then keeps the preconditioned BiCGStab -- when a pivot is not finite, below
// GJ_TINY in magnitude (C's entries are O(1): the identity plus the dipoles' responses), or, without a border (spd),
// not positive; the bordered (E-outflow) system is indefinite, so there only the magnitude is tested
constexpr double GJ_TINY = 1e-12;
__global__ __launch_bounds__(256) void k_gj_prep(double* __restrict__ A, int m, int k, double* __restrict__ t,
                                                 double* __restrict__ u, double* __restrict__ flag, int spd) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= m) return;
    const double p = A[(size_t)k * m + k];
    if (c == 0 && !(isfinite(p) && fabs(p) >= GJ_TINY && (!spd || p > 0.0))) flag[0] = 1.0;
    t[c] = c == k ? 1.0 / p : A[(size_t)k * m + c] / p;
    u[c] = A[(size_t)c * m + k];
}
// ... then the rank-1 update of every other entry
__global__ __launch_bounds__(256) void k_gj_step(double* __restrict__ A, int m, int k, const double* __restrict__ t,
                                                 const double* __restrict__ u) {
    const int c = blockIdx.x * 64 + threadIdx.x, r = blockIdx.y * 4 + threadIdx.y;
    if (c >= m || r >= m) return;
    double& e = A[(size_t)r * m + c];
    if (r == k) e = t[c];
    else if (c == k) e = -u[r] * t[k];
    else e = fma(-u[r], t[c], e);
}

}  // namespace

hipError_t launch_cap_gemv(const CapArgs& a, const double* z, hipStream_t st) {
    const int M = a.m + a.border;
    // (the interface differences in dynamic LDS: cap_setup bounds M by CAP_LDS_MAX doubles -- 64 KiB, the launch
    // limit without a raised attribute -- and the launch is checked: a failed one must not leave y stale)
    if ((size_t)M > CAP_LDS_MAX) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_cap_gemv, dim3((M + 3) / 4), dim3(256), M * sizeof(double), st, a, z);
    return hipGetLastError();
}
void launch_cap_scatter(const CapArgs& a, double* q, int mode, hipStream_t st) {
    hipLaunchKernelGGL(k_cap_scatter, dim3((a.ncell + 255) / 256), dim3(256), 0, st, a, q, mode);
}
void launch_cap_axpy(const Geo& g, const CapArgs& a, double* x, const double* z, int set, hipStream_t st) {
    hipLaunchKernelGGL(k_cap_axpy, dim3((g.ny + 63) / 64, (g.nxl + 3) / 4), dim3(64, 4), 0, st, g, a, x, z, set);
}
void launch_cap_fill(const Geo& g, double* q, double val, hipStream_t st) {
    hipLaunchKernelGGL(k_cap_fill, dim3((g.ny + 63) / 64, (g.nxl + 3) / 4), dim3(64, 4), 0, st, g, q, val);
}
void launch_cap_rhs(const Geo& g, const double* b, const double* shift, double* r, hipStream_t st) {
    hipLaunchKernelGGL(k_cap_rhs, dim3((g.ny + 63) / 64, (g.nxl + 3) / 4), dim3(64, 4), 0, st, g, b, shift, r);
}
void launch_cap_src(const CapArgs& a, double* q, int fprev, int f, hipStream_t st) {
    hipLaunchKernelGGL(k_cap_src, dim3(1), dim3(1), 0, st, a, q, fprev, f);
}
void launch_cap_col(const CapArgs& a, const double* z, int f, double* cmat, hipStream_t st) {
    hipLaunchKernelGGL(k_cap_col, dim3((a.m + a.border + 255) / 256), dim3(256), 0, st, a, z, f, cmat);
}
void launch_gj_invert(double* A, int m, double* t, double* u, double* flag, int spd, hipStream_t st) {
    for (int k = 0; k < m; k++) {
        hipLaunchKernelGGL(k_gj_prep, dim3((m + 255) / 256), dim3(256), 0, st, A, m, k, t, u, flag, spd);
        hipLaunchKernelGGL(k_gj_step, dim3((m + 63) / 64, (m + 3) / 4), dim3(64, 4), 0, st, A, m, k, (const double*)t,
                           (const double*)u);
    }
}

void launch_fps_scan(const FpsArgs& a, bool backward, const FpsRank& R, double* rout, hipStream_t st) {
    if (FPS_SSEG > 1 && a.ngrp >= 2 * FPS_SSEG)
        hipLaunchKernelGGL(k_fps_scan_seg<FPS_SSEG>, dim3((a.ny + 63) / 64), dim3(64, FPS_SSEG), 0, st, a.ngrp, a.ld,
                           a.ny, backward ? a.gb : a.ga, backward ? a.gx : a.gc, R, rout, backward ? 1 : 0);
    else
        hipLaunchKernelGGL(k_fps_scan, dim3((a.ny + 63) / 64), dim3(64), 0, st, a.ngrp, a.ld, a.ny,
                           backward ? a.gb : a.ga, backward ? a.gx : a.gc, R, rout, backward ? 1 : 0);
}

}  // namespace nsg
