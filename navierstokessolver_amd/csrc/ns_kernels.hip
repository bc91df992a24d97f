// ns_kernels.hip -- gfx950 (MI355X / CDNA4) kernels of the incompressible-flow
// time step.  fp64 throughout (the reference is `double` everywhere).
//
// Layout (DESIGN.md "Data layout"): every field is a struct-of-arrays plane of
// (nxl + 2*HALO) rows x ld doubles, j (y) contiguous, i (x) outer -- the
// reference's compact-id order for a rectangle (Grid.cpp:149-162) -- so one
// x-slab's halo row is one contiguous ny*8-byte message.  Kernels see pointers
// at local row 0; global row gi = i0 + li.
//
// Kernels (bytes/cell are the algorithmic HBM traffic, fp64):
//   K1 rhs_velocity   64 B  ConstructRHS_V + fluxes + BCs  (FluidSolver.cpp:183-363,458-510)
//   K2 helm sweep     48 B  fused red-black SOR of (I - a L_V) on u and v (:547-548)
//   K3 divergence     24 B  ConstructRHS_phi / Div_V (:365-418) + sums for the null space (:550)
//   K4 poisson sweep  24 B  fused red-black SOR (or Jacobi) of L phi = rhs - mean (:551)
//   K5 correct        40 B  CorrectVelocities / GradP (:420-456,512-534) + min/max (:554-557)
// No MFMA: every kernel is a stencil far below the fp64 VALU ridge point; HBM bound.
#include "ns_internal.h"

namespace nsg {

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ double ldf(const double* f, int ld, int li, int j) {
    return f[(ptrdiff_t)li * ld + j];
}

// velocity ghost, EvaluateGhostStencil_V (FluidSolver.cpp:166-173):
//   walls / inlets: weights {-1} + constant[d];  NEUMANN: weights {1}
__device__ __forceinline__ double ghost_v(const Geo& g, double q, int side, int d) {
    return g.neu[side] ? q : (-q + (d == 0 ? g.c0[side] : g.c1[side]));
}

// minmode (FluidSolver.cpp:671-674)
__device__ __forceinline__ double minmode(double a, double b) {
    return (a * b > 0) ? a * fmin(1.0, fabs(b / a)) : 0.0;
}

// one SlopeLimiter component (FluidSolver.cpp:283-325) along a line:
// qc centre, qp/qm the +/- neighbours (valid if hp/hm), gp/gm the ghosts used otherwise
__device__ __forceinline__ double slope1(double qc, double qp, double qm, bool hp, bool hm, double hc,
                                         double hpn, double hmn, double gp, double gm) {
    double a = hp ? 2 * (qp - qc) / (hpn + hc) : (gp - qc) / hc;
    double b = hm ? 2 * (qc - qm) / (hmn + hc) : (qc - gm) / hc;
    return minmode(a, b);
}

__device__ __forceinline__ double fnn(double l, double r) {
    return 0.5 * (l * l + r * r - fabs(l + r) * (r - l));
}
__device__ __forceinline__ double fuv(double u1, double v1, double u2, double v2) {
    return 0.5 * (u1 * v1 + u2 * v2 - 0.5 * fabs(v1 + v2) * (u2 - u1) - 0.5 * fabs(u2 + u1) * (v2 - v1));
}

template <int NV>
__device__ __forceinline__ void block_reduce_sum(double (&x)[NV], double* out) {
    __shared__ double sh[16][NV];
#pragma unroll
    for (int k = 0; k < NV; k++)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x[k] += __shfl_xor(x[k], off, 64);
    const int tid = threadIdx.x + threadIdx.y * blockDim.x;
    const int lane = tid & 63, w = tid >> 6, nw = (blockDim.x * blockDim.y + 63) >> 6;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NV; k++) sh[w][k] = x[k];
    __syncthreads();
    if (tid == 0)
#pragma unroll
        for (int k = 0; k < NV; k++) {
            double s = 0.0;
            for (int q = 0; q < nw; q++) s += sh[q][k];
            out[k] = s;
        }
}

template <int NV>
__device__ __forceinline__ void block_reduce_min(double (&x)[NV], double* out) {
    __shared__ double sh[16][NV];
#pragma unroll
    for (int k = 0; k < NV; k++)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x[k] = fmin(x[k], __shfl_xor(x[k], off, 64));
    const int tid = threadIdx.x + threadIdx.y * blockDim.x;
    const int lane = tid & 63, w = tid >> 6, nw = (blockDim.x * blockDim.y + 63) >> 6;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NV; k++) sh[w][k] = x[k];
    __syncthreads();
    if (tid == 0)
#pragma unroll
        for (int k = 0; k < NV; k++) {
            double s = sh[0][k];
            for (int q = 1; q < nw; q++) s = fmin(s, sh[q][k]);
            out[k] = s;
        }
}

// ------------------------------------------------ grad phi (GradP, FluidSolver.cpp:420-456)
// Dirichlet-type faces only (phi ghost = phi, FluidSolver.cpp:87-88): boundary face value = phi_c.
__device__ __forceinline__ void grad_phi(const Geo& g, const Coef& c, const double* phi, int li, int j,
                                         double& gx, double& gy) {
    const int gi = g.i0 + li, ld = g.ld;
    const double pc = ldf(phi, ld, li, j);
    const double hx = c.hx[gi], hy = c.hy[j];
    double V0, V1, V2, V3, r;
    if (gi > 0) { r = hx / (c.hx[gi - 1] + hx); V0 = ldf(phi, ld, li - 1, j) * r + pc * (1 - r); }
    else V0 = 0.5 * (pc + pc);
    if (gi < g.nx - 1) { r = hx / (c.hx[gi + 1] + hx); V1 = ldf(phi, ld, li + 1, j) * r + pc * (1 - r); }
    else V1 = 0.5 * (pc + pc);
    if (j > 0) { r = hy / (c.hy[j - 1] + hy); V2 = ldf(phi, ld, li, j - 1) * r + pc * (1 - r); }
    else V2 = 0.5 * (pc + pc);
    if (j < g.ny - 1) { r = hy / (c.hy[j + 1] + hy); V3 = ldf(phi, ld, li, j + 1) * r + pc * (1 - r); }
    else V3 = 0.5 * (pc + pc);
    gx = (V1 - V0) / hx;
    gy = (V3 - V2) / hy;
}

// ---------------------------------------------------------------- K1
// ConstructRHS_V (FluidSolver.cpp:327-363): one thread per cell.  MUSCL needs
// the neighbour's slope, so the stencil reaches 2 cells along each axis.
// grad phi^{n-1} (divPhi) is recomputed from phi^{n-1} on the fly for boundary
// cells -- bit-identical to the stored divPhi of the reference (GradP of the
// same phi) and it saves a 16 B/cell state array.
__global__ __launch_bounds__(256) void k_rhs(Geo g, Coef c, double dt, double re, const double* __restrict__ u,
                                             const double* __restrict__ v, const double* __restrict__ phi,
                                             double* __restrict__ cu, double* __restrict__ cv,
                                             double* __restrict__ ru, double* __restrict__ rv,
                                             double* __restrict__ part) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int li = blockIdx.y * 4 + threadIdx.y;
    double acc[2] = {0.0, 0.0};
    if (j < g.ny && li < g.nxl) {
        const int gi = g.i0 + li, ld = g.ld, nx = g.nx, ny = g.ny;
        const bool hW = gi > 0, hWW = gi > 1, hE = gi < nx - 1, hEE = gi < nx - 2;
        const bool hS = j > 0, hSS = j > 1, hN = j < ny - 1, hNN = j < ny - 2;
        const double hx = c.hx[gi], hy = c.hy[j];
        const double hxW = hW ? c.hx[gi - 1] : 0.0, hxWW = hWW ? c.hx[gi - 2] : 0.0;
        const double hxE = hE ? c.hx[gi + 1] : 0.0, hxEE = hEE ? c.hx[gi + 2] : 0.0;
        const double hyS = hS ? c.hy[j - 1] : 0.0, hySS = hSS ? c.hy[j - 2] : 0.0;
        const double hyN = hN ? c.hy[j + 1] : 0.0, hyNN = hNN ? c.hy[j + 2] : 0.0;
        (void)hxWW; (void)hxEE; (void)hySS; (void)hyNN;

        const double uc = ldf(u, ld, li, j), vc = ldf(v, ld, li, j);
        const double uW = hW ? ldf(u, ld, li - 1, j) : 0.0, vW = hW ? ldf(v, ld, li - 1, j) : 0.0;
        const double uE = hE ? ldf(u, ld, li + 1, j) : 0.0, vE = hE ? ldf(v, ld, li + 1, j) : 0.0;
        const double uS = hS ? ldf(u, ld, li, j - 1) : 0.0, vS = hS ? ldf(v, ld, li, j - 1) : 0.0;
        const double uN = hN ? ldf(u, ld, li, j + 1) : 0.0, vN = hN ? ldf(v, ld, li, j + 1) : 0.0;
        const double uWW = hWW ? ldf(u, ld, li - 2, j) : 0.0, vWW = hWW ? ldf(v, ld, li - 2, j) : 0.0;
        const double uEE = hEE ? ldf(u, ld, li + 2, j) : 0.0, vEE = hEE ? ldf(v, ld, li + 2, j) : 0.0;
        const double uSS = hSS ? ldf(u, ld, li, j - 2) : 0.0, vSS = hSS ? ldf(v, ld, li, j - 2) : 0.0;
        const double uNN = hNN ? ldf(u, ld, li, j + 2) : 0.0, vNN = hNN ? ldf(v, ld, li, j + 2) : 0.0;

        // ---- DiffusiveFlux (FluidSolver.cpp:183-203) for u (d=0) and v (d=1)
        double ru_ = 0.0 + 1.0 * uc, rv_ = 0.0 + 1.0 * vc;    // VecSet + VecAXPY(1, u) (:335-338)
        ru_ += 0.5 * dt * cu[(ptrdiff_t)li * ld + j];           // VecAXPY(0.5dt, conv0) (:339-340)
        rv_ += 0.5 * dt * cv[(ptrdiff_t)li * ld + j];
        {
            double D0, D1, D2, D3;
            D0 = hW ? (1 / re) * (uc - uW) / (hx + hxW) : (0.5 / re / hx) * (uc - ghost_v(g, uc, 0, 0));
            D1 = hE ? (1 / re) * (uE - uc) / (hx + hxE) : -(0.5 / re / hx) * (uc - ghost_v(g, uc, 1, 0));
            D2 = hS ? (1 / re) * (uc - uS) / (hy + hyS) : (0.5 / re / hy) * (uc - ghost_v(g, uc, 2, 0));
            D3 = hN ? (1 / re) * (uN - uc) / (hy + hyN) : -(0.5 / re / hy) * (uc - ghost_v(g, uc, 3, 0));
            ru_ += dt * ((D1 - D0) / hx + (D3 - D2) / hy);
            D0 = hW ? (1 / re) * (vc - vW) / (hx + hxW) : (0.5 / re / hx) * (vc - ghost_v(g, vc, 0, 1));
            D1 = hE ? (1 / re) * (vE - vc) / (hx + hxE) : -(0.5 / re / hx) * (vc - ghost_v(g, vc, 1, 1));
            D2 = hS ? (1 / re) * (vc - vS) / (hy + hyS) : (0.5 / re / hy) * (vc - ghost_v(g, vc, 2, 1));
            D3 = hN ? (1 / re) * (vN - vc) / (hy + hyN) : -(0.5 / re / hy) * (vc - ghost_v(g, vc, 3, 1));
            rv_ += dt * ((D1 - D0) / hx + (D3 - D2) / hy);
        }

        // ---- ConvectiveFlux (FluidSolver.cpp:205-281)
        double C[8];
        {
            // x slopes of the cell and of its W/E neighbours (each needs its own ghosts at the wall)
            const double sxu = slope1(uc, uE, uW, hE, hW, hx, hxE, hxW, ghost_v(g, uc, 1, 0), ghost_v(g, uc, 0, 0));
            const double sxv = slope1(vc, vE, vW, hE, hW, hx, hxE, hxW, ghost_v(g, vc, 1, 1), ghost_v(g, vc, 0, 1));
            double u1, v1, u2, v2;
            u2 = uc - hx / 2 * sxu;
            v2 = vc - hx / 2 * sxv;
            if (hW) {
                const double su = slope1(uW, uc, uWW, true, hWW, hxW, hx, hxWW, 0.0, ghost_v(g, uW, 0, 0));
                const double sv = slope1(vW, vc, vWW, true, hWW, hxW, hx, hxWW, 0.0, ghost_v(g, vW, 0, 1));
                u1 = uW + hxW / 2 * su;
                v1 = vW + hxW / 2 * sv;
            } else {
                u1 = 0.5 * (uc + ghost_v(g, uc, 0, 0));
                v1 = 0.5 * (vc + ghost_v(g, vc, 0, 1));
            }
            C[0] = fnn(u1, u2);
            C[1] = fuv(u1, v1, u2, v2);
            u1 = uc + hx / 2 * sxu;
            v1 = vc + hx / 2 * sxv;
            if (hE) {
                const double su = slope1(uE, uEE, uc, hEE, true, hxE, hxEE, hx, ghost_v(g, uE, 1, 0), 0.0);
                const double sv = slope1(vE, vEE, vc, hEE, true, hxE, hxEE, hx, ghost_v(g, vE, 1, 1), 0.0);
                u2 = uE - hxE / 2 * su;
                v2 = vE - hxE / 2 * sv;
            } else {
                u2 = 0.5 * (uc + ghost_v(g, uc, 1, 0));
                v2 = 0.5 * (vc + ghost_v(g, vc, 1, 1));
            }
            C[2] = fnn(u1, u2);
            C[3] = fuv(u1, v1, u2, v2);

            const double syu = slope1(uc, uN, uS, hN, hS, hy, hyN, hyS, ghost_v(g, uc, 3, 0), ghost_v(g, uc, 2, 0));
            const double syv = slope1(vc, vN, vS, hN, hS, hy, hyN, hyS, ghost_v(g, vc, 3, 1), ghost_v(g, vc, 2, 1));
            u2 = uc - hy / 2 * syu;
            v2 = vc - hy / 2 * syv;
            if (hS) {
                const double su = slope1(uS, uc, uSS, true, hSS, hyS, hy, hySS, 0.0, ghost_v(g, uS, 2, 0));
                const double sv = slope1(vS, vc, vSS, true, hSS, hyS, hy, hySS, 0.0, ghost_v(g, vS, 2, 1));
                u1 = uS + hyS / 2 * su;
                v1 = vS + hyS / 2 * sv;
            } else {
                u1 = 0.5 * (uc + ghost_v(g, uc, 2, 0));
                v1 = 0.5 * (vc + ghost_v(g, vc, 2, 1));
            }
            C[5] = fnn(v1, v2);
            C[4] = fuv(u1, v1, u2, v2);
            u1 = uc + hy / 2 * syu;
            v1 = vc + hy / 2 * syv;
            if (hN) {
                const double su = slope1(uN, uNN, uc, hNN, true, hyN, hyNN, hy, ghost_v(g, uN, 3, 0), 0.0);
                const double sv = slope1(vN, vNN, vc, hNN, true, hyN, hyNN, hy, ghost_v(g, vN, 3, 1), 0.0);
                u2 = uN - hyN / 2 * su;
                v2 = vN - hyN / 2 * sv;
            } else {
                u2 = 0.5 * (uc + ghost_v(g, uc, 3, 0));
                v2 = 0.5 * (vc + ghost_v(g, vc, 3, 1));
            }
            C[7] = fnn(v1, v2);
            C[6] = fuv(u1, v1, u2, v2);
        }
        double val = (C[2] - C[0]) / hx + (C[6] - C[4]) / hy;   // (:352-355)
        cu[(ptrdiff_t)li * ld + j] = val;
        ru_ += val * (-1.5 * dt);
        val = (C[3] - C[1]) / hx + (C[7] - C[5]) / hy;          // (:356-359)
        cv[(ptrdiff_t)li * ld + j] = val;
        rv_ += val * (-1.5 * dt);

        // ---- ApplyBoundaryConditions (FluidSolver.cpp:458-510), boundary cells only
        if (!hW || !hE || !hS || !hN) {
            const int first = !hW ? 0 : (!hE ? 1 : (!hS ? 2 : 3));
            double gxc, gyc;
            grad_phi(g, c, phi, li, j, gxc, gyc);
            double D;
            if (first < 2) {  // vertical edge: D = d/dy of (dphi/dx) along the wall (:469-473)
                double gxn = 0.0, gxs = 0.0, dum;
                if (hN) grad_phi(g, c, phi, li, j + 1, gxn, dum);
                if (hS) grad_phi(g, c, phi, li, j - 1, gxs, dum);
                if (!hN) D = 2.0 * (gxc - gxs) / (hy + hyS);
                else if (!hS) D = 2.0 * (gxn - gxc) / (hy + hyN);
                else D = gxn / (hy + hyN) - gxs / (hy + hyS) - gxc * (1 / (hy + hyN) - 1 / (hy + hyS));
            } else {          // horizontal edge: D = d/dx of (dphi/dy) (:474-478)
                double gye = 0.0, gyw = 0.0, dum;
                if (hE) grad_phi(g, c, phi, li + 1, j, dum, gye);
                if (hW) grad_phi(g, c, phi, li - 1, j, dum, gyw);
                if (!hE) D = 2.0 * (gyc - gyw) / (hx + hxW);
                else if (!hW) D = 2.0 * (gye - gyc) / (hx + hxE);
                else D = gye / (hx + hxE) - gyw / (hx + hxW) - gyc * (1 / (hx + hxE) - 1 / (hx + hxW));
            }
            const bool bnd[4] = {!hW, !hE, !hS, !hN};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                if (!bnd[k]) continue;
                double w, W;
                if (g.neu[k]) {
                    if (k < 2) { w = dt * g.enx[k] * hx * D; W = dt * (0.5 / re / (hx * hx)) * w; rv_ += W; }
                    else       { w = dt * g.eny[k] * hy * D; W = dt * (0.5 / re / (hy * hy)) * w; ru_ += W; }
                } else if (k < 2) {
                    W = dt * (0.5 / re / (hx * hx)) * g.c0[k];
                    ru_ += W;
                    w = 2 * dt * (gyc + g.enx[k] * hx * D / 2);
                    W = dt * (0.5 / re / (hx * hx)) * (g.c1[k] + w);
                    rv_ += W;
                } else {
                    W = dt * (0.5 / re / (hy * hy)) * g.c1[k];
                    rv_ += W;
                    w = 2 * dt * (gxc + g.eny[k] * hy * D / 2);
                    W = dt * (0.5 / re / (hy * hy)) * (g.c0[k] + w);
                    ru_ += W;
                }
            }
        }
        ru[(ptrdiff_t)li * ld + j] = ru_;
        rv[(ptrdiff_t)li * ld + j] = rv_;
        acc[0] = ru_ * ru_;
        acc[1] = rv_ * rv_;
    }
    block_reduce_sum<2>(acc, part + 2 * (blockIdx.x + gridDim.x * blockIdx.y));
}

// ---------------------------------------------------------------- K3
// ConstructRHS_phi / Div_V (FluidSolver.cpp:365-418): rhs = div(u*)/dt, plus
// block partials of (sum rhs, sum rhs^2) for the null-space mean (:550) and ||b||.
__global__ __launch_bounds__(256) void k_div(Geo g, Coef c, double dt, const double* __restrict__ u,
                                             const double* __restrict__ v, double* __restrict__ rp,
                                             double* __restrict__ part) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int li = blockIdx.y * 4 + threadIdx.y;
    double acc[2] = {0.0, 0.0};
    if (j < g.ny && li < g.nxl) {
        const int gi = g.i0 + li, ld = g.ld;
        const double uc = ldf(u, ld, li, j), vc = ldf(v, ld, li, j);
        const double hx = c.hx[gi], hy = c.hy[j];
        double V0, V1, V2, V3, r;
        if (gi > 0) { r = hx / (c.hx[gi - 1] + hx); V0 = ldf(u, ld, li - 1, j) * r + uc * (1 - r); }
        else V0 = 0.5 * (uc + ghost_v(g, uc, 0, 0));
        if (gi < g.nx - 1) { r = hx / (c.hx[gi + 1] + hx); V1 = ldf(u, ld, li + 1, j) * r + uc * (1 - r); }
        else V1 = 0.5 * (uc + ghost_v(g, uc, 1, 0));
        if (j > 0) { r = hy / (c.hy[j - 1] + hy); V2 = ldf(v, ld, li, j - 1) * r + vc * (1 - r); }
        else V2 = 0.5 * (vc + ghost_v(g, vc, 2, 1));
        if (j < g.ny - 1) { r = hy / (c.hy[j + 1] + hy); V3 = ldf(v, ld, li, j + 1) * r + vc * (1 - r); }
        else V3 = 0.5 * (vc + ghost_v(g, vc, 3, 1));
        const double val = ((V1 - V0) / hx + (V3 - V2) / hy) / dt;
        rp[(ptrdiff_t)li * ld + j] = val;
        acc[0] = val;
        acc[1] = val * val;
    }
    block_reduce_sum<2>(acc, part + 2 * (blockIdx.x + gridDim.x * blockIdx.y));
}

// ---------------------------------------------------------------- K5
// CorrectVelocities (FluidSolver.cpp:512-534): u = u* - dt dphi/dx, v = v* - dt dphi/dy,
// in place; fused VecMin/VecMax partials (:554-557) as (umin, -umax, vmin, -vmax).
__global__ __launch_bounds__(256) void k_correct(Geo g, Coef c, double dt, double* __restrict__ u,
                                                 double* __restrict__ v, const double* __restrict__ phi,
                                                 double* __restrict__ part) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int li = blockIdx.y * 4 + threadIdx.y;
    double acc[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
    if (j < g.ny && li < g.nxl) {
        double gx, gy;
        grad_phi(g, c, phi, li, j, gx, gy);
        const ptrdiff_t o = (ptrdiff_t)li * g.ld + j;
        const double un = u[o] - dt * gx, vn = v[o] - dt * gy;
        u[o] = un;
        v[o] = vn;
        // NaN-propagating min so a blown-up step is visible in the stats
        acc[0] = un != un ? -INFINITY : un;
        acc[1] = un != un ? -INFINITY : -un;
        acc[2] = vn != vn ? -INFINITY : vn;
        acc[3] = vn != vn ? -INFINITY : -vn;
    }
    block_reduce_min<4>(acc, part + 4 * (blockIdx.x + gridDim.x * blockIdx.y));
}

// ------------------------------------------------------- K2 / K4: fused red-black sweep
// One workgroup owns a TI x TJ tile.  It stages the tile plus a 2-cell ring of
// the OLD iterate (and a 1-cell ring of the rhs) in LDS, updates the red cells
// of the tile + 1-cell ring (the ring reds are recomputed redundantly by the
// neighbouring tiles -- identical arithmetic, so the result is exactly a
// red-black SOR sweep), then the black cells of the tile, and writes the tile
// once: one HBM pass per full sweep (24 B/cell Poisson, 48 B/cell u+v).
// Out of place (ping-pong): an in-place sweep would let a late tile stage a
// ring that an early tile already overwrote -- chaotic relaxation, which is
// nondeterministic and diverges at omega ~ 2.
// With RES the true residual of the input iterate is accumulated from the
// staged old values at no extra traffic.
//
// OP 0: Poisson   L phi = b - shift,   (L q)_c = sum_nb p_nb (q_nb - q_c)      (FluidSolver.cpp:121-131)
// OP 1: Helmholtz (I - a L_V) q = b,   L_V adds -2/h^2 per Dirichlet face       (:130,140-141,153-157)
template <int OP>
struct Op {
    // returns A q at the cell given neighbours; dg receives the diagonal
    static __device__ __forceinline__ double apply(double qc, double qw, double qe, double qs, double qn, double cw,
                                                   double ce, double cs, double cn, double bxy, double a, double& dg) {
        if (OP == 0) {
            dg = -(cw + ce + cs + cn);
            return cw * qw + ce * qe + cs * qs + cn * qn + dg * qc;
        } else {
            dg = 1.0 + a * (cw + ce + cs + cn + bxy);
            return dg * qc - a * (cw * qw + ce * qe + cs * qs + cn * qn);
        }
    }
};

struct SweepArgs {
    const double* q[2];   // input iterate (read only: tiles never see each other's writes)
    double* qo[2];        // output iterate (ping-pong partner)
    const double* b[2];
    const double* shift;  // Poisson: device mean of rhs (null-space removal), else null
    double alpha, omega;
    Coef c;
    Geo g;
    double* part;
    int tiles_j, ntiles;
};

__device__ __forceinline__ int xcd_swizzle(int b, int n) {
    // 8 XCDs take blocks round-robin: give XCD k a contiguous range of tiles so
    // tiles that share halo rows/columns share an L2 (speed only, never correctness)
    if (n % 8 != 0) return b;
    return (b % 8) * (n / 8) + b / 8;
}

template <int TI, int TJ, int OP, int NF, bool RES>
__global__ __launch_bounds__(256) void k_rb_sweep(SweepArgs A) {
    constexpr int EI = TI + 4, EJ = TJ + 4;      // old iterate: tile + 2-ring
    constexpr int BI = TI + 2, BJ = TJ + 2;      // rhs: tile + 1-ring
    __shared__ double sq[NF][EI][EJ];
    __shared__ double sb[NF][BI][BJ];
    __shared__ double rcw[BI], rce[BI], rbx[BI], ccs[BJ], ccn[BJ], cby[BJ];
    const Geo& g = A.g;
    const int tid = threadIdx.x;
    const int t = xcd_swizzle(blockIdx.x, A.ntiles);
    const int ti = t / A.tiles_j, tj = t - ti * A.tiles_j;
    const int li0 = ti * TI, j0 = tj * TJ;
    const int ld = g.ld;
    const double shift = (OP == 0 && A.shift) ? A.shift[0] : 0.0;

    for (int q = tid; q < EI * EJ; q += 256) {
        const int r = q / EJ, cc = q - r * EJ;
        const int li = min(max(li0 - 2 + r, -HALO), g.nxl + HALO - 1);
        const int j = min(max(j0 - 2 + cc, 0), g.ny - 1);
#pragma unroll
        for (int f = 0; f < NF; f++) sq[f][r][cc] = ldf(A.q[f], ld, li, j);
    }
    for (int q = tid; q < BI * BJ; q += 256) {
        const int r = q / BJ, cc = q - r * BJ;
        const int li = min(max(li0 - 1 + r, -HALO), g.nxl + HALO - 1);
        const int j = min(max(j0 - 1 + cc, 0), g.ny - 1);
#pragma unroll
        for (int f = 0; f < NF; f++) sb[f][r][cc] = ldf(A.b[f], ld, li, j) - shift;
    }
    for (int q = tid; q < BI; q += 256) {
        const int gi = min(max(g.i0 + li0 - 1 + q, 0), g.nx - 1);
        rcw[q] = A.c.pw[gi]; rce[q] = A.c.pe[gi]; rbx[q] = A.c.bx[gi];
    }
    for (int q = tid; q < BJ; q += 256) {
        const int j = min(max(j0 - 1 + q, 0), g.ny - 1);
        ccs[q] = A.c.ps[j]; ccn[q] = A.c.pn[j]; cby[q] = A.c.by[j];
    }
    __syncthreads();

    double res[NF];
#pragma unroll
    for (int f = 0; f < NF; f++) res[f] = 0.0;
    if (RES) {
        for (int q = tid; q < TI * TJ; q += 256) {
            const int r = q / TJ, cc = q - r * TJ;
            const int li = li0 + r, j = j0 + cc;
            if (li >= g.nxl || j >= g.ny) continue;
            const int R = r + 2, Cc = cc + 2, rb = r + 1, cb = cc + 1;
#pragma unroll
            for (int f = 0; f < NF; f++) {
                double dg;
                const double aq = Op<OP>::apply(sq[f][R][Cc], sq[f][R - 1][Cc], sq[f][R + 1][Cc], sq[f][R][Cc - 1],
                                                sq[f][R][Cc + 1], rcw[rb], rce[rb], ccs[cb], ccn[cb],
                                                rbx[rb] + cby[cb], A.alpha, dg);
                const double rr = sb[f][rb][cb] - aq;
                res[f] += rr * rr;
            }
        }
    }

    // red cells ((gi + j) even) of the tile and its 1-ring
#pragma unroll
    for (int color = 0; color < 2; color++) {
        const int lo = color == 0 ? -1 : 0;
        const int hiI = color == 0 ? TI + 1 : TI, hiJ = color == 0 ? TJ + 1 : TJ;
        const int wI = hiI - lo, wJ = hiJ - lo;
        for (int q = tid; q < wI * wJ; q += 256) {
            const int r = lo + q / wJ, cc = lo + (q - (q / wJ) * wJ);
            const int li = li0 + r, j = j0 + cc, gi = g.i0 + li;
            if (((gi + j) & 1) != color) continue;
            if (gi < 0 || gi >= g.nx || j < 0 || j >= g.ny || li < -1 || li > g.nxl) continue;
            const int R = r + 2, Cc = cc + 2, rb = r + 1, cb = cc + 1;
#pragma unroll
            for (int f = 0; f < NF; f++) {
                double dg;
                const double qc = sq[f][R][Cc];
                const double aq = Op<OP>::apply(qc, sq[f][R - 1][Cc], sq[f][R + 1][Cc], sq[f][R][Cc - 1],
                                                sq[f][R][Cc + 1], rcw[rb], rce[rb], ccs[cb], ccn[cb],
                                                rbx[rb] + cby[cb], A.alpha, dg);
                sq[f][R][Cc] = qc + A.omega * (sb[f][rb][cb] - aq) / dg;
            }
        }
        __syncthreads();
    }

    for (int q = tid; q < TI * TJ; q += 256) {
        const int r = q / TJ, cc = q - r * TJ;
        const int li = li0 + r, j = j0 + cc;
        if (li >= g.nxl || j >= g.ny) continue;
#pragma unroll
        for (int f = 0; f < NF; f++) A.qo[f][(ptrdiff_t)li * ld + j] = sq[f][r + 2][cc + 2];
    }
    if (RES) block_reduce_sum<NF>(res, A.part + NF * blockIdx.x);
}

// weighted Jacobi: out = in + w (b - shift - L in)/diag, residual of `in` fused
template <int TI, int TJ>
__global__ __launch_bounds__(256) void k_jacobi(SweepArgs A, const double* __restrict__ in, double* __restrict__ out,
                                                int write) {
    constexpr int EI = TI + 2, EJ = TJ + 2;
    __shared__ double sq[EI][EJ];
    __shared__ double rcw[TI], rce[TI], ccs[TJ], ccn[TJ];
    const Geo& g = A.g;
    const int tid = threadIdx.x;
    const int t = xcd_swizzle(blockIdx.x, A.ntiles);
    const int ti = t / A.tiles_j, tj = t - ti * A.tiles_j;
    const int li0 = ti * TI, j0 = tj * TJ, ld = g.ld;
    const double shift = A.shift ? A.shift[0] : 0.0;
    for (int q = tid; q < EI * EJ; q += 256) {
        const int r = q / EJ, cc = q - r * EJ;
        const int li = min(max(li0 - 1 + r, -HALO), g.nxl + HALO - 1);
        const int j = min(max(j0 - 1 + cc, 0), g.ny - 1);
        sq[r][cc] = ldf(in, ld, li, j);
    }
    for (int q = tid; q < TI; q += 256) {
        const int gi = min(g.i0 + li0 + q, g.nx - 1);
        rcw[q] = A.c.pw[gi]; rce[q] = A.c.pe[gi];
    }
    for (int q = tid; q < TJ; q += 256) {
        const int j = min(j0 + q, g.ny - 1);
        ccs[q] = A.c.ps[j]; ccn[q] = A.c.pn[j];
    }
    __syncthreads();
    double res[1] = {0.0};
    for (int q = tid; q < TI * TJ; q += 256) {
        const int r = q / TJ, cc = q - r * TJ;
        const int li = li0 + r, j = j0 + cc;
        if (li >= g.nxl || j >= g.ny) continue;
        double dg;
        const double qc = sq[r + 1][cc + 1];
        const double aq = Op<0>::apply(qc, sq[r][cc + 1], sq[r + 2][cc + 1], sq[r + 1][cc], sq[r + 1][cc + 2],
                                       rcw[r], rce[r], ccs[cc], ccn[cc], 0.0, 0.0, dg);
        const double rr = (A.b[0][(ptrdiff_t)li * ld + j] - shift) - aq;
        res[0] += rr * rr;
        if (write) out[(ptrdiff_t)li * ld + j] = qc + A.omega * rr / dg;
    }
    if (A.part) block_reduce_sum<1>(res, A.part + blockIdx.x);
}

// ---------------------------------------------------------------- reductions
__global__ __launch_bounds__(1024) void k_reduce_sum(const double* __restrict__ p, int n, int nv,
                                                     double* __restrict__ out) {
    __shared__ double sh[1024];
    for (int v = 0; v < nv; v++) {
        double s = 0.0;
        for (int k = threadIdx.x; k < n; k += 1024) s += p[(size_t)k * nv + v];
        sh[threadIdx.x] = s;
        __syncthreads();
        for (int w = 512; w > 0; w >>= 1) {
            if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) out[v] = sh[0];
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void k_reduce_min(const double* __restrict__ p, int n, int nv,
                                                     double* __restrict__ out) {
    __shared__ double sh[1024];
    for (int v = 0; v < nv; v++) {
        double s = INFINITY;
        for (int k = threadIdx.x; k < n; k += 1024) s = fmin(s, p[(size_t)k * nv + v]);
        sh[threadIdx.x] = s;
        __syncthreads();
        for (int w = 512; w > 0; w >>= 1) {
            if ((int)threadIdx.x < w) sh[threadIdx.x] = fmin(sh[threadIdx.x], sh[threadIdx.x + w]);
            __syncthreads();
        }
        if (threadIdx.x == 0) out[v] = sh[0];
        __syncthreads();
    }
}

__global__ void k_finish_mean(const double* __restrict__ sums, double n, double* __restrict__ out) {
    const double s = sums[0], s2 = sums[1];
    out[0] = s / n;                 // MatNullSpaceRemove: subtract the plain mean (FluidSolver.cpp:550)
    out[1] = fmax(s2 - s * s / n, 0.0);  // ||rhs - mean||^2
}

// (sum f, sum f^2) block partials over the slab's own cells
__global__ __launch_bounds__(256) void k_sums(Geo g, const double* __restrict__ f, double* __restrict__ part) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int li = blockIdx.y * 4 + threadIdx.y;
    double acc[2] = {0.0, 0.0};
    if (j < g.ny && li < g.nxl) {
        const double x = ldf(f, g.ld, li, j);
        acc[0] = x;
        acc[1] = x * x;
    }
    block_reduce_sum<2>(acc, part + 2 * (blockIdx.x + gridDim.x * blockIdx.y));
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void k_fill_random(Geo g, double* phi, double* rp, uint64_t seed) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int li = blockIdx.y * 4 + threadIdx.y;
    if (j >= g.ny || li >= g.nxl) return;
    const uint64_t cell = (uint64_t)(g.i0 + li) * (uint64_t)g.ny + (uint64_t)j;
    const uint64_t a = splitmix64(seed ^ (2 * cell)), b = splitmix64(seed ^ (2 * cell + 1));
    const double s = 1.0 / 9007199254740992.0;  // 2^-53
    phi[(ptrdiff_t)li * g.ld + j] = 2.0 * ((a >> 11) * s) - 1.0;
    rp[(ptrdiff_t)li * g.ld + j] = 2.0 * ((b >> 11) * s) - 1.0;
}

// ---------------------------------------------------------------- launchers
static inline dim3 cell_grid(const Geo& g) { return dim3((g.ny + 63) / 64, (g.nxl + 3) / 4); }

int max_partials(const Geo& g) {
    const dim3 cg = cell_grid(g);
    int n = (int)(cg.x * cg.y) * 4;
    const int tiles = ((g.nxl + 7) / 8) * ((g.ny + 63) / 64) * 2;  // generous bound over sweep tilings
    return n > tiles ? n : tiles;
}

}  // namespace nsg

namespace nsg {

int launch_rhs(const Geo& g, const Coef& c, double dt, double re, const double* u, const double* v,
               const double* phi, double* cu, double* cv, double* ru, double* rv, double* part, hipStream_t st) {
    const dim3 cg = cell_grid(g);
    hipLaunchKernelGGL(k_rhs, cg, dim3(64, 4), 0, st, g, c, dt, re, u, v, phi, cu, cv, ru, rv, part);
    return (int)(cg.x * cg.y);
}

int launch_div(const Geo& g, const Coef& c, double dt, const double* u, const double* v, double* rp, double* part,
               hipStream_t st) {
    const dim3 cg = cell_grid(g);
    hipLaunchKernelGGL(k_div, cg, dim3(64, 4), 0, st, g, c, dt, u, v, rp, part);
    return (int)(cg.x * cg.y);
}

int launch_correct(const Geo& g, const Coef& c, double dt, double* u, double* v, const double* phi, double* part,
                   hipStream_t st) {
    const dim3 cg = cell_grid(g);
    hipLaunchKernelGGL(k_correct, cg, dim3(64, 4), 0, st, g, c, dt, u, v, phi, part);
    return (int)(cg.x * cg.y);
}

// Poisson tile: 32 x 128 (73 KB LDS, 2 workgroups / CU); Helmholtz u+v tile: 16 x 128.
constexpr int PTI = 32, PTJ = 128, HTI = 16, HTJ = 128, JTI = 16, JTJ = 128;

static SweepArgs make_args(const Geo& g, const Coef& c, int TI, int TJ) {
    SweepArgs a{};
    a.g = g;
    a.c = c;
    a.tiles_j = (g.ny + TJ - 1) / TJ;
    a.ntiles = a.tiles_j * ((g.nxl + TI - 1) / TI);
    return a;
}

int launch_pois_rbsor(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                      const double* rp, const double* shift, double* part, hipStream_t st) {
    SweepArgs a = make_args(g, c, PTI, PTJ);
    a.q[0] = phi; a.q[1] = nullptr;
    a.qo[0] = out; a.qo[1] = nullptr;
    a.b[0] = rp; a.b[1] = nullptr;
    a.shift = shift;
    a.omega = omega;
    a.alpha = 0.0;
    a.part = part;
    if (part) hipLaunchKernelGGL((k_rb_sweep<PTI, PTJ, 0, 1, true>), dim3(a.ntiles), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((k_rb_sweep<PTI, PTJ, 0, 1, false>), dim3(a.ntiles), dim3(256), 0, st, a);
    return a.ntiles;
}

int launch_helm_sweep(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                      double* uo, double* vo, const double* ru, const double* rv, double* part, hipStream_t st) {
    SweepArgs a = make_args(g, c, HTI, HTJ);
    a.q[0] = u; a.q[1] = v;
    a.qo[0] = uo; a.qo[1] = vo;
    a.b[0] = ru; a.b[1] = rv;
    a.shift = nullptr;
    a.omega = omega;
    a.alpha = alpha;
    a.part = part;
    if (part) hipLaunchKernelGGL((k_rb_sweep<HTI, HTJ, 1, 2, true>), dim3(a.ntiles), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((k_rb_sweep<HTI, HTJ, 1, 2, false>), dim3(a.ntiles), dim3(256), 0, st, a);
    return a.ntiles;
}

int launch_pois_jacobi(const Geo& g, const Coef& c, double omega, const double* in, double* out, const double* rp,
                       const double* shift, double* part, hipStream_t st) {
    SweepArgs a = make_args(g, c, JTI, JTJ);
    a.b[0] = rp;
    a.shift = shift;
    a.omega = omega;
    a.part = part;
    hipLaunchKernelGGL((k_jacobi<JTI, JTJ>), dim3(a.ntiles), dim3(256), 0, st, a, in, out, 1);
    return a.ntiles;
}

int launch_pois_residual(const Geo& g, const Coef& c, const double* phi, const double* rp, const double* shift,
                         double* part, hipStream_t st) {
    SweepArgs a = make_args(g, c, JTI, JTJ);
    a.b[0] = rp;
    a.shift = shift;
    a.omega = 0.0;
    a.part = part;
    hipLaunchKernelGGL((k_jacobi<JTI, JTJ>), dim3(a.ntiles), dim3(256), 0, st, a, phi, (double*)nullptr, 0);
    return a.ntiles;
}

void launch_reduce_sum(const double* p, int n, int nv, double* out, hipStream_t st) {
    hipLaunchKernelGGL(k_reduce_sum, dim3(1), dim3(1024), 0, st, p, n, nv, out);
}
void launch_reduce_min(const double* p, int n, int nv, double* out, hipStream_t st) {
    hipLaunchKernelGGL(k_reduce_min, dim3(1), dim3(1024), 0, st, p, n, nv, out);
}
void launch_finish_mean(const double* sums, double ncells, double* out, hipStream_t st) {
    hipLaunchKernelGGL(k_finish_mean, dim3(1), dim3(1), 0, st, sums, ncells, out);
}
int launch_sums(const Geo& g, const double* f, double* part, hipStream_t st) {
    const dim3 cg = cell_grid(g);
    hipLaunchKernelGGL(k_sums, cg, dim3(64, 4), 0, st, g, f, part);
    return (int)(cg.x * cg.y);
}
void launch_fill_random(const Geo& g, double* phi, double* rp, uint64_t seed, hipStream_t st) {
    hipLaunchKernelGGL(k_fill_random, cell_grid(g), dim3(64, 4), 0, st, g, phi, rp, seed);
}

}  // namespace nsg
