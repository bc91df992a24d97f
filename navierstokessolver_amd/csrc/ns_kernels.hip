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
#include <hip/hip_ext.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <mutex>

#include <algorithm>

namespace nsg {

// ---------------------------------------------------------------- helpers
// The j-neighbour of a lane's column pair: the value of lane l - 1 (lane_up1) or l + 1
// (lane_dn1), lane 0 / 63 keeping its own (__shfl_up / __shfl_down(x, 1, 64) semantics).  DPP
// wave_shr:1 / wave_shl:1 row moves (two v_mov_b32_dpp per double, VALU) instead of the
// ds_bpermute pair a shuffle compiles to: no LDS round trip on the sweeps' critical path
// (LANE_DPP=0: the shuffles, A/B).
#ifndef LANE_DPP
#define LANE_DPP 1
#endif
__device__ __forceinline__ double lane_up1(double x) {
#if LANE_DPP
    const int lo = __double2loint(x), hi = __double2hiint(x);
    return __hiloint2double(__builtin_amdgcn_update_dpp(hi, hi, 0x138, 0xf, 0xf, false),
                            __builtin_amdgcn_update_dpp(lo, lo, 0x138, 0xf, 0xf, false));
#else
    return __shfl_up(x, 1, 64);
#endif
}
__device__ __forceinline__ double lane_dn1(double x) {
#if LANE_DPP
    const int lo = __double2loint(x), hi = __double2hiint(x);
    return __hiloint2double(__builtin_amdgcn_update_dpp(hi, hi, 0x130, 0xf, 0xf, false),
                            __builtin_amdgcn_update_dpp(lo, lo, 0x130, 0xf, 0xf, false));
#else
    return __shfl_down(x, 1, 64);
#endif
}

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

// ------------------------------------------------ cell topology: rectangle or masked polygon
// The reference's existence tests (Grid::inDomain, Cell::edges[k] == -1) and ghost stencils
// (EvaluateGhostStencil_V/_P, FluidSolver.cpp:166-181) seen from cell (li, j):
//   in(di, dj)          the cell at that offset is in the domain;
//   gv(di, dj, k, q, d) the velocity ghost across face k of the cell at (di, dj), value q;
//   edge(k)             the edge on face k of this cell (ApplyBoundaryConditions).
// TopoRect folds to bound checks on the compile-time offsets and per-side constants (the
// rectangle kernels compile to what they were); TopoMask reads the int32 topology plane
// (FC_*) and the edge table of a non-rectangular domain.
struct TopoRect {
    const Geo& g;
    int gi, j;
    __device__ __forceinline__ TopoRect(const Geo& g_, int li, int j_) : g(g_), gi(g_.i0 + li), j(j_) {}
    __device__ __forceinline__ bool cell() const { return true; }
    __device__ __forceinline__ bool in(int di, int dj) const {
        if (dj == 0) return di < 0 ? gi + di >= 0 : gi + di < g.nx;
        if (di == 0) return dj < 0 ? j + dj >= 0 : j + dj < g.ny;
        return gi + di >= 0 && gi + di < g.nx && j + dj >= 0 && j + dj < g.ny;
    }
    __device__ __forceinline__ double gv(int, int, int k, double q, int d) const { return ghost_v(g, q, k, d); }
    __device__ __forceinline__ EdgeDev edge(int k) const { return EdgeDev{g.neu[k], g.enx[k], g.eny[k], g.c0[k], g.c1[k]}; }
};
// a cell at least two cells from every wall (the MUSCL stencil's reach): every neighbour exists,
// no ghost is evaluated -- K1's interior tiles (k_rhs_lds) skip the existence selects
struct TopoInner {
    __device__ __forceinline__ TopoInner(const Geo&, int, int) {}
    __device__ __forceinline__ bool cell() const { return true; }
    __device__ __forceinline__ bool in(int, int) const { return true; }
    __device__ __forceinline__ double gv(int, int, int, double q, int) const { return q; }
    __device__ __forceinline__ EdgeDev edge(int) const { return EdgeDev{}; }   // (never reached)
};
struct TopoMask {
    const Geo& g;
    int li, j, code;
    __device__ __forceinline__ int at(int di, int dj) const {
        const int jj = j + dj;
        return (jj >= 0 && jj < g.ny) ? g.fc[(ptrdiff_t)(li + di) * g.ld + jj] : 0;
    }
    __device__ __forceinline__ TopoMask(const Geo& g_, int li_, int j_) : g(g_), li(li_), j(j_), code(0) { code = at(0, 0); }
    __device__ __forceinline__ bool cell() const { return (code & FC_IN) != 0; }
    __device__ __forceinline__ bool in(int di, int dj) const {
        // (r5) a face neighbour from the cell's own code (its face is FC_INT exactly when the neighbour is in the
        // domain: ns_create checks Grid::inDomain against Cell::edges) -- no load of the neighbour's code
        if (di * di + dj * dj == 1) return fc_edge(code, di < 0 ? 0 : di > 0 ? 1 : dj < 0 ? 2 : 3) == FC_INT;
        return (at(di, dj) & FC_IN) != 0;
    }
    __device__ __forceinline__ double gv(int di, int dj, int k, double q, int d) const {
        const EdgeDev& E = g.et[fc_edge(di == 0 && dj == 0 ? code : at(di, dj), k)];
        return E.neu ? q : (-q + (d == 0 ? E.c0 : E.c1));
    }
    __device__ __forceinline__ EdgeDev edge(int k) const { return g.et[fc_edge(code, k)]; }
};

// ------------------------------------------------ grad phi (GradP, FluidSolver.cpp:420-456)
// phi ghost (EvaluateGhostStencil_P, :175-181; stencils :87-88, :98-101): walls / inlets
// phi_c (face value 0.5 (p + p)); a NEUMANN outflow face 2.5 phi_c - 2 phi_1 + 0.5 phi_2
// with phi_1, phi_2 the next two cells inward along the edge normal (slab rows / columns)
__device__ __forceinline__ double ghost_p_e(const Geo& g, const EdgeDev& E, const double* phi, int li, int j,
                                            double pc) {
    if (!E.neu) return pc;
    return 2.5 * pc - 2.0 * ldf(phi, g.ld, li - E.enx, j - E.eny) + 0.5 * ldf(phi, g.ld, li - 2 * E.enx, j - 2 * E.eny);
}
__device__ __forceinline__ double ghost_p(const Geo& g, const double* phi, int li, int j, int side, double pc) {
    if (!g.neu[side]) return pc;
    const int di = side == 0 ? 1 : (side == 1 ? -1 : 0), dj = side == 2 ? 1 : (side == 3 ? -1 : 0);
    return 2.5 * pc - 2.0 * ldf(phi, g.ld, li + di, j + dj) + 0.5 * ldf(phi, g.ld, li + 2 * di, j + 2 * dj);
}

template <class T = TopoRect>
__device__ __forceinline__ void grad_phi(const Geo& g, const Coef& c, const double* phi, int li, int j,
                                         double& gx, double& gy) {
    const T t(g, li, j);
    const int gi = g.i0 + li, ld = g.ld;
    const double pc = ldf(phi, ld, li, j);
    const double hx = c.hx[gi], hy = c.hy[j];
    double V0, V1, V2, V3, r;
    if (t.in(-1, 0)) { r = hx / (c.hx[gi - 1] + hx); V0 = ldf(phi, ld, li - 1, j) * r + pc * (1 - r); }
    else V0 = 0.5 * (pc + ghost_p_e(g, t.edge(0), phi, li, j, pc));
    if (t.in(1, 0)) { r = hx / (c.hx[gi + 1] + hx); V1 = ldf(phi, ld, li + 1, j) * r + pc * (1 - r); }
    else V1 = 0.5 * (pc + ghost_p_e(g, t.edge(1), phi, li, j, pc));
    if (t.in(0, -1)) { r = hy / (c.hy[j - 1] + hy); V2 = ldf(phi, ld, li, j - 1) * r + pc * (1 - r); }
    else V2 = 0.5 * (pc + ghost_p_e(g, t.edge(2), phi, li, j, pc));
    if (t.in(0, 1)) { r = hy / (c.hy[j + 1] + hy); V3 = ldf(phi, ld, li, j + 1) * r + pc * (1 - r); }
    else V3 = 0.5 * (pc + ghost_p_e(g, t.edge(3), phi, li, j, pc));
    gx = (V1 - V0) / hx;
    gy = (V3 - V2) / hy;
}

// ---------------------------------------------------------------- K1
// ConstructRHS_V (FluidSolver.cpp:327-363): one thread per cell.  MUSCL needs
// the neighbour's slope, so the stencil reaches 2 cells along each axis.
// grad phi^{n-1} (divPhi) is recomputed from phi^{n-1} on the fly for boundary
// cells -- the reference's stored divPhi is GradP of the same phi -- saving a
// 16 B/cell state array.  Divisions by spacings use reciprocal tables (1/h,
// 2/(h+h_nb)); minmode(a,b) = a*min(1,|b/a|) is evaluated as "the smaller of the two
// (same sign)", its exact value, without the division.

// minmode without the division: for a*b > 0, a*min(1, |b/a|) = (|b| < |a| ? b : a)
__device__ __forceinline__ double minmode_nd(double a, double b) {
    return (a * b > 0) ? (fabs(b) < fabs(a) ? b : a) : 0.0;
}

// SlopeLimiter component along one axis: forward difference a (2(qp-qc)/(h+hp) or
// (gp-qc)/h at a wall), backward difference b; rsp / rsm = 2/(h+h_nb), rh = 1/h
__device__ __forceinline__ double slope_r(double qc, double qp, double qm, bool hp, bool hm, double rh, double rsp,
                                         double rsm, double gp, double gm) {
    const double a = hp ? (qp - qc) * rsp : (gp - qc) * rh;
    const double b = hm ? (qc - qm) * rsm : (qc - gm) * rh;
    return minmode_nd(a, b);
}

// the ApplyBoundaryConditions terms of cell (li, j) added to its RHS (no-op off the walls)
template <class T = TopoRect>
__device__ __forceinline__ void rhs_bc(const Geo& g, const Coef& c, double dt, double re,
                                       const double* __restrict__ phi, int li, int j, double& ru_, double& rv_) {
    const T t(g, li, j);
    const int gi = g.i0 + li;
    const bool hW = t.in(-1, 0), hE = t.in(1, 0), hS = t.in(0, -1), hN = t.in(0, 1);
    if (!hW || !hE || !hS || !hN) {
        const double hx = c.hx[gi], hy = c.hy[j];
        const double hxW = hW ? c.hx[gi - 1] : 0.0, hxE = hE ? c.hx[gi + 1] : 0.0;
        const double hyS = hS ? c.hy[j - 1] : 0.0, hyN = hN ? c.hy[j + 1] : 0.0;
        const int first = !hW ? 0 : (!hE ? 1 : (!hS ? 2 : 3));
        double gxc, gyc;
        grad_phi<T>(g, c, phi, li, j, gxc, gyc);
        double D;
        if (first < 2) {  // vertical edge: D = d/dy of (dphi/dx) along the wall (:469-473)
            double gxn = 0.0, gxs = 0.0, dum;
            if (hN) grad_phi<T>(g, c, phi, li, j + 1, gxn, dum);
            if (hS) grad_phi<T>(g, c, phi, li, j - 1, gxs, dum);
            if (!hN) D = 2.0 * (gxc - gxs) / (hy + hyS);
            else if (!hS) D = 2.0 * (gxn - gxc) / (hy + hyN);
            else D = gxn / (hy + hyN) - gxs / (hy + hyS) - gxc * (1 / (hy + hyN) - 1 / (hy + hyS));
        } else {          // horizontal edge: D = d/dx of (dphi/dy) (:474-478)
            double gye = 0.0, gyw = 0.0, dum;
            if (hE) grad_phi<T>(g, c, phi, li + 1, j, dum, gye);
            if (hW) grad_phi<T>(g, c, phi, li - 1, j, dum, gyw);
            if (!hE) D = 2.0 * (gyc - gyw) / (hx + hxW);
            else if (!hW) D = 2.0 * (gye - gyc) / (hx + hxE);
            else D = gye / (hx + hxE) - gyw / (hx + hxW) - gyc * (1 / (hx + hxE) - 1 / (hx + hxW));
        }
        const bool bnd[4] = {!hW, !hE, !hS, !hN};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (!bnd[k]) continue;
            const EdgeDev E = t.edge(k);
            double w, W;
            if (E.neu) {
                if (k < 2) { w = dt * E.enx * hx * D; W = dt * (0.5 / re / (hx * hx)) * w; rv_ += W; }
                else       { w = dt * E.eny * hy * D; W = dt * (0.5 / re / (hy * hy)) * w; ru_ += W; }
            } else if (k < 2) {
                W = dt * (0.5 / re / (hx * hx)) * E.c0;
                ru_ += W;
                w = 2 * dt * (gyc + E.enx * hx * D / 2);
                W = dt * (0.5 / re / (hx * hx)) * (E.c1 + w);
                rv_ += W;
            } else {
                W = dt * (0.5 / re / (hy * hy)) * E.c1;
                rv_ += W;
                w = 2 * dt * (gxc + E.eny * hy * D / 2);
                W = dt * (0.5 / re / (hy * hy)) * (E.c0 + w);
                ru_ += W;
            }
        }
    }
}

// one cell of ConstructRHS_V (FluidSolver.cpp:327-363): u / v values at offsets (di, dj)
// come from U(di, dj) / V(di, dj) (global loads or an LDS tile); cu0 / cv0 are the previous
// step's convective derivatives; returns the new ones (cun, cvn) and the RHS (ru_, rv_).
// grad phi^{n-1} (divPhi) is recomputed from phi^{n-1} on the fly for boundary cells -- the
// reference's stored divPhi is GradP of the same phi -- saving a 16 B/cell state array.
// X(t, d) / Y(t, d): spacing table t (0: h, 1: 1/h, 2: 2/(h_{k-1} + h_k)) at row gi + d /
// column j + d (global tables or an LDS copy)
template <bool BC = true, class T = TopoRect, class FU, class FV, class FX, class FY>
__device__ __forceinline__ void rhs_cell(const Geo& g, const Coef& c, double dt, double re, FU&& U, FV&& V,
                                         FX&& X, FY&& Y, const double* __restrict__ phi, int li, int j,
                                         double cu0, double cv0, double& cun, double& cvn, double& ru_,
                                         double& rv_) {
    const T t(g, li, j);
    // existence (Grid::inDomain / Cell::edges, which agree on a consistent polygon); a masked
    // domain's second neighbour only counts behind an existing first one (SlopeLimiter of the
    // neighbour reads it only then)
    const bool hW = t.in(-1, 0), hWW = hW && t.in(-2, 0), hE = t.in(1, 0), hEE = hE && t.in(2, 0);
    const bool hS = t.in(0, -1), hSS = hS && t.in(0, -2), hN = t.in(0, 1), hNN = hN && t.in(0, 2);
    const double hx = X(0, 0), hy = Y(0, 0);
    const double hxW = hW ? X(0, -1) : 0.0, hxE = hE ? X(0, 1) : 0.0;
    const double hyS = hS ? Y(0, -1) : 0.0, hyN = hN ? Y(0, 1) : 0.0;
    // reciprocals: 1/h of the cell and its neighbours, 2/(h+h') of each face
    const double rx = X(1, 0), ry = Y(1, 0);
    const double rxW = hW ? X(1, -1) : 0.0, rxE = hE ? X(1, 1) : 0.0;
    const double ryS = hS ? Y(1, -1) : 0.0, ryN = hN ? Y(1, 1) : 0.0;
    const double sxW = X(2, 0), sxE = X(2, 1), sxWW = hW ? X(2, -1) : 0.0, sxEE = hE ? X(2, 2) : 0.0;
    const double syS = Y(2, 0), syN = Y(2, 1), sySS = hS ? Y(2, -1) : 0.0, syNN = hN ? Y(2, 2) : 0.0;

    const double uc = U(0, 0), vc = V(0, 0);
    const double uW = hW ? U(-1, 0) : 0.0, vW = hW ? V(-1, 0) : 0.0;
    const double uE = hE ? U(1, 0) : 0.0, vE = hE ? V(1, 0) : 0.0;
    const double uS = hS ? U(0, -1) : 0.0, vS = hS ? V(0, -1) : 0.0;
    const double uN = hN ? U(0, 1) : 0.0, vN = hN ? V(0, 1) : 0.0;
    const double uWW = hWW ? U(-2, 0) : 0.0, vWW = hWW ? V(-2, 0) : 0.0;
    const double uEE = hEE ? U(2, 0) : 0.0, vEE = hEE ? V(2, 0) : 0.0;
    const double uSS = hSS ? U(0, -2) : 0.0, vSS = hSS ? V(0, -2) : 0.0;
    const double uNN = hNN ? U(0, 2) : 0.0, vNN = hNN ? V(0, 2) : 0.0;

    // ---- DiffusiveFlux (FluidSolver.cpp:183-203) for u (d=0) and v (d=1); (1/re)/(h+h') = (0.5/re) * 2/(h+h')
    const double hre = 0.5 / re;
    ru_ = 0.0 + 1.0 * uc;                                   // VecSet + VecAXPY(1, u) (:335-338)
    rv_ = 0.0 + 1.0 * vc;
    ru_ += 0.5 * dt * cu0;                                  // VecAXPY(0.5dt, conv0) (:339-340)
    rv_ += 0.5 * dt * cv0;
    {
        double D0, D1, D2, D3;
        D0 = hW ? hre * (uc - uW) * sxW : hre * rx * (uc - t.gv(0, 0, 0, uc, 0));
        D1 = hE ? hre * (uE - uc) * sxE : -hre * rx * (uc - t.gv(0, 0, 1, uc, 0));
        D2 = hS ? hre * (uc - uS) * syS : hre * ry * (uc - t.gv(0, 0, 2, uc, 0));
        D3 = hN ? hre * (uN - uc) * syN : -hre * ry * (uc - t.gv(0, 0, 3, uc, 0));
        ru_ += dt * ((D1 - D0) * rx + (D3 - D2) * ry);
        D0 = hW ? hre * (vc - vW) * sxW : hre * rx * (vc - t.gv(0, 0, 0, vc, 1));
        D1 = hE ? hre * (vE - vc) * sxE : -hre * rx * (vc - t.gv(0, 0, 1, vc, 1));
        D2 = hS ? hre * (vc - vS) * syS : hre * ry * (vc - t.gv(0, 0, 2, vc, 1));
        D3 = hN ? hre * (vN - vc) * syN : -hre * ry * (vc - t.gv(0, 0, 3, vc, 1));
        rv_ += dt * ((D1 - D0) * rx + (D3 - D2) * ry);
    }

    // ---- ConvectiveFlux (FluidSolver.cpp:205-281)
    double C[8];
    {
        // x slopes of the cell and of its W/E neighbours (each needs its own ghosts at the wall)
        const double sxu = slope_r(uc, uE, uW, hE, hW, rx, sxE, sxW, t.gv(0, 0, 1, uc, 0), t.gv(0, 0, 0, uc, 0));
        const double sxv = slope_r(vc, vE, vW, hE, hW, rx, sxE, sxW, t.gv(0, 0, 1, vc, 1), t.gv(0, 0, 0, vc, 1));
        double u1, v1, u2, v2;
        u2 = uc - hx / 2 * sxu;
        v2 = vc - hx / 2 * sxv;
        if (hW) {
            const double su = slope_r(uW, uc, uWW, true, hWW, rxW, sxW, sxWW, 0.0, t.gv(-1, 0, 0, uW, 0));
            const double sv = slope_r(vW, vc, vWW, true, hWW, rxW, sxW, sxWW, 0.0, t.gv(-1, 0, 0, vW, 1));
            u1 = uW + hxW / 2 * su;
            v1 = vW + hxW / 2 * sv;
        } else {
            u1 = 0.5 * (uc + t.gv(0, 0, 0, uc, 0));
            v1 = 0.5 * (vc + t.gv(0, 0, 0, vc, 1));
        }
        C[0] = fnn(u1, u2);
        C[1] = fuv(u1, v1, u2, v2);
        u1 = uc + hx / 2 * sxu;
        v1 = vc + hx / 2 * sxv;
        if (hE) {
            const double su = slope_r(uE, uEE, uc, hEE, true, rxE, sxEE, sxE, t.gv(1, 0, 1, uE, 0), 0.0);
            const double sv = slope_r(vE, vEE, vc, hEE, true, rxE, sxEE, sxE, t.gv(1, 0, 1, vE, 1), 0.0);
            u2 = uE - hxE / 2 * su;
            v2 = vE - hxE / 2 * sv;
        } else {
            u2 = 0.5 * (uc + t.gv(0, 0, 1, uc, 0));
            v2 = 0.5 * (vc + t.gv(0, 0, 1, vc, 1));
        }
        C[2] = fnn(u1, u2);
        C[3] = fuv(u1, v1, u2, v2);

        const double syu = slope_r(uc, uN, uS, hN, hS, ry, syN, syS, t.gv(0, 0, 3, uc, 0), t.gv(0, 0, 2, uc, 0));
        const double syv = slope_r(vc, vN, vS, hN, hS, ry, syN, syS, t.gv(0, 0, 3, vc, 1), t.gv(0, 0, 2, vc, 1));
        u2 = uc - hy / 2 * syu;
        v2 = vc - hy / 2 * syv;
        if (hS) {
            const double su = slope_r(uS, uc, uSS, true, hSS, ryS, syS, sySS, 0.0, t.gv(0, -1, 2, uS, 0));
            const double sv = slope_r(vS, vc, vSS, true, hSS, ryS, syS, sySS, 0.0, t.gv(0, -1, 2, vS, 1));
            u1 = uS + hyS / 2 * su;
            v1 = vS + hyS / 2 * sv;
        } else {
            u1 = 0.5 * (uc + t.gv(0, 0, 2, uc, 0));
            v1 = 0.5 * (vc + t.gv(0, 0, 2, vc, 1));
        }
        C[5] = fnn(v1, v2);
        C[4] = fuv(u1, v1, u2, v2);
        u1 = uc + hy / 2 * syu;
        v1 = vc + hy / 2 * syv;
        if (hN) {
            const double su = slope_r(uN, uNN, uc, hNN, true, ryN, syNN, syN, t.gv(0, 1, 3, uN, 0), 0.0);
            const double sv = slope_r(vN, vNN, vc, hNN, true, ryN, syNN, syN, t.gv(0, 1, 3, vN, 1), 0.0);
            u2 = uN - hyN / 2 * su;
            v2 = vN - hyN / 2 * sv;
        } else {
            u2 = 0.5 * (uc + t.gv(0, 0, 3, uc, 0));
            v2 = 0.5 * (vc + t.gv(0, 0, 3, vc, 1));
        }
        C[7] = fnn(v1, v2);
        C[6] = fuv(u1, v1, u2, v2);
    }
    double val = (C[2] - C[0]) * rx + (C[6] - C[4]) * ry;   // (:352-355)
    cun = val;
    ru_ += val * (-1.5 * dt);
    val = (C[3] - C[1]) * rx + (C[7] - C[5]) * ry;          // (:356-359)
    cvn = val;
    rv_ += val * (-1.5 * dt);

    // ---- ApplyBoundaryConditions (FluidSolver.cpp:458-510), boundary cells only
    if (BC) rhs_bc<T>(g, c, dt, re, phi, li, j, ru_, rv_);
}

template <class T>
__global__ __launch_bounds__(256) void k_rhs(Geo g, Coef c, double dt, double re, const double* __restrict__ u,
                                             const double* __restrict__ v, const double* __restrict__ phi,
                                             double* __restrict__ cu, double* __restrict__ cv,
                                             double* __restrict__ ru, double* __restrict__ rv,
                                             double* __restrict__ part, int rows) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int lend = min((int)(blockIdx.y + 1) * 4 * rows, g.nxl);
    double acc[2] = {0.0, 0.0};
    for (int li = blockIdx.y * 4 * rows + threadIdx.y; li < lend && j < g.ny; li += 4) {
        const int ld = g.ld;
        const ptrdiff_t o = (ptrdiff_t)li * ld + j;
        if (!T(g, li, j).cell()) continue;   // outside a masked domain: stays 0
        auto U = [&](int di, int dj) { return ldf(u, ld, li + di, j + dj); };
        auto V = [&](int di, int dj) { return ldf(v, ld, li + di, j + dj); };
        const int gi = g.i0 + li;
        auto X = [&](int t, int d) { return (t == 0 ? c.hx : t == 1 ? c.rhx : c.rsx)[gi + d]; };
        auto Y = [&](int t, int d) { return (t == 0 ? c.hy : t == 1 ? c.rhy : c.rsy)[j + d]; };
        double cun, cvn, ru_, rv_;
        // (r5) a masked domain's cell whose MUSCL stencil lies in the domain (FC_DEEP): the interior arithmetic, no
        // topology or edge-table reads (the same values: every existence test is true, no ghost is used)
        if (g.fc && (g.fc[o] & FC_DEEP))
            rhs_cell<false, TopoInner>(g, c, dt, re, U, V, X, Y, phi, li, j, cu[o], cv[o], cun, cvn, ru_, rv_);
        else
            rhs_cell<true, T>(g, c, dt, re, U, V, X, Y, phi, li, j, cu[o], cv[o], cun, cvn, ru_, rv_);
        cu[o] = cun;
        cv[o] = cvn;
        ru[o] = ru_;
        rv[o] = rv_;
        acc[0] += ru_ * ru_;
        acc[1] += rv_ * rv_;
    }
    block_reduce_sum<2>(acc, part + 2 * (blockIdx.x + gridDim.x * blockIdx.y));
}

// K1 with everything staged in LDS: a 256-thread workgroup owns RT x 64 cells and loads u, v
// over them plus the MUSCL stencil's 2-cell ring, cu0 / cv0, and the tile's spacing tables
// in ONE round of coalesced loads (the global-load version fetches every u / v value ~13
// times through L1/L2 and reloads ~30 table entries per cell); the cell loop then reads
// LDS only.  Same per-cell arithmetic (rhs_cell).
// exchange / compute overlap (set_strip_phase): 0 all strips / tiles, 1 those whose read cone
// lies inside the slab, 2 the others
static int g_phase = 0;

// the row-block subset of phase g_phase for blocks of `rows` rows (n of them) reading `depth`
// rows beyond their own: launch block k is block k if k < *lo, else *hi0 + (k - *lo); returns
// how many blocks the launch covers
// The strip rows of a streaming launch for the exchange / compute overlap phase (set_strip_phase),
// for a kernel reading `depth` rows beyond its own (plan_rows below):
//   phase 0: the slab's rows in strips of L;
//   phase 1: rows [d, nxl - d) (their read cone inside the slab: launched while the ghost rows
//            travel), in strips of L;
//   phase 2: the two edge bands [0, d) and [nxl - d, nxl), one strip of d rows each -- a short
//            row pipeline after the exchange instead of a whole strip of L rows;
// d = depth rounded up to even.  Launch strip row k covers rows [ib, min(ib + L, rend)) with
// ib = rb0 + k L for k < slo, else rb1 + (k - slo) L; its partial slot is (pbase + k) nsj + sj.
// (r5) rend0: the end of the low runs (rend but in phase 2, where the low edge band [0, d) may be cut into
// several runs -- plan_rows' esplit)
struct RowPlan {
    int L, slo, nrun, rb0, rb1, rend, pbase, rend0;
    __device__ __forceinline__ void rows(int run, int& ib, int& ie) const {
        ib = run < slo ? rb0 + run * L : rb1 + (run - slo) * L;
        ie = min(ib + L, run < slo ? rend0 : rend);
    }
};

// host side of RowPlan: the strip rows of the current phase (g_phase) for `nxl` rows in strips of
// `L` (one resident round), reading `depth` rows beyond their own; returns the pass's strip-row
// count (partial slots / nsj, the same in every phase) and sets the plan's launch subset
// (r5) esplit > 0: phase 2 cuts each edge band into runs of esplit rows (K1's deep edge bands are ~22 rows:
// one run each left 132 waves walking them one row at a time after the exchange -- 31.7 us at 8192 P8)
static int plan_rows(int nxl, int L, int depth, RowPlan* p, int esplit = 0) {
    const int d = (depth + 1) & ~1, R = nxl - 2 * d;
    p->pbase = 0;
    p->rb1 = 0;
    p->L = L;
    if (g_phase == 0 || R < 2) {
        const int n = (nxl + L - 1) / L;
        p->nrun = g_phase == 1 ? 0 : n;   // (a slab too thin to split: all of it after the exchange)
        p->slo = n;
        p->rb0 = 0;
        p->rend = p->rend0 = nxl;
        return n;
    }
    const int n1 = (R + L - 1) / L;
    const int le = esplit > 0 && esplit < d ? esplit : d, m = (d + le - 1) / le;   // runs per edge band
    if (g_phase == 1) {
        p->nrun = p->slo = n1;
        p->rb0 = d;
        p->rend = p->rend0 = nxl - d;
    } else {
        p->L = le;
        p->nrun = 2 * m;
        p->slo = m;
        p->rb0 = 0;
        p->rend0 = d;
        p->rb1 = nxl - d;
        p->rend = nxl;
        p->pbase = n1;
    }
    return n1 + 2 * m;
}

static int phase_range(int nxl, int rows, int n, int depth, int* lo, int* hi0) {
    *lo = n; *hi0 = 0;
    if (!g_phase) return n;
    const int sa = std::min(n, (depth + rows - 1) / rows);        // first block clear of the low ghosts
    const int sb = std::max(sa, std::min(n, (nxl - depth) / rows));   // blocks [sa, sb) are interior
    if (g_phase == 1) { *lo = 0; *hi0 = sa; return sb - sa; }
    *lo = sa; *hi0 = sb;
    return sa + (n - sb);
}
__device__ __forceinline__ int phase_block(int k, int lo, int hi0) { return k < lo ? k : hi0 + (k - lo); }


constexpr int RT = 16;
// (r5) MASK: a masked domain's K1 (launch_rhs) -- cells outside the domain skipped (they stay 0), FC_DEEP cells (the
// MUSCL stencil inside the domain) with the interior arithmetic, the others with the polygon's topology and their
// wall terms inline; every domain cell's ||RHS||^2 in the partials (no k_rhs_bc pass).  The global-load k_rhs<TopoMask>
// fetched every u / v value ~13 times through L1 / L2 (105 us at the 1024^2 L-shape)
template <bool MASK>
__global__ __launch_bounds__(256) void k_rhs_lds(Geo g, Coef c, double dt, double re, const double* __restrict__ u,
                                                 const double* __restrict__ v, const double* __restrict__ phi,
                                                 double* __restrict__ cu, double* __restrict__ cv,
                                                 double* __restrict__ ru, double* __restrict__ rv,
                                                 double* __restrict__ part, int tlo, int thi0) {
    constexpr int EI = RT + 4, EJ = 64 + 4;
    __shared__ double su[EI][EJ], sv[EI][EJ];
    __shared__ double scu[RT][64], scv[RT][64];
    __shared__ double tx[3][RT + 4], ty[3][64 + 4];   // tables at rows gi-1 .. / columns j-1 ..
    const int tj = blockIdx.x, ti = phase_block(blockIdx.y, tlo, thi0);
    const int li0 = ti * RT, j0 = tj * 64, ld = g.ld;
    const int tid = threadIdx.x + 64 * threadIdx.y;
    // stage rows li0-2 .. li0+RT+1, columns j0-2 .. j0+65 (clamped into the field; a clamped
    // value is never used: the stencil reads past a wall only through its ghost formula)
    constexpr int NQ = (EI * EJ + 255) / 256, NC = (RT * 64) / 256;
    double pu[NQ], pv[NQ], pc[NC], pd[NC];
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const int q = tid + 256 * k;
        if (q < EI * EJ) {
            const int r = q / EJ, cc = q - r * EJ;
            const int li = min(max(li0 - 2 + r, -HALO), g.nxl + HALO - 1);
            const int j = min(max(j0 - 2 + cc, 0), g.ny - 1);
            pu[k] = ldf(u, ld, li, j);
            pv[k] = ldf(v, ld, li, j);
        }
    }
#pragma unroll
    for (int k = 0; k < NC; k++) {
        const int q = tid + 256 * k, r = q >> 6, cc = q & 63;
        const int li = min(li0 + r, g.nxl - 1), j = min(j0 + cc, g.ny - 1);
        pc[k] = ldf(cu, ld, li, j);
        pd[k] = ldf(cv, ld, li, j);
    }
    // spacing tables: entries q < NTX are rows (table q / (RT+4)), the rest columns
    constexpr int NTX = 3 * (RT + 4), NT = NTX + 3 * 68;
    auto table = [&](int q) {
        if (q < NTX) {
            const int t = q / (RT + 4), k = q - t * (RT + 4);
            const int gi = min(max(g.i0 + li0 - 1 + k, 0), g.nx);   // rsx has nx + 1 entries
            return t == 0 ? c.hx[min(gi, g.nx - 1)] : t == 1 ? c.rhx[min(gi, g.nx - 1)] : c.rsx[gi];
        }
        const int t = (q - NTX) / 68, k = q - NTX - t * 68;
        const int j = min(max(j0 - 1 + k, 0), g.ny);
        return t == 0 ? c.hy[min(j, g.ny - 1)] : t == 1 ? c.rhy[min(j, g.ny - 1)] : c.rsy[j];
    };
    const double tv0 = table(tid), tv1 = tid + 256 < NT ? table(tid + 256) : 0.0;
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const int q = tid + 256 * k;
        if (q < EI * EJ) {
            const int r = q / EJ, cc = q - r * EJ;
            su[r][cc] = pu[k];
            sv[r][cc] = pv[k];
        }
    }
#pragma unroll
    for (int k = 0; k < NC; k++) {
        const int q = tid + 256 * k;
        scu[q >> 6][q & 63] = pc[k];
        scv[q >> 6][q & 63] = pd[k];
    }
    auto put = [&](int q, double x) {
        if (q < NTX) tx[q / (RT + 4)][q % (RT + 4)] = x;
        else ty[(q - NTX) / 68][(q - NTX) % 68] = x;
    };
    put(tid, tv0);
    if (tid + 256 < NT) put(tid + 256, tv1);
    __syncthreads();
    double acc[2] = {0.0, 0.0};
    const int j = j0 + threadIdx.x;
    const int lend = min(li0 + RT, g.nxl);
    // tiles whose every cell is >= 2 cells from the walls (96 % at 4096^2) run rhs_cell with
    // every neighbour known to exist: no existence selects, no ghosts (block-uniform branch)
    const bool inner = g.i0 + li0 >= 2 && g.i0 + li0 + RT + 2 <= g.nx && j0 >= 2 && j0 + 64 + 2 <= g.ny;
    auto rows = [&](auto topo) {
        using T = decltype(topo);
        // one wave = one row (blockDim.x == 64): the row index is wave-uniform
        for (int li = __builtin_amdgcn_readfirstlane(li0 + (int)threadIdx.y); li < lend && j < g.ny; li += 4) {
            const int R = li - li0 + 2, C = threadIdx.x + 2;
            const ptrdiff_t o = (ptrdiff_t)li * ld + j;
            auto U = [&](int di, int dj) { return su[R + di][C + dj]; };
            auto V = [&](int di, int dj) { return sv[R + di][C + dj]; };
            auto X = [&](int t, int d) { return tx[t][R - 1 + d]; };
            auto Y = [&](int t, int d) { return ty[t][C - 1 + d]; };
            double cun, cvn, ru_, rv_;
            if (MASK) {
                // (the other domain cells: k_rhs_cells' list -- in this loop their topology path, taken by every
                // wave holding one, cost the whole launch 3.3x: 93 vs 28 us at 1024^2)
                if (!(g.fc[o] & FC_DEEP)) continue;
                rhs_cell<false, TopoInner>(g, c, dt, re, U, V, X, Y, phi, li, j, scu[R - 2][C - 2], scv[R - 2][C - 2],
                                           cun, cvn, ru_, rv_);
            } else {
                rhs_cell<false, T>(g, c, dt, re, U, V, X, Y, phi, li, j, scu[R - 2][C - 2], scv[R - 2][C - 2], cun,
                                   cvn, ru_, rv_);
            }
            cu[o] = cun;
            cv[o] = cvn;
            ru[o] = ru_;
            rv[o] = rv_;
            const int gi = g.i0 + li;
            if (MASK || (gi > 0 && gi < g.nx - 1 && j > 0 && j < g.ny - 1)) {   // wall cells: k_rhs_bc
                acc[0] += ru_ * ru_;
                acc[1] += rv_ * rv_;
            }
        }
    };
    if (MASK) rows(TopoInner(g, 0, 0));   // (the topology per cell above)
    else if (inner) rows(TopoInner(g, 0, 0));
    else rows(TopoRect(g, 0, 0));
    block_reduce_sum<2>(acc, part + 2 * (blockIdx.x + gridDim.x * ti));
}

// (r5) K1 of a masked domain's listed cells (Geo::ecell: the domain cells within 2 of its boundary), one thread
// each, with the polygon's topology and wall terms (k_rhs<TopoMask>'s cell)
__global__ __launch_bounds__(256) void k_rhs_cells(Geo g, Coef c, double dt, double re, const double* __restrict__ u,
                                                   const double* __restrict__ v, const double* __restrict__ phi,
                                                   double* __restrict__ cu, double* __restrict__ cv,
                                                   double* __restrict__ ru, double* __restrict__ rv,
                                                   double* __restrict__ part) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    double acc[2] = {0.0, 0.0};
    if (k < g.necell) {
        const int ld = g.ld, o = g.ecell[k], li = o / ld, j = o - li * ld;
        auto U = [&](int di, int dj) { return ldf(u, ld, li + di, j + dj); };
        auto V = [&](int di, int dj) { return ldf(v, ld, li + di, j + dj); };
        const int gi = g.i0 + li;
        auto X = [&](int t, int d) { return (t == 0 ? c.hx : t == 1 ? c.rhx : c.rsx)[gi + d]; };
        auto Y = [&](int t, int d) { return (t == 0 ? c.hy : t == 1 ? c.rhy : c.rsy)[j + d]; };
        double cun, cvn, ru_, rv_;
        rhs_cell<true, TopoMask>(g, c, dt, re, U, V, X, Y, phi, li, j, cu[o], cv[o], cun, cvn, ru_, rv_);
        cu[o] = cun;
        cv[o] = cvn;
        ru[o] = ru_;
        rv[o] = rv_;
        acc[0] = ru_ * ru_;
        acc[1] = rv_ * rv_;
    }
    block_reduce_sum<2>(acc, part + 2 * blockIdx.x);
}

// the wall cells' ApplyBoundaryConditions terms (rhs_bc) on top of k_rhs_lds's values -- the
// same additions in the same order as the fused k_rhs -- plus their ||RHS||^2 partials.  Out
// of the main kernel because the wall branch (three grad phi evaluations) would cost it ~40
// VGPRs (197 -> 153) for 0.05 % of the cells.  Thread k: the slab's column j = 0 / ny-1
// cells (2 nxl), then the W / E wall rows if this slab holds them (ny - 2 each).
__global__ __launch_bounds__(256) void k_rhs_bc(Geo g, Coef c, double dt, double re, const double* __restrict__ phi,
                                                double* __restrict__ ru, double* __restrict__ rv,
                                                double* __restrict__ part) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    const bool wrow = g.i0 == 0, erow = g.i0 + g.nxl == g.nx;
    int li = -1, j = 0;
    if (k < 2 * g.nxl) { li = k >> 1; j = (k & 1) ? g.ny - 1 : 0; }
    else {
        int q = k - 2 * g.nxl;
        if (wrow) { if (q < g.ny - 2) { li = 0; j = q + 1; } q -= g.ny - 2; }
        if (li < 0 && erow && q >= 0 && q < g.ny - 2) { li = g.nxl - 1; j = q + 1; }
    }
    double acc[2] = {0.0, 0.0};
    if (li >= 0) {
        const ptrdiff_t o = (ptrdiff_t)li * g.ld + j;
        double ru_ = ru[o], rv_ = rv[o];
        rhs_bc(g, c, dt, re, phi, li, j, ru_, rv_);
        ru[o] = ru_;
        rv[o] = rv_;
        acc[0] = ru_ * ru_;
        acc[1] = rv_ * rv_;
    }
    block_reduce_sum<2>(acc, part + 2 * blockIdx.x);
}

// ---------------------------------------------------------------- K3
// ConstructRHS_phi / Div_V (FluidSolver.cpp:365-418): rhs = div(u*)/dt, plus
// block partials of (sum rhs, sum rhs^2) for the null-space mean (:550) and ||b||.
template <class T>
__global__ __launch_bounds__(256) void k_div(Geo g, Coef c, double dt, const double* __restrict__ u,
                                             const double* __restrict__ v, double* __restrict__ rp,
                                             double* __restrict__ part, int rows) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int lend = min((int)(blockIdx.y + 1) * 4 * rows, g.nxl);
    double acc[2] = {0.0, 0.0};
    for (int li = blockIdx.y * 4 * rows + threadIdx.y; li < lend && j < g.ny; li += 4) {
        const T t(g, li, j);
        if (!t.cell()) continue;
        const int gi = g.i0 + li, ld = g.ld;
        const double uc = ldf(u, ld, li, j), vc = ldf(v, ld, li, j);
        const double hx = c.hx[gi], hy = c.hy[j];
        double V0, V1, V2, V3, r;
        if (t.in(-1, 0)) { r = hx / (c.hx[gi - 1] + hx); V0 = ldf(u, ld, li - 1, j) * r + uc * (1 - r); }
        else V0 = 0.5 * (uc + t.gv(0, 0, 0, uc, 0));
        if (t.in(1, 0)) { r = hx / (c.hx[gi + 1] + hx); V1 = ldf(u, ld, li + 1, j) * r + uc * (1 - r); }
        else V1 = 0.5 * (uc + t.gv(0, 0, 1, uc, 0));
        if (t.in(0, -1)) { r = hy / (c.hy[j - 1] + hy); V2 = ldf(v, ld, li, j - 1) * r + vc * (1 - r); }
        else V2 = 0.5 * (vc + t.gv(0, 0, 2, vc, 1));
        if (t.in(0, 1)) { r = hy / (c.hy[j + 1] + hy); V3 = ldf(v, ld, li, j + 1) * r + vc * (1 - r); }
        else V3 = 0.5 * (vc + t.gv(0, 0, 3, vc, 1));
        const double val = ((V1 - V0) / hx + (V3 - V2) / hy) / dt;
        rp[(ptrdiff_t)li * ld + j] = val;
        acc[0] += val;
        acc[1] += val * val;
    }
    block_reduce_sum<2>(acc, part + 2 * (blockIdx.x + gridDim.x * blockIdx.y));
}

// ---------------------------------------------------------------- K5
// CorrectVelocities (FluidSolver.cpp:512-534): u = u* - dt dphi/dx, v = v* - dt dphi/dy,
// out of place; fused VecMin/VecMax partials (:554-557) as (umin, -umax, vmin, -vmax).
template <class T>
__global__ __launch_bounds__(256) void k_correct(Geo g, Coef c, double dt, const double* __restrict__ us,
                                                 const double* __restrict__ vs, double* __restrict__ u,
                                                 double* __restrict__ v, const double* __restrict__ phi,
                                                 double* __restrict__ part, int rows) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int lend = min((int)(blockIdx.y + 1) * 4 * rows, g.nxl);
    double acc[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
    for (int li = blockIdx.y * 4 * rows + threadIdx.y; li < lend && j < g.ny; li += 4) {
        if (!T(g, li, j).cell()) continue;
        double gx, gy;
        grad_phi<T>(g, c, phi, li, j, gx, gy);
        const ptrdiff_t o = (ptrdiff_t)li * g.ld + j;
        const double un = us[o] - dt * gx, vn = vs[o] - dt * gy;
        u[o] = un;
        v[o] = vn;
        // NaN-propagating min so a blown-up step is visible in the stats
        acc[0] = fmin(acc[0], un != un ? -INFINITY : un);
        acc[1] = fmin(acc[1], un != un ? -INFINITY : -un);
        acc[2] = fmin(acc[2], vn != vn ? -INFINITY : vn);
        acc[3] = fmin(acc[3], vn != vn ? -INFINITY : -vn);
    }
    block_reduce_min<4>(acc, part + 4 * (blockIdx.x + gridDim.x * blockIdx.y));
}

// (r6) K3 / K5 of a masked domain's listed cells (Geo::ecell: the domain cells that are not FC_DEEP), one thread
// each, k_div<TopoMask> / k_correct<TopoMask>'s arithmetic; the FC_DEEP cells are k_cell_s's
__global__ __launch_bounds__(256) void k_div_cells(Geo g, Coef c, double dt, const double* __restrict__ u,
                                                   const double* __restrict__ v, double* __restrict__ rp,
                                                   double* __restrict__ part) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    double acc[2] = {0.0, 0.0};
    if (k < g.necell) {
        const int ld = g.ld, o = g.ecell[k], li = o / ld, j = o - li * ld;
        const TopoMask t(g, li, j);
        const int gi = g.i0 + li;
        const double uc = ldf(u, ld, li, j), vc = ldf(v, ld, li, j);
        const double hx = c.hx[gi], hy = c.hy[j];
        double V0, V1, V2, V3, r;
        if (t.in(-1, 0)) { r = hx / (c.hx[gi - 1] + hx); V0 = ldf(u, ld, li - 1, j) * r + uc * (1 - r); }
        else V0 = 0.5 * (uc + t.gv(0, 0, 0, uc, 0));
        if (t.in(1, 0)) { r = hx / (c.hx[gi + 1] + hx); V1 = ldf(u, ld, li + 1, j) * r + uc * (1 - r); }
        else V1 = 0.5 * (uc + t.gv(0, 0, 1, uc, 0));
        if (t.in(0, -1)) { r = hy / (c.hy[j - 1] + hy); V2 = ldf(v, ld, li, j - 1) * r + vc * (1 - r); }
        else V2 = 0.5 * (vc + t.gv(0, 0, 2, vc, 1));
        if (t.in(0, 1)) { r = hy / (c.hy[j + 1] + hy); V3 = ldf(v, ld, li, j + 1) * r + vc * (1 - r); }
        else V3 = 0.5 * (vc + t.gv(0, 0, 3, vc, 1));
        const double val = ((V1 - V0) / hx + (V3 - V2) / hy) / dt;
        rp[o] = val;
        acc[0] = val;
        acc[1] = val * val;
    }
    block_reduce_sum<2>(acc, part + 2 * blockIdx.x);
}
__global__ __launch_bounds__(256) void k_correct_cells(Geo g, Coef c, double dt, const double* __restrict__ us,
                                                       const double* __restrict__ vs, double* __restrict__ u,
                                                       double* __restrict__ v, const double* __restrict__ phi,
                                                       double* __restrict__ part) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    double acc[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
    if (k < g.necell) {
        const int ld = g.ld, o = g.ecell[k], li = o / ld, j = o - li * ld;
        double gx, gy;
        grad_phi<TopoMask>(g, c, phi, li, j, gx, gy);
        const double un = us[o] - dt * gx, vn = vs[o] - dt * gy;
        u[o] = un;
        v[o] = vn;
        acc[0] = un != un ? -INFINITY : un;
        acc[1] = un != un ? -INFINITY : -un;
        acc[2] = vn != vn ? -INFINITY : vn;
        acc[3] = vn != vn ? -INFINITY : -vn;
    }
    block_reduce_min<4>(acc, part + 4 * blockIdx.x);
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

// ------------------------------------------------ K2 / K4: register-streaming sweep
// One wave owns a strip of rows [ib, ib+L) x 128 loaded columns [jb-2, jb+126)
// (2 per lane, double2 = 16 B/lane loads: 1 KiB per wave-instruction) and walks
// it along i with a 3-row window in registers.  Strips overlap by 2 columns on
// each side: lane 0's and lane 63's cells only feed their neighbours, so every
// j-neighbour a written cell needs is in an adjacent lane (cross-lane shuffle) --
// no halo loads, no halo registers -- and each strip writes 124 columns.
// Red-black: while row r arrives, row r-1 gets its red update (old neighbours)
// and row r-2 its black update (red neighbours) and is stored: one read of phi
// and b and one write of phi per cell and sweep (24 B/cell).  Jacobi: row r-1 is
// relaxed from old rows r-2..r and stored.  Rows are prefetched D ahead.
// Out of place (in -> out): strips never observe each other's writes.
constexpr int SW = 124;   // written columns per strip
constexpr int SD = 4;     // rows in flight per wave

struct StreamArgs {
    const double* in;
    double* out;
    const double* b;
    const double* shift;              // Poisson: device mean of b (null-space removal), else null
    const double *cw, *ce, *bx;       // per global row: weights toward i-1 / i+1, Helmholtz wall term
    const double *cs, *cn, *by;       // per column
    double alpha, omega;
    int nx, ny, i0, nxl, ld;
    int nsj, nsi, L;                  // strips along j, along i, rows per strip
    double* part;                     // one residual partial per strip
    // fused restriction (k_sweep2 FUSE_R): spacings, coarse rhs / phi and their stride;
    // fused prolongation (FUSE_P): the coarse correction ec, its global size and first row
    const double *hx, *hy;
    double *bc, *pc;
    int ldc;
    const double* ec;
    int ncx, ncy, ci0;
    int dsx;                          // FUSE_P: x sides closed by a value-0 ghost (Geo::dsx)
    int nt;                           // non-temporal output stores
    int ntl;                          // non-temporal iterate loads
    // strip subset of this launch (k_sweep2; exchange / compute overlap): launch strip-row k
    // is strip row k if k < slo, else shi0 + (k - slo); nrun strip rows in all
    // strip rows of this launch (plan_strips2; k_sweep2): launch strip row k covers rows
    // [ib, min(ib + L, rend)) with ib = rb0 + k L for k < slo, else rb1 + (k - slo) L; its
    // residual partials go to slot (pbase + k) nsj + j; nrun strip rows in all
    int slo, nrun, rb0, rb1, rend, pbase;
    // (r5) the launch rows whose residual is summed (a deep-ghost launch: its slab's own rows; Geo::sr0 / sr1)
    int sr0, sr1;
    // k_sweep2<..., FUSE_UV>: two fields in one launch (the multi-rank Helmholtz pair pass, u and
    // v): waves [nstr, 2 nstr) take in2 / out2 / b2 and write their partials to part2
    const double* in2;
    double* out2;
    const double* b2;
    double* part2;
    // GIN (k_sweep2<FUSE_R>, r4): the input iterate is the Poisson guess gc0 in + gc1 gh1 + gc2 gh2
    // + gc3 gh3 (the phi extrapolation, extrap_comb), formed per row as it enters the pipeline
    const double *gh1, *gh2, *gh3;
    double gc0, gc1, gc2, gc3;
};

// diagonal of the operator at a cell from its row / column coefficient sums
template <int OP>
__device__ __forceinline__ double diag(double rowd, double cold, double alpha) {
    return OP == 0 ? -(rowd + cold) : 1.0 + alpha * (rowd + cold);
}

// relaxed value q + w (b - A q), w = omega / diag; `res` = b - A q of the input values
// (OP 0: Poisson L, OP 1: Helmholtz I - a L_V)
template <int OP>
__device__ __forceinline__ double relax(double q, double xm, double xp, double ym, double yp, double b, double cw,
                                        double ce, double cs, double cn, double dg, double w, double alpha,
                                        double& res) {
    // explicit fmas: every instantiation (walk direction, branch-free or not, strip or tile) rounds
    // alike, so a cell's value does not depend on which strip or pass shape computed it
    const double s = fma(cn, yp, fma(cs, ym, fma(cw, xm, ce * xp)));
    const double aq = OP == 0 ? fma(dg, q, s) : fma(dg, q, -(alpha * s));
    res = b - aq;
    return fma(w, res, q);
}

// Streamed field stores bypass the Infinity Cache (non-temporal): the 256 MiB die cache then
// keeps what the NEXT pass re-reads -- the rhs b, read by every sweep of a solve -- instead
// of filling with this pass's output (tools/membw2.hip, 4096^2 2-read + 1-write stream:
// 5.3 TB/s with plain stores, 6.8-7.5 TB/s with nt stores).
typedef double nsd2 __attribute__((ext_vector_type(2)));
// the iterate's loads may be non-temporal too: it is read once per pass (the prolongation pass)
__device__ __forceinline__ double2 ld_stream(const double* p, int nt) {
    if (nt > 0) {
        const nsd2 v = __builtin_nontemporal_load(reinterpret_cast<const nsd2*>(p));
        return make_double2(v.x, v.y);
    }
    return *reinterpret_cast<const double2*>(p);
}
__device__ __forceinline__ void st_stream(double* p, double2 v, bool nt) {
    if (nt) __builtin_nontemporal_store(nsd2{v.x, v.y}, reinterpret_cast<nsd2*>(p));
    else *reinterpret_cast<double2*>(p) = v;
}

// 1/x to within an ulp without a division: v_rcp_f64 + two Newton steps
__device__ __forceinline__ double rcp_nr(double x) {
    double y = __builtin_amdgcn_rcp(x);
    double e = fma(-x, y, 1.0);
    y = fma(y, e, y);
    e = fma(-x, y, 1.0);
    return fma(y, e, y);
}

// diag and omega/diag of a row's two columns, recomputed per use (no division, and no
// registers held across the row pipeline: the stages of k_sweep2 would need 40 VGPRs
// to cache them)
template <int OP>
struct DiagCache {
    double d0, d1, w0, w1;
    __device__ __forceinline__ void at(double rd, double cd0, double cd1, double alpha, double omega) {
        d0 = diag<OP>(rd, cd0, alpha);
        d1 = diag<OP>(rd, cd1, alpha);
        w0 = omega * rcp_nr(d0);
        w1 = omega * rcp_nr(d1);
    }
};

// per-wave LDS copy of the row coefficients (cw, ce, cw + ce [+ bx], hx) for rows ib-5 .. ib+L+4:
// read with a wave-uniform address (broadcast) instead of a global load on every row's
// critical path (hipcc cannot prove the tables read-only against the `out` stores)
constexpr int RC_OFF = 5;            // table row of strip row ib
constexpr int RC_MAX = 64 + 2 * RC_OFF;  // L <= 64
constexpr int RC_OFF3 = 6;           // k_sweep3: its first stage reads rows ib-5 .. ie+4 (ib-6 .. ie+5 with RES)
constexpr int L3_MAX = 128;          // k_sweep3's longest strip (the two-field pass: one resident round)
constexpr int RC_MAX3 = L3_MAX + 2 * RC_OFF3;
template <int OP, int RCO = RC_OFF, int LMAX = 64>
__device__ __forceinline__ void stage_rows(const StreamArgs& a, double (*rc)[4], int ib, int lane) {
    for (int t = lane; t < a.L + 2 * RCO && t < LMAX + 2 * RCO; t += 64) {
        const int gi = min(max(a.i0 + ib - RCO + t, 0), a.nx - 1);
        const double cw = a.cw[gi], ce = a.ce[gi];
        rc[t][0] = cw;
        rc[t][1] = ce;
        rc[t][2] = cw + ce + (OP == 1 ? a.bx[gi] : 0.0);
        rc[t][3] = a.hx ? a.hx[gi] : 0.0;
    }
}

template <int OP, bool RB, bool RES>
__global__ __launch_bounds__(256) void k_sweep(StreamArgs a) {
    __shared__ double rcs[4][RC_MAX][4];
    const int lane = threadIdx.x & 63;
    const int nstr = a.nsj * a.nsi;
    const int wid = xcd_swizzle(blockIdx.x, gridDim.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double (*rc)[4] = rcs[threadIdx.x >> 6];
    if (wid < nstr) stage_rows<OP>(a, rc, (wid / a.nsj) * a.L, lane);
    __syncthreads();
    double res = 0.0;
    if (wid < nstr) {
        const int si = wid / a.nsj, sj = wid - si * a.nsj;
        const int jb = sj * SW, ib = si * a.L;
        const int ie = min(ib + a.L, a.nxl);
        const int ny = a.ny, ld = a.ld;
        const int c0 = jb - 2 + 2 * lane, c1 = c0 + 1;
        const int lc = min(max(c0, 0), ld - 2);                 // clamped 16-B aligned pair
        const bool v0 = c0 >= 0 && c0 < ny, v1 = c1 >= 0 && c1 < ny;   // cells inside the domain
        const bool wr = lane >= 1 && lane <= 62 && c0 < ny;      // this lane's pair is written
        const bool o0 = wr && v0, o1 = wr && v1;                 // ... and counts in the residual
        const int k0 = min(max(c0, 0), ny - 1), k1 = min(max(c1, 0), ny - 1);
        const double cs0 = a.cs[k0], cn0 = a.cn[k0], cd0 = cs0 + cn0 + (OP == 1 ? a.by[k0] : 0.0);
        const double cs1 = a.cs[k1], cn1 = a.cn[k1], cd1 = cs1 + cn1 + (OP == 1 ? a.by[k1] : 0.0);
        const double shift = (OP == 0 && a.shift) ? a.shift[0] : 0.0;
        const double alpha = a.alpha, omega = a.omega;
        const int rlo = -HALO, rhi = a.nxl + HALO - 1;

        // one row of phi (row r) and of b (row r-1), per lane.  Rows no stage reads -- phi
        // past r1 (the prefetch overrun) and b before the first red / relaxed row -- are
        // clamped onto a row this wave fetches anyway: a cache hit instead of an HBM row,
        // with no branch in the load pipeline.
        double2 Q[SD], QB[SD];
        const int r1 = RB ? ie + 1 : ie;
        const int blo = max(RB ? ib - 1 : ib, rlo), phi_hi = min(r1, rhi);
        auto load = [&](int slot_r, double2& p, double2& bb) {
            const int lp = min(max(slot_r, rlo), phi_hi), lb = min(max(slot_r - 1, blo), rhi);
            p = ld_stream(a.in + (ptrdiff_t)lp * ld + lc, a.ntl);
            bb = *reinterpret_cast<const double2*>(a.b + (ptrdiff_t)lb * ld + lc);
        };

        double2 P0 = {0, 0}, P1 = {0, 0}, P2 = {0, 0}, R0 = {0, 0}, R1 = {0, 0}, R2 = {0, 0};
        double2 Bm = {0, 0}, Bk = {0, 0};

        DiagCache<OP> dm, dk;   // red-stage row m / black-stage row k
        auto step = [&](const double2 p, const double2 bb, int r) {
            P0 = P1; P1 = P2; P2 = p;
            Bk = Bm;
            Bm = make_double2(bb.x - shift, bb.y - shift);
            const int m = r - 1, gim = a.i0 + m;
            double2 Rn = P1;
            if (m >= ib - 1 && m <= ie) {
                double lf = lane_up1(P1.y), rt = lane_dn1(P1.x);
                const double* rw = rc[m - ib + RC_OFF];
                const double cw = rw[0], ce = rw[1];
                dm.at(rw[2], cd0, cd1, alpha, omega);
                double r0, r1;
                if (RES && m >= ib && m < ie) {
                    relax<OP>(P1.x, P0.x, P2.x, lf, P1.y, Bm.x, cw, ce, cs0, cn0, dm.d0, dm.w0, alpha, r0);
                    relax<OP>(P1.y, P0.y, P2.y, P1.x, rt, Bm.y, cw, ce, cs1, cn1, dm.d1, dm.w1, alpha, r1);
                    res += (o0 ? r0 * r0 : 0.0) + (o1 ? r1 * r1 : 0.0);
                }
                if (!RB) {
                    if (m >= ib && m < ie) {
                        double2 o = P1;
                        if (v0) o.x = relax<OP>(P1.x, P0.x, P2.x, lf, P1.y, Bm.x, cw, ce, cs0, cn0, dm.d0, dm.w0, alpha, r0);
                        if (v1) o.y = relax<OP>(P1.y, P0.y, P2.y, P1.x, rt, Bm.y, cw, ce, cs1, cn1, dm.d1, dm.w1, alpha, r1);
                        if (wr) st_stream(a.out + (ptrdiff_t)m * ld + c0, o, a.nt);
                    }
                } else if (gim >= 0 && gim < a.nx) {
                    if ((gim & 1) == 0) {  // red = (gi + j) even = c0
                        if (v0) Rn.x = relax<OP>(P1.x, P0.x, P2.x, lf, P1.y, Bm.x, cw, ce, cs0, cn0, dm.d0, dm.w0, alpha, r0);
                    } else {               // red = c1
                        if (v1) Rn.y = relax<OP>(P1.y, P0.y, P2.y, P1.x, rt, Bm.y, cw, ce, cs1, cn1, dm.d1, dm.w1, alpha, r1);
                    }
                }
            }
            if (RB) {
                R0 = R1; R1 = R2; R2 = Rn;
                const int k = r - 2, gik = a.i0 + k;
                if (k >= ib && k < ie) {
                    const double lf = lane_up1(R1.y), rt = lane_dn1(R1.x);
                    const double* rw = rc[k - ib + RC_OFF];
                    const double cw = rw[0], ce = rw[1];
                    dk.at(rw[2], cd0, cd1, alpha, omega);
                    double2 o = R1;
                    double rr;
                    if ((gik & 1) == 0) {  // black = c1
                        if (v1) o.y = relax<OP>(R1.y, R0.y, R2.y, R1.x, rt, Bk.y, cw, ce, cs1, cn1, dk.d1, dk.w1, alpha, rr);
                    } else {               // black = c0
                        if (v0) o.x = relax<OP>(R1.x, R0.x, R2.x, lf, R1.y, Bk.x, cw, ce, cs0, cn0, dk.d0, dk.w0, alpha, rr);
                    }
                    if (wr) st_stream(a.out + (ptrdiff_t)k * ld + c0, o, a.nt);
                }
            }
        };

        // rows ib-2 .. ie+1 (RB) / ib-1 .. ie (Jacobi); SD rows in flight
        const int r0 = RB ? ib - 2 : ib - 1;
#pragma unroll
        for (int q = 0; q < SD; q++) load(r0 + q, Q[q], QB[q]);
        for (int r = r0; r <= r1; r += SD) {
#pragma unroll
            for (int q = 0; q < SD; q++) {
                if (r + q <= r1) step(Q[q], QB[q], r + q);
                load(r + q + SD, Q[q], QB[q]);
            }
        }
    }
    if (RES) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) res += __shfl_xor(res, off, 64);
        if (lane == 0 && wid < nstr) a.part[wid] = res;
    }
}

// ------------------------------------------------ K4 Jacobi, branch-free streaming sweep
// The Jacobi sweep on fp64 fields (the north star's roofline kernel) and on fp32 fields
// (configs[4]: "fp32 fields + fp64 Poisson residual", SURVEY.md 8(d) C5: 12 B/cell).  Every
// cell's update and residual are computed in fp64 from the widened values; only the new
// iterate is rounded (fp32), and the residual norm is summed in fp64.  The strip walk of
// k_sweep<Jacobi> with 16 B per lane per row (fp64: 2 columns, 124 written per strip; fp32:
// 4 columns, 248), but the row loop is branch-free: every step computes, and a lane that
// must not write (a halo lane, a column past ny, a pipeline-fill or tail row) stores through
// a buffer resource at an out-of-range offset, which the hardware drops.  With the stores in
// branches the compiler's vmcnt accounting assumed the fewest issued operations at each
// join and waited for nearly every prefetched row.  fp32 rows are ld floats long (the fp64
// planes' ld), so a ghost row exchange is ld/2 doubles.
typedef unsigned nsu4 __attribute__((ext_vector_type(4)));
typedef unsigned nsu2 __attribute__((ext_vector_type(2)));
constexpr unsigned OOB = 0xFFFFFFF0u;
// (the streamed stores are nt: sc1 write-through lost the Infinity-Cache reuse -- Jacobi 73 ->
// 88 us -- and sc1 nt measured the same as nt)

// A copy the compiler cannot coalesce away.  A row window (rows r-2, r-1, r) that takes the
// freshly consumed prefetch slot by plain assignment ends up sharing the slot's register;
// the slot's next load must then land elsewhere, and the loop latch moves it back -- a move
// that waits for the in-flight load, which cut the effective prefetch depth to ~1 row.
// Copying into the window at consumption time (when the value has arrived anyway) frees
// the slot's register for its next load.
__device__ __forceinline__ nsu4 vcopy(const nsu4 x) {
    nsu4 y;
    asm volatile("v_mov_b32 %0, %1" : "=v"(y.x) : "v"(x.x));
    asm volatile("v_mov_b32 %0, %1" : "=v"(y.y) : "v"(x.y));
    asm volatile("v_mov_b32 %0, %1" : "=v"(y.z) : "v"(x.z));
    asm volatile("v_mov_b32 %0, %1" : "=v"(y.w) : "v"(x.w));
    return y;
}
__device__ __forceinline__ double2 vcopy(const double2 x) {
    const nsu4 y = vcopy((nsu4){(unsigned)__double2loint(x.x), (unsigned)__double2hiint(x.x),
                                (unsigned)__double2loint(x.y), (unsigned)__double2hiint(x.y)});
    return make_double2(__hiloint2double((int)y.y, (int)y.x), __hiloint2double((int)y.w, (int)y.z));
}

template <class T> struct Lane16;
template <> struct Lane16<float> {
    static constexpr int V = 4;
    __device__ static double get(const nsu4& u, int q) { return (double)__uint_as_float(u[q]); }
    __device__ static void put(nsu4& u, int q, double x) { u[q] = __float_as_uint((float)x); }
};
template <> struct Lane16<double> {
    static constexpr int V = 2;
    __device__ static double get(const nsu4& u, int q) { return __hiloint2double((int)u[2 * q + 1], (int)u[2 * q]); }
    __device__ static void put(nsu4& u, int q, double x) {
        u[2 * q] = (unsigned)__double2loint(x);
        u[2 * q + 1] = (unsigned)__double2hiint(x);
    }
};

template <class T>
struct JacobiArgs {
    const T* in;
    T* out;
    const T* b;
    const double* shift;
    const double *cw, *ce, *cs, *cn;
    double omega;
    int nx, ny, i0, nxl, ld;          // ld in elements
    int nsj, nsi, L;
    double* part;
};

template <class T, bool RES, bool NT>
__global__ __launch_bounds__(256) void k_jacobi_s(JacobiArgs<T> a) {
    constexpr int V = Lane16<T>::V, SWV = 62 * V;
    __shared__ double rcs[4][RC_MAX][3];
    const int lane = threadIdx.x & 63;
    const int nstr = a.nsj * a.nsi;
    const int wid = xcd_swizzle(blockIdx.x, gridDim.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double (*rc)[3] = rcs[threadIdx.x >> 6];
    if (wid < nstr) {
        const int ib = (wid / a.nsj) * a.L;
        for (int t = lane; t < a.L + 2 * RC_OFF && t < RC_MAX; t += 64) {
            const int gi = min(max(a.i0 + ib - RC_OFF + t, 0), a.nx - 1);
            const double cw = a.cw[gi], ce = a.ce[gi];
            rc[t][0] = cw;
            rc[t][1] = ce;
            rc[t][2] = cw + ce;
        }
    }
    __syncthreads();
    double res = 0.0;
    if (wid < nstr) {
        const int si = wid / a.nsj, sj = wid - si * a.nsj;
        const int jb = sj * SWV, ib = si * a.L;
        const int ie = min(ib + a.L, a.nxl);
        const int ny = a.ny, ld = a.ld;
        const int c0 = jb - V + V * lane;
        const int lc = min(max(c0, 0), ld - V);
        const bool wr = lane >= 1 && lane <= 62 && c0 < ny;
        double cs[V], cn[V];
        bool in[V];
#pragma unroll
        for (int q = 0; q < V; q++) {
            const int c = c0 + q, k = min(max(c, 0), ny - 1);
            in[q] = c >= 0 && c < ny;
            cs[q] = a.cs[k];
            cn[q] = a.cn[k];
        }
        const double shift = a.shift ? a.shift[0] : 0.0;
        const double omega = a.omega;
        const int rlo = -HALO, rhi = a.nxl + HALO - 1;
        const int r1 = ie, blo = max(ib, rlo), phi_hi = min(r1, rhi);
        // the output plane (ghost rows included) as a buffer: offsets past its end are dropped
        const __amdgpu_buffer_rsrc_t out = __builtin_amdgcn_make_buffer_rsrc(
            a.out - (ptrdiff_t)HALO * ld, (short)0, (int)((unsigned)(a.nxl + 2 * HALO) * ld * (unsigned)sizeof(T)),
            0x00020000);
        nsu4 Q[SD], QB[SD];
        auto load = [&](int slot_r, nsu4& p, nsu4& bb) {
            const int lp = min(max(slot_r, rlo), phi_hi), lb = min(max(slot_r - 1, blo), rhi);
            p = *reinterpret_cast<const nsu4*>(a.in + (ptrdiff_t)lp * ld + lc);
            bb = *reinterpret_cast<const nsu4*>(a.b + (ptrdiff_t)lb * ld + lc);
        };
        nsu4 P0 = {0, 0, 0, 0}, P1 = {0, 0, 0, 0}, P2 = {0, 0, 0, 0};
        double dg[V], wq[V], rd_last = -1.0;
        auto step = [&](const nsu4 p, const nsu4 bb, int r) {
            P0 = P1; P1 = P2; P2 = vcopy(p);
            const int m = r - 1;
            const bool live = m >= ib && m < ie;
            const double* rw = rc[min(max(m - ib + RC_OFF, 0), RC_MAX - 1)];
            const double cw = rw[0], ce = rw[1], rd = rw[2];
            double xm[V], xq[V], xp[V], bq[V];
#pragma unroll
            for (int q = 0; q < V; q++) {
                xm[q] = Lane16<T>::get(P0, q);
                xq[q] = Lane16<T>::get(P1, q);
                xp[q] = Lane16<T>::get(P2, q);
                bq[q] = Lane16<T>::get(bb, q);
            }
            const double lf = lane_up1(xq[V - 1]), rt = lane_dn1(xq[0]);
            if (rd != rd_last) {   // the diagonal's row part repeats on a uniform grid
#pragma unroll
                for (int q = 0; q < V; q++) {
                    dg[q] = diag<0>(rd, cs[q] + cn[q], 0.0);
                    wq[q] = omega * rcp_nr(dg[q]);
                }
                rd_last = rd;
            }
            nsu4 o;
#pragma unroll
            for (int q = 0; q < V; q++) {
                const double ym = q == 0 ? lf : xq[q - 1], yp = q == V - 1 ? rt : xq[q + 1];
                double rr;
                const double v = relax<0>(xq[q], xm[q], xp[q], ym, yp, bq[q] - shift, cw, ce, cs[q], cn[q], dg[q],
                                          wq[q], 0.0, rr);
                Lane16<T>::put(o, q, in[q] ? v : xq[q]);
                if (RES) res += (live && wr && in[q]) ? rr * rr : 0.0;
            }
            const unsigned off =
                (live && wr) ? ((unsigned)(m + HALO) * (unsigned)ld + (unsigned)c0) * (unsigned)sizeof(T) : OOB;
            __builtin_amdgcn_raw_buffer_store_b128(o, out, (int)off, 0, NT ? 2 : 0);
        };
        const int r0 = ib - 1;
#pragma unroll
        for (int q = 0; q < SD; q++) {
            load(r0 + q, Q[q], QB[q]);
            asm volatile("" ::: "memory");   // keep the slots' issue order (the loop's vmcnt bookkeeping)
        }
        for (int r = r0; r <= r1; r += SD) {
#pragma unroll
            for (int q = 0; q < SD; q++) {
                step(Q[q], QB[q], r + q);       // rows past r1: computed, not stored
                load(r + q + SD, Q[q], QB[q]);
            }
        }
    }
    if (RES) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) res += __shfl_xor(res, off, 64);
        if (lane == 0 && wid < nstr) a.part[wid] = res;
    }
}

// fp64 <-> fp32 copies of a slab's own rows (fp32 rows: ld floats)
__global__ __launch_bounds__(256) void k_to_f32(const double* __restrict__ src, float* __restrict__ dst, long n) {
    for (long k = (long)blockIdx.x * 256 + threadIdx.x; k < n; k += (long)gridDim.x * 256) dst[k] = (float)src[k];
}
__global__ __launch_bounds__(256) void k_to_f64(const float* __restrict__ src, double* __restrict__ dst, long n) {
    for (long k = (long)blockIdx.x * 256 + threadIdx.x; k < n; k += (long)gridDim.x * 256) dst[k] = (double)src[k];
}

// ---------------------------------------------------------------- K1 as streaming strips
// k_rhs_s: ConstructRHS_V on the cells at least two from every wall -- the MUSCL stencil's
// reach, so every neighbour exists and no ghost is evaluated (TopoInner) -- with every MUSCL
// slope and every face flux computed ONCE.  (rhs_cell, per cell, evaluates 12 slopes and 8 face
// fluxes -- each face twice, once from each side: ~500 fp64 wave-instructions per cell, K1's
// bound.)  The strip walk of the sweeps: a wave owns 128 columns (2 per lane, 124 written) and
// walks L rows; when row r arrives, row r-1's x-slopes are formed (rows r-2 .. r in the
// window), then the x-face between rows r-2 and r-1 (its two states from those rows' slopes),
// and row r-2 is complete: its W face is the previous step's, its E face this one's, its y-faces
// come from row r-2's y-slopes across the lanes (face (c0-1 | c0) per lane, (c0 | c1) inside the
// lane, the third from lane + 1 by DPP).  Face states / fluxes / the RHS assembly are rhs_cell's
// expressions, so every value equals the tile kernel's up to FMA contraction.  The ring of cells
// within two of a wall (and an odd ny's last column) is k_rhs_ring's: rhs_cell<BC> per cell, the
// ApplyBoundaryConditions terms included.  u, v rows ib-2 .. ie+1 are read (2 ghost rows), cu0 /
// cv0 at the output rows (updated in place: each lane reads its cells' old values before it
// stores them), stores through buffer resources (dropped offsets for unwritten lanes / rows).
// (r6) CorrectVelocities + GradP of one cell (FluidSolver.cpp:420-456, 512-534): u = u* - dt dphi/dx, v = v* - dt
// dphi/dy from the face values of phi (the wall / inlet ghost phi itself: 0.5 (p + p)).  Explicit fmas and one
// expression for every caller -- K5 (k_cell_s<5>), K1's deferred correction (k_rhs_s CORR) and its wall ring --
// so a deferred correction gives K5's bits
__device__ __forceinline__ double fvp(double q, double qn, bool has, double r) {
    return has ? fma(qn, r, q * (1.0 - r)) : 0.5 * (q + q);
}
// (r6, A/B) hx, hy: CORR_H(1 / h, h) -- CORR_RCP=1 takes the reciprocal tables' 1 / hx, 1 / hy, a product instead of
// the IEEE division (four per cell pair); measured no faster (K1' 342 vs 343 us, K5 140 vs 137), so the default keeps
// the division and its bits
#ifndef CORR_RCP
#define CORR_RCP 0
#endif
#define CORR_H(r, h) (CORR_RCP ? (r) : (h))
__device__ __forceinline__ void corr1(double us, double vs, double pc, double pw, double pe, double ps, double pn,
                                      bool hW, bool hE, bool hS, bool hN, double fw, double fe, double fs, double fn,
                                      double hx, double hy, double dt, double& u, double& v) {
    const double V0 = fvp(pc, pw, hW, fw), V1 = fvp(pc, pe, hE, fe);
    const double V2 = fvp(pc, ps, hS, fs), V3 = fvp(pc, pn, hN, fn);
    u = fma(-dt, CORR_RCP ? (V1 - V0) * hx : (V1 - V0) / hx, us);
    v = fma(-dt, CORR_RCP ? (V3 - V2) * hy : (V3 - V2) / hy, vs);
}
// the same at cell (li, j) from global loads (K1's wall ring; a rectangle without NEUMANN sides)
__device__ __forceinline__ void corr_at(const Geo& g, const Coef& c, double dt, const double* __restrict__ us,
                                        const double* __restrict__ vs, const double* __restrict__ phi, int li, int j,
                                        double& u, double& v) {
    const int gi = g.i0 + li, ld = g.ld;
    const bool hW = gi > 0, hE = gi < g.nx - 1, hS = j > 0, hN = j < g.ny - 1;
    const ptrdiff_t o = (ptrdiff_t)li * ld + j;
    const double pc = phi[o];
    const double pw = hW ? phi[o - ld] : pc, pe = hE ? phi[o + ld] : pc;
    const double ps = hS ? phi[o - 1] : pc, pn = hN ? phi[o + 1] : pc;
    corr1(us[o], vs[o], pc, pw, pe, ps, pn, hW, hE, hS, hN, c.fwx[gi], c.fex[gi], c.fsy[j], c.fny[j],
          CORR_H(c.rhx[gi], c.hx[gi]), CORR_H(c.rhy[j], c.hy[j]), dt, u, v);
}

// the ring of k_rhs_s (below): the slab's cells within two rows of the W / E walls (whole rows),
// and on the other rows the columns 0, 1 and [jhi, ny).  Thread k: the whole wall rows first
// (nfull of them, from local row fr[q]), then (ncol columns) x the other rows.
struct RhsRingArgs {
    int nfull, fr[4];             // whole rows (local indices)
    int ncol, jhi;                // ring columns per other row: 0, 1, jhi .. ny-1
    int rlo, rhi;                 // the other rows: local [rlo, rhi)
    int n;                        // ring cells
};
struct RhsStreamArgs {
    Geo g;
    Coef c;
    double dt, re;
    const double *u, *v, *phi;
    double *cu, *cv, *ru, *rv;
    double* part;                 // 2 per strip: sum ru^2, sum rv^2 of its written cells; then 2 per ring block
    int nsj;
    RowPlan P;                    // strip rows of this launch (plan_rows)
    int ilo, ihi, jhi;            // written cells: local rows [ilo, ihi), columns [2, jhi)
    int nsblk;                    // workgroups of strips; those past it take the ring (nring of them)
    int nring, nstr;              // ring workgroups of this launch, the pass's strip count (partial offset)
    RhsRingArgs R;
    // (r6) CORR: the previous step's CorrectVelocities folded in -- u, v above are u*, v*, phi is phi^n: every u, v
    // value the stencil reads is corrected on the fly (corr1, K5's arithmetic), the written cells' corrected u, v
    // go to uo, vo and their min / max to mm (4 per strip, then 4 per ring block)
    double *uo, *vo, *mm;
};
template <bool CORR = false>
__device__ __forceinline__ void rhs_ring_body(const Geo& g, const Coef& c, double dt, double re,
                                              const double* __restrict__ u, const double* __restrict__ v,
                                              const double* __restrict__ phi, double* __restrict__ cu,
                                              double* __restrict__ cv, double* __restrict__ ru,
                                              double* __restrict__ rv, double* __restrict__ part, const RhsRingArgs& R,
                                              int blk, double* __restrict__ uo = nullptr, double* __restrict__ vo = nullptr,
                                              double* __restrict__ mm = nullptr) {
    const int k = blk * 256 + threadIdx.x;
    double acc[2] = {0.0, 0.0};
    double amm[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
    if (k < R.n) {
        int li, j;
        const int nf = R.nfull * g.ny;
        if (k < nf) {
            const int q = k / g.ny;
            li = R.fr[q];
            j = k - q * g.ny;
        } else {
            const int q = (k - nf) / R.ncol, e = (k - nf) - q * R.ncol;
            li = R.rlo + q;
            j = e < 2 ? e : R.jhi + (e - 2);
        }
        const int ld = g.ld, gi = g.i0 + li;
        const ptrdiff_t o = (ptrdiff_t)li * ld + j;
        // (CORR: the stencil's u, v corrected from u*, v* and phi^n on the fly, each value by corr_at)
        auto U = [&](int di, int dj) {
            if (!CORR) return ldf(u, ld, li + di, j + dj);
            double a, b;
            corr_at(g, c, dt, u, v, phi, li + di, j + dj, a, b);
            return a;
        };
        auto V = [&](int di, int dj) {
            if (!CORR) return ldf(v, ld, li + di, j + dj);
            double a, b;
            corr_at(g, c, dt, u, v, phi, li + di, j + dj, a, b);
            return b;
        };
        auto X = [&](int t, int d) { return (t == 0 ? c.hx : t == 1 ? c.rhx : c.rsx)[gi + d]; };
        auto Y = [&](int t, int d) { return (t == 0 ? c.hy : t == 1 ? c.rhy : c.rsy)[j + d]; };
        double cun, cvn, ru_, rv_;
        rhs_cell<true, TopoRect>(g, c, dt, re, U, V, X, Y, phi, li, j, cu[o], cv[o], cun, cvn, ru_, rv_);
        cu[o] = cun;
        cv[o] = cvn;
        ru[o] = ru_;
        rv[o] = rv_;
        if (li >= g.sr0 && li < g.sr1) {   // (r5: own rows only)
            acc[0] = ru_ * ru_;
            acc[1] = rv_ * rv_;
        }
        if (CORR) {
            double un, vn;
            corr_at(g, c, dt, u, v, phi, li, j, un, vn);
            uo[o] = un;
            vo[o] = vn;
            amm[0] = un != un ? -INFINITY : un;
            amm[1] = un != un ? -INFINITY : -un;
            amm[2] = vn != vn ? -INFINITY : vn;
            amm[3] = vn != vn ? -INFINITY : -vn;
        }
    }
    block_reduce_sum<2>(acc, part + 2 * blk);
    if (CORR) block_reduce_min<4>(amm, mm + 4 * blk);
}

// (r6, A/B, measured and not kept: K1' 342-347 us with both against 338 without, same box,
// profiles/r06/ab/k1_loop_*_summary.txt -- the drain is not what bounds K1', its bytes are)
#ifndef K1_UR6
#define K1_UR6 0
#endif
#ifndef K1_QE_ALL
#define K1_QE_ALL 0
#endif
constexpr int K1_LMAX = 128;      // k_rhs_s: rows per strip at most (one resident round of strips)
#ifndef K1_ESPLIT
#define K1_ESPLIT 4               // (r5) k_rhs_s: rows per run of the edge bands after a slab's exchange (0: one run)
#endif
constexpr int RC_K1 = 4;          // k_rhs_s: row tables from row ib-4 (the window-fill steps read ib-4 .. )
template <bool NT, int SK, bool UY = false, bool CORR = false>
__device__ __forceinline__ void rhs_s_body(const RhsStreamArgs& A) {
    const Geo& g = A.g;
    const Coef& c = A.c;
    // the wall ring's workgroups, after the strips' (block-uniform).  (r6: the ring's workgroups first measured
    // 12 us slower, 305.5 vs 293.3 us on one box -- they then hold resident slots the strips' one round needs;
    // without the ring -- a timing probe, wrong results -- K1' took 331 vs 338 us: the ring is ~7 us of it)
    if ((int)blockIdx.x >= A.nsblk) {
        rhs_ring_body<CORR>(g, c, A.dt, A.re, A.u, A.v, A.phi, A.cu, A.cv, A.ru, A.rv, A.part + 2 * A.nstr, A.R,
                            (int)blockIdx.x - A.nsblk, A.uo, A.vo, CORR ? A.mm + 4 * A.nstr : nullptr);
        return;
    }
    const int sbx = (int)blockIdx.x;
    // per row: hx, 1/hx, 2/(h_{i-1}+h_i), 2/(h_i+h_{i+1}); (r6, CORR) + GradP's face weights fwx, fex -- read per row by
    // the folded correction, as global (scalar) loads they put a memory round trip into every row step
    constexpr int RCW = CORR ? 6 : 4;
    __shared__ double rcs[4][K1_LMAX + 2 * RC_K1 + 2][RCW];
    const int lane = threadIdx.x & 63;
    const int nstr = A.nsj * A.P.nrun;
    const int w = xcd_swizzle(sbx, A.nsblk) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double (*rc)[RCW] = rcs[threadIdx.x >> 6];
    const int run = w / A.nsj, sj = w - run * A.nsj;
    const int wid = (A.P.pbase + run) * A.nsj + sj;
    int ib, ie;
    A.P.rows(run, ib, ie);
    if (w < nstr) {
        for (int t = lane; t < ie - ib + 2 * RC_K1 + 2; t += 64) {
            const int gi = min(max(g.i0 + ib - RC_K1 + t, 0), g.nx - 1);
            rc[t][0] = c.hx[gi];
            rc[t][1] = c.rhx[gi];
            rc[t][2] = c.rsx[gi];
            rc[t][3] = c.rsx[gi + 1];
            if constexpr (CORR) {
                rc[t][4] = c.fwx[gi];
                rc[t][5] = c.fex[gi];
            }
        }
    }
    __syncthreads();
    double acc0 = 0.0, acc1 = 0.0;
    double amm[4] = {INFINITY, INFINITY, INFINITY, INFINITY};   // (CORR: umin, -umax, vmin, -vmax)
    if (w < nstr) {
        const int ny = g.ny, ld = g.ld;
        const int jb = sj * SW;
        const int c0 = jb - 2 + 2 * lane;
        const int lc = min(max(c0, 0), ld - 2);
        const bool wr = lane >= 1 && lane <= 62 && c0 >= 2 && c0 < A.jhi;
        // column tables (clamped; a clamped column only feeds unwritten lanes).  (r5) UY: hy uniform -- every
        // column's hy, 1 / hy and 2 / (hy + hy) are one value (the same doubles: written cells never reach
        // rsy[0] or rsy[ny], the only different entries), kept wave-uniform (SGPRs): 16 VGPRs less, three
        // waves per SIMD
        const int k0 = min(max(c0, 0), ny - 1), k1 = min(max(c0 + 1, 0), ny - 1), km = min(max(c0 - 1, 0), ny - 1);
        const double hy0 = UY ? c.hy[0] : c.hy[k0], hy1 = UY ? c.hy[0] : c.hy[k1], hym = UY ? c.hy[0] : c.hy[km];
        const double ry0 = UY ? c.rhy[0] : c.rhy[k0], ry1 = UY ? c.rhy[0] : c.rhy[k1];
        const double rs0 = UY ? c.rsy[1] : c.rsy[k0], rs1 = UY ? c.rsy[1] : c.rsy[k1],
                     rs2 = UY ? c.rsy[1] : c.rsy[min(k1 + 1, ny)];
        const double dt = A.dt, hre = 0.5 / A.re;
        const int rlo = -HALO, rhi = g.nxl + HALO - 1;
        const __amdgpu_buffer_rsrc_t bcu = __builtin_amdgcn_make_buffer_rsrc(A.cu, (short)0, 0x7FFFFFF0, 0x00020000);
        const __amdgpu_buffer_rsrc_t bcv = __builtin_amdgcn_make_buffer_rsrc(A.cv, (short)0, 0x7FFFFFF0, 0x00020000);
        const __amdgpu_buffer_rsrc_t bru = __builtin_amdgcn_make_buffer_rsrc(A.ru, (short)0, 0x7FFFFFF0, 0x00020000);
        const __amdgpu_buffer_rsrc_t brv = __builtin_amdgcn_make_buffer_rsrc(A.rv, (short)0, 0x7FFFFFF0, 0x00020000);
        // one row of u, v (row r) and of cu0, cv0 (row r-2, the output row of that step)
        // SK rows in flight, 4 double2 each (u, v, cu0, cv0)
        // (CORR: + phi^n's row r+1, and for the wave's edge lanes the phi value beyond their outer column -- lane 0
        // column c0 - 1, lane 63 column c1 + 1 -- the correction's y-neighbour no lane holds)
        const int ce = lane == 0 ? max(c0 - 1, 0) : min(c0 + 2, ny - 1);
        double2 QU[SK], QV[SK], QC[SK], QD[SK], QP[CORR ? SK : 1];
        double QE[CORR ? SK : 1];
        auto load = [&](int r, double2& qu, double2& qv, double2& qc, double2& qd, double2& qp, double& qe) {
            const int lr = min(max(r, rlo), rhi), lo = min(max(r - 2, 0), g.nxl - 1);
            qu = *reinterpret_cast<const double2*>(A.u + (ptrdiff_t)lr * ld + lc);
            qv = *reinterpret_cast<const double2*>(A.v + (ptrdiff_t)lr * ld + lc);
            qc = *reinterpret_cast<const double2*>(A.cu + (ptrdiff_t)lo * ld + lc);
            qd = *reinterpret_cast<const double2*>(A.cv + (ptrdiff_t)lo * ld + lc);
            if (CORR) {
                const int lp = min(max(r + 1, rlo), rhi);
                qp = *reinterpret_cast<const double2*>(A.phi + (ptrdiff_t)lp * ld + lc);
                // (r6, A/B K1_QE_ALL=1: every lane loads -- the branch-free form; with K1_UR6 it removes the loop head's
                // s_waitcnt vmcnt(0), which measured no faster)
                if (K1_QE_ALL || lane == 0 || lane == 63) qe = A.phi[(ptrdiff_t)lp * ld + ce];
            }
        };
        // CORR: phi^n rows r-1 .. r+1 (PH0..PH2) and the edge lanes' outer values of rows r, r+1 (E1, E2); the
        // correction's column constants (hy uniform on the direct-solve grids that defer K5: GradP's face weights
        // there are 0.5 exactly, fsy / fny's values)
        double2 PH0 = {0, 0}, PH1 = {0, 0}, PH2 = {0, 0};
        double E1 = 0.0, E2 = 0.0;
        const bool cs0 = c0 > 0, cn0 = c0 < ny - 1, cs1 = c0 + 1 > 0, cn1 = c0 + 1 < ny - 1;
        const double hyc = CORR_H(c.rhy[0], c.hy[0]);
        auto corr_row = [&](double2& qu, double2& qv, int r) {
            const int gi = g.i0 + min(max(r, rlo), rhi);
            const bool hW = gi > 0, hE = gi < g.nx - 1;
            // (the row table: row r is entry r - ib + RC_K1, the same clamped row)
            const double* rq = rc[r - ib + RC_K1];
            const double fw = rq[CORR ? 4 : 0], fe = rq[CORR ? 5 : 0], hx = CORR_H(rq[1], rq[0]), hy = hyc;
            double pl = lane_up1(PH1.y), pr = lane_dn1(PH1.x);
            if (lane == 0) pl = E1;
            if (lane == 63) pr = E1;
            double2 un, vn;
            corr1(qu.x, qv.x, PH1.x, PH0.x, PH2.x, pl, PH1.y, hW, hE, cs0, cn0, fw, fe, 0.5, 0.5, hx, hy, dt, un.x, vn.x);
            corr1(qu.y, qv.y, PH1.y, PH0.y, PH2.y, PH1.x, pr, hW, hE, cs1, cn1, fw, fe, 0.5, 0.5, hx, hy, dt, un.y, vn.y);
            qu = un;
            qv = vn;
        };
        // window rows r-3 .. r; x-slopes of rows r-2 (SP*) and r-1 (SC*); the x-face (r-3 | r-2)'s fluxes
        double2 U0 = {0, 0}, U1 = {0, 0}, U2 = {0, 0}, U3 = {0, 0};
        double2 V0 = {0, 0}, V1 = {0, 0}, V2 = {0, 0}, V3 = {0, 0};
        double2 SPu = {0, 0}, SPv = {0, 0};
        double2 FWnn = {0, 0}, FWuv = {0, 0};
        auto xslope = [&](double qm, double qc, double qp, const double* rw) {
            return minmode_nd((qp - qc) * rw[3], (qc - qm) * rw[2]);
        };
        auto step = [&](double2 qu, double2 qv, const double2 cu0, const double2 cv0, const double2 qp, const double qe,
                        int r) {
            if (CORR) {
                // row r's u, v from u*, v* and phi^n rows r-1 .. r+1 (r5's K5 of the previous step, folded in);
                // the strip's own cells of row r store them, with their min / max
                PH0 = PH1; PH1 = PH2; PH2 = qp;
                E1 = E2; E2 = qe;
                corr_row(qu, qv, r);
                const bool lr = r >= ib && r < ie && r >= A.ilo && r < A.ihi && wr;
                const unsigned off = lr ? ((unsigned)r * (unsigned)ld + (unsigned)c0) * 8u : OOB;
                const __amdgpu_buffer_rsrc_t buo = __builtin_amdgcn_make_buffer_rsrc(A.uo, (short)0, 0x7FFFFFF0, 0x00020000);
                const __amdgpu_buffer_rsrc_t bvo = __builtin_amdgcn_make_buffer_rsrc(A.vo, (short)0, 0x7FFFFFF0, 0x00020000);
                const nsu4 du = {(unsigned)__double2loint(qu.x), (unsigned)__double2hiint(qu.x),
                                 (unsigned)__double2loint(qu.y), (unsigned)__double2hiint(qu.y)};
                const nsu4 dv = {(unsigned)__double2loint(qv.x), (unsigned)__double2hiint(qv.x),
                                 (unsigned)__double2loint(qv.y), (unsigned)__double2hiint(qv.y)};
                __builtin_amdgcn_raw_buffer_store_b128(du, buo, (int)off, 0, NT ? 2 : 0);
                __builtin_amdgcn_raw_buffer_store_b128(dv, bvo, (int)off, 0, NT ? 2 : 0);
                if (lr) {
#pragma unroll
                    for (int e = 0; e < 2; e++) {
                        const double un = e ? qu.y : qu.x, vn = e ? qv.y : qv.x;
                        amm[0] = fmin(amm[0], un != un ? -INFINITY : un);
                        amm[1] = fmin(amm[1], un != un ? -INFINITY : -un);
                        amm[2] = fmin(amm[2], vn != vn ? -INFINITY : vn);
                        amm[3] = fmin(amm[3], vn != vn ? -INFINITY : -vn);
                    }
                }
            }
            U0 = U1; U1 = U2; U2 = U3; U3 = vcopy(qu);
            V0 = V1; V1 = V2; V2 = V3; V3 = vcopy(qv);
            const double* rm = rc[r - 2 - ib + RC_K1];   // output row m = r-2
            const double* rn = rc[r - 1 - ib + RC_K1];   // row r-1
            // x-slopes of row r-1
            const double2 SCu = make_double2(xslope(U1.x, U2.x, U3.x, rn), xslope(U1.y, U2.y, U3.y, rn));
            const double2 SCv = make_double2(xslope(V1.x, V2.x, V3.x, rn), xslope(V1.y, V2.y, V3.y, rn));
            // x-face (r-2 | r-1): left states from row r-2, right from row r-1 (rhs_cell's C[2] / C[0])
            const double hxm = rm[0], hxn = rn[0];
            double2 FEnn, FEuv;
            {
                const double ul0 = U1.x + hxm / 2 * SPu.x, vl0 = V1.x + hxm / 2 * SPv.x;
                const double ur0 = U2.x - hxn / 2 * SCu.x, vr0 = V2.x - hxn / 2 * SCv.x;
                const double ul1 = U1.y + hxm / 2 * SPu.y, vl1 = V1.y + hxm / 2 * SPv.y;
                const double ur1 = U2.y - hxn / 2 * SCu.y, vr1 = V2.y - hxn / 2 * SCv.y;
                FEnn = make_double2(fnn(ul0, ur0), fnn(ul1, ur1));
                FEuv = make_double2(fuv(ul0, vl0, ur0, vr0), fuv(ul1, vl1, ur1, vr1));
            }
            // row m = r-2: y-slopes across the lanes (columns c0 - 1 .. c1 + 1)
            const double um = lane_up1(U1.y), up = lane_dn1(U1.x), vm = lane_up1(V1.y), vp = lane_dn1(V1.x);
            const double su0 = minmode_nd((U1.y - U1.x) * rs1, (U1.x - um) * rs0);
            const double su1 = minmode_nd((up - U1.y) * rs2, (U1.y - U1.x) * rs1);
            const double sv0 = minmode_nd((V1.y - V1.x) * rs1, (V1.x - vm) * rs0);
            const double sv1 = minmode_nd((vp - V1.y) * rs2, (V1.y - V1.x) * rs1);
            const double sum_ = lane_up1(su1), svm = lane_up1(sv1);   // column c0 - 1's slopes
            // y-faces (c0-1 | c0) and (c0 | c1): lower / upper states (rhs_cell's C[4..7])
            double fa_nn, fa_uv, fb_nn, fb_uv;
            {
                const double u1 = um + hym / 2 * sum_, v1 = vm + hym / 2 * svm;
                const double u2 = U1.x - hy0 / 2 * su0, v2 = V1.x - hy0 / 2 * sv0;
                fa_nn = fnn(v1, v2);
                fa_uv = fuv(u1, v1, u2, v2);
            }
            {
                const double u1 = U1.x + hy0 / 2 * su0, v1 = V1.x + hy0 / 2 * sv0;
                const double u2 = U1.y - hy1 / 2 * su1, v2 = V1.y - hy1 / 2 * sv1;
                fb_nn = fnn(v1, v2);
                fb_uv = fuv(u1, v1, u2, v2);
            }
            const double fc_nn = lane_dn1(fa_nn), fc_uv = lane_dn1(fa_uv);   // (c1 | c1+1)
            // the cells of row m
            const double rx = rm[1], sxW = rm[2], sxE = rm[3];
            double out[4][2];
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const double uc = e ? U1.y : U1.x, vc = e ? V1.y : V1.x;
                const double uW = e ? U0.y : U0.x, vW = e ? V0.y : V0.x, uE = e ? U2.y : U2.x, vE = e ? V2.y : V2.x;
                const double uS = e ? U1.x : um, vS = e ? V1.x : vm, uN = e ? up : U1.y, vN = e ? vp : V1.y;
                const double ry = e ? ry1 : ry0, syS = e ? rs1 : rs0, syN = e ? rs2 : rs1;
                double ru_ = 0.0 + 1.0 * uc, rv_ = 0.0 + 1.0 * vc;
                ru_ += 0.5 * dt * (e ? cu0.y : cu0.x);
                rv_ += 0.5 * dt * (e ? cv0.y : cv0.x);
                double D0 = hre * (uc - uW) * sxW, D1 = hre * (uE - uc) * sxE;
                double D2 = hre * (uc - uS) * syS, D3 = hre * (uN - uc) * syN;
                ru_ += dt * ((D1 - D0) * rx + (D3 - D2) * ry);
                D0 = hre * (vc - vW) * sxW; D1 = hre * (vE - vc) * sxE;
                D2 = hre * (vc - vS) * syS; D3 = hre * (vN - vc) * syN;
                rv_ += dt * ((D1 - D0) * rx + (D3 - D2) * ry);
                // C[0..3] from the x-faces (W: previous step, E: this one), C[4..7] from the y-faces
                const double C0 = e ? FWnn.y : FWnn.x, C1 = e ? FWuv.y : FWuv.x;
                const double C2 = e ? FEnn.y : FEnn.x, C3 = e ? FEuv.y : FEuv.x;
                const double C4 = e ? fb_uv : fa_uv, C5 = e ? fb_nn : fa_nn;
                const double C6 = e ? fc_uv : fb_uv, C7 = e ? fc_nn : fb_nn;
                double val = (C2 - C0) * rx + (C6 - C4) * ry;
                out[0][e] = val;
                ru_ += val * (-1.5 * dt);
                val = (C3 - C1) * rx + (C7 - C5) * ry;
                out[1][e] = val;
                rv_ += val * (-1.5 * dt);
                out[2][e] = ru_;
                out[3][e] = rv_;
            }
            const int m = r - 2;
            const bool live = m >= ib && m < ie && m >= A.ilo && m < A.ihi;
            if (live && wr && m >= g.sr0 && m < g.sr1) {   // (r5: a deep-ghost launch sums its own rows only)
                acc0 += out[2][0] * out[2][0] + out[2][1] * out[2][1];
                acc1 += out[3][0] * out[3][0] + out[3][1] * out[3][1];
            }
            const unsigned off = (live && wr) ? ((unsigned)m * (unsigned)ld + (unsigned)c0) * 8u : OOB;
            auto st2 = [&](__amdgpu_buffer_rsrc_t rs, int k) {
                const nsu4 d = {(unsigned)__double2loint(out[k][0]), (unsigned)__double2hiint(out[k][0]),
                                (unsigned)__double2loint(out[k][1]), (unsigned)__double2hiint(out[k][1])};
                __builtin_amdgcn_raw_buffer_store_b128(d, rs, (int)off, 0, NT ? 2 : 0);
            };
            st2(bcu, 0);
            st2(bcv, 1);
            st2(bru, 2);
            st2(brv, 3);
            FWnn = FEnn; FWuv = FEuv;
            SPu = SCu; SPv = SCv;
        };
        // rows ib-2 .. ie+1 (the first two steps only fill the window; row ib-1's slope needs ib)
        const int r0 = ib - 2, r1 = ie + 1;
        if (CORR) {   // phi^n rows r0 - 1, r0 (the window's first two rows) and row r0's edge value
            const int la = min(max(r0 - 1, rlo), rhi), lb = min(max(r0, rlo), rhi);
            PH1 = *reinterpret_cast<const double2*>(A.phi + (ptrdiff_t)la * ld + lc);
            PH2 = *reinterpret_cast<const double2*>(A.phi + (ptrdiff_t)lb * ld + lc);
            if (lane == 0 || lane == 63) E2 = A.phi[(ptrdiff_t)lb * ld + ce];
        }
#pragma unroll
        for (int q = 0; q < SK; q++) {
            load(r0 + q, QU[q], QV[q], QC[q], QD[q], QP[CORR ? q : 0], QE[CORR ? q : 0]);
            asm volatile("" ::: "memory");
        }
        // (r6, A/B K1_UR6=1, CORR) 3 SK rows per iteration: the correction's phi rows rotate with period 3 (PH0 <- PH1
        // <- PH2 <- qp), so a 2-row body ends on register copies of the rows just loaded -- an s_waitcnt vmcnt(0) at the
        // loop head that drains the row pipeline every two rows; 6 rows bring every register home.  Not the default:
        // K1' measured 342-347 us with it against 338 without (same box) -- the row loop is bandwidth-bound, not
        // drain-bound
        constexpr int UR = CORR && K1_UR6 ? 3 * SK : SK;
        for (int r = r0; r <= r1; r += UR) {
#pragma unroll
            for (int q = 0; q < UR; q++) {
                // (rows past r1: computed, not stored)
                const int k = q % SK;
                step(QU[k], QV[k], QC[k], QD[k], QP[CORR ? k : 0], QE[CORR ? k : 0], r + q);
                load(r + q + SK, QU[k], QV[k], QC[k], QD[k], QP[CORR ? k : 0], QE[CORR ? k : 0]);
            }
        }
    }
    if (CORR) {
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) amm[k] = fmin(amm[k], __shfl_xor(amm[k], off, 64));
        if (lane == 0 && w < nstr)
#pragma unroll
            for (int k = 0; k < 4; k++) A.mm[4 * wid + k] = amm[k];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        acc0 += __shfl_xor(acc0, off, 64);
        acc1 += __shfl_xor(acc1, off, 64);
    }
    if (lane == 0 && w < nstr) {
        A.part[2 * wid] = acc0;
        A.part[2 * wid + 1] = acc1;
    }
}
// SK = 2 rows in flight: 176 VGPRs, 2 waves / SIMD; held to 168 (3 waves: k_rhs_s3) it spills 36 B per
// lane.  NSGPU_K1S picks the variant (A/B): 3 = k_rhs_s3, 23 / 24 = 2 waves with 3 / 4 rows in flight
template <bool NT, int SK>
__global__ __launch_bounds__(256) void k_rhs_s(RhsStreamArgs A) { rhs_s_body<NT, SK>(A); }
// (r6) K1 with the previous step's K5 folded in (CORR)
template <bool NT, int SK>
__global__ __launch_bounds__(256) void k_rhs_sc(RhsStreamArgs A) { rhs_s_body<NT, SK, false, true>(A); }
template <bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_rhs_s3(RhsStreamArgs A) {
    rhs_s_body<NT, 2>(A);
}
// (r5) uniform hy: the column tables in SGPRs -- three waves per SIMD, SK rows in flight
template <bool NT, int SK>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_rhs_su(RhsStreamArgs A) {
    rhs_s_body<NT, SK, true>(A);
}

// the ring of k_rhs_s: the slab's cells within two rows of the W / E walls (whole rows), and on
// the other rows the columns 0, 1 and [jhi, ny) -- rhs_cell<BC> per cell (ghosts, the MUSCL
// stencil's wall cases and the ApplyBoundaryConditions terms), global loads; partials (ru^2, rv^2)
// per block.  Thread k: the whole wall rows first (nfull of them, from local row fr[q]), then
// (ncol columns) x the other rows.

// ------------------------------------------------ K3 / K5 as streaming strips
// The same strip walk as k_sweep (128 loaded columns, 124 written, 2 per lane, x-neighbours
// from a 3-row register window, y-neighbours by cross-lane shuffle, rows prefetched SD ahead):
// every value is loaded once instead of ~3 times through L1/L2, and the face weights
// r = h / (h_nb + h) come from tables (the same values Div_V / GradP compute).
//   K3 (k_div_s):     rhs_phi = div(u*) / dt, + per-strip (sum, sum^2)     (FluidSolver.cpp:365-418)
//   K5 (k_correct_s): u = u* - dt dphi/dx, v = v* - dt dphi/dy, + per-strip min/max (:420-456, 512-534)
//   K7 (Poisson apply of the rectangle's BiCGStab): y = A x (LHS_phi with the NEUMANN outflow
//       ghosts, :105-163), + per-strip (sum y, sum q y)
struct CellStreamArgs {
    Geo g;
    Coef c;
    double dt;
    const double *a0, *a1, *a2;   // K3: u, v, -;  K5: phi, u*, v*;  K7: x, q (or null), -
    double *o0, *o1;              // K3: rhs_phi, -;  K5: u, v;  K7: y, -
    double* part;
    int nsj;
    RowPlan P;                    // strip rows of this launch (plan_rows)
    // K6 = K5 + the next step's Poisson guess (r4): gout = gc0 phi + gc1 h1 + gc2 h2 + gc3 h3 (the
    // phi extrapolation, k_axpby's arithmetic), h2 / h3 null when unused
    const double *h1, *h2, *h3;
    double* gout;
    double gc0, gc1, gc2, gc3;
    // (r6) a masked domain (K3 / K5, one rank): only the FC_DEEP cells -- every face interior, so the rectangle's
    // interior arithmetic -- are written and reduced; the rest (Geo::ecell) take k_div_cells / k_correct_cells
    const int32_t* fc;
};

// one face value along a line: interior r-weighted interpolation, or the wall's (q + ghost)/2
__device__ __forceinline__ double face_val(double q, double qn, bool has, double r, double ghost) {
    return has ? qn * r + q * (1 - r) : 0.5 * (q + ghost);
}

// the phi extrapolation's combination, in one order for k_axpby and K6 (bit-identical guesses)
__device__ __forceinline__ double extrap_comb(double a, double x, double b, double y, double c, const double* z,
                                              double zv, double d, const double* w, double wv) {
    double r = fma(b, y, a * x);
    if (z) r = fma(c, zv, r);
    if (w) r = fma(d, wv, r);
    return r;
}

// K5's u, v stores non-temporal (A/B: make variant DEFS=-DK5_NT=1)
#ifndef K5_NT
#define K5_NT 0
#endif
// K5's rows in flight (A/B: make variant DEFS=-DK5_SD=n)
#ifndef K5_SD
#define K5_SD 4
#endif
// K6's rows in flight (A/B: make variant DEFS=-DK6_SD=n)
#ifndef K6_SD
#define K6_SD 2
#endif
template <int K>   // 3: divergence, 5: correction, 6: correction + the next Poisson guess, 7: Poisson apply
__global__ __launch_bounds__(256) void k_cell_s(CellStreamArgs A) {
    const Geo& g = A.g;
    const Coef& c = A.c;
    const int lane = threadIdx.x & 63;
    const int nstr = A.nsj * A.P.nrun;
    const int w = __builtin_amdgcn_readfirstlane(xcd_swizzle(blockIdx.x, gridDim.x) * 4 + (int)(threadIdx.x >> 6));
    const int run = w / A.nsj;
    // the strip's partial slot: pbase + run, or (pbase < 0: K3's fixed strips) the strip-row index
    const int srow = A.P.pbase >= 0 ? A.P.pbase + run : (run < A.P.slo ? run : A.P.rb1 / A.P.L + (run - A.P.slo));
    const int wid = srow * A.nsj + (w - run * A.nsj);
    constexpr bool K5 = K == 5 || K == 6;
    constexpr int SDK = K == 6 ? K6_SD : K == 5 ? K5_SD : SD;   // rows in flight (K6 streams six planes)
    double acc[4] = {0.0, 0.0, INFINITY, INFINITY};   // K3: sum, sum^2; K5: (umin, -umax, vmin, -vmax)
    if (K5) acc[0] = acc[1] = INFINITY;
    if (w < nstr) {
        const int sj = w - run * A.nsj;
        int ib, ie;
        A.P.rows(run, ib, ie);
        const int jb = sj * SW;
        const int ny = g.ny, ld = g.ld;
        const int c0 = jb - 2 + 2 * lane, c1 = c0 + 1;
        const int lc = min(max(c0, 0), ld - 2);
        const bool v0 = c0 >= 0 && c0 < ny, v1 = c1 >= 0 && c1 < ny;
        const bool wr = lane >= 1 && lane <= 62 && c0 < ny;
        const bool o0 = wr && v0, o1 = wr && v1;
        const int k0 = min(max(c0, 0), ny - 1), k1 = min(max(c1, 0), ny - 1);
        const double hy0 = c.hy[k0], hy1 = c.hy[k1];
        const double fs0 = c.fsy[k0], fn0 = c.fny[k0], fs1 = c.fsy[k1], fn1 = c.fny[k1];
        const bool s0 = c0 > 0, n0 = c0 < ny - 1, s1 = c1 > 0, n1 = c1 < ny - 1;
        // (K7: the operator's y weights toward S / N)
        const double ps0 = K == 7 ? c.ps[k0] : 0.0, pn0c = K == 7 ? c.pn[k0] : 0.0;
        const double ps1 = K == 7 ? c.ps[k1] : 0.0, pn1c = K == 7 ? c.pn[k1] : 0.0;
        const int rlo = -HALO, rhi = g.nxl + HALO - 1;
        // window field (K3: u; K5: phi) at rows ib-1 .. ie, row fields (K3: v; K5: u*, v*) at
        // row r-1 when row r arrives (prefetch overruns clamped onto fetched rows)
        double2 W0 = {0, 0}, W1 = {0, 0}, W2 = {0, 0};
        double2 Q[SDK], X[SDK], Y[SDK];
        constexpr int SH = K == 6 ? SDK : 1;   // K6: the history planes' rows, prefetched alike
        double2 H1[SH], H2[SH], H3[SH];
        constexpr int SM = (K == 3 || K == 5) ? SDK : 1;   // (masked K3 / K5: the codes' rows)
        int2 CD[SM];
        auto load = [&](int r, double2& q, double2& x, double2& y, double2& h1, double2& h2, double2& h3, int2& cd) {
            const int lw = min(max(r, max(ib - 1, rlo)), min(ie, rhi));
            const int lr = min(max(r - 1, ib), ie - 1);
            if ((K == 3 || K == 5) && A.fc) cd = *reinterpret_cast<const int2*>(A.fc + (ptrdiff_t)lr * ld + lc);
            q = *reinterpret_cast<const double2*>(A.a0 + (ptrdiff_t)lw * ld + lc);
            if (K == 3 || (K == 7 && A.a1)) {
                x = *reinterpret_cast<const double2*>(A.a1 + (ptrdiff_t)lr * ld + lc);
            } else if (K5) {
                x = *reinterpret_cast<const double2*>(A.a1 + (ptrdiff_t)lr * ld + lc);
                y = *reinterpret_cast<const double2*>(A.a2 + (ptrdiff_t)lr * ld + lc);
            }
            if (K == 6) {
                h1 = *reinterpret_cast<const double2*>(A.h1 + (ptrdiff_t)lr * ld + lc);
                if (A.h2) h2 = *reinterpret_cast<const double2*>(A.h2 + (ptrdiff_t)lr * ld + lc);
                if (A.h3) h3 = *reinterpret_cast<const double2*>(A.h3 + (ptrdiff_t)lr * ld + lc);
            }
        };
        auto step = [&](const double2 q, const double2 x, const double2 y, const double2 h1, const double2 h2,
                        const double2 h3, const int2 cd, int r) {
            W0 = W1; W1 = W2; W2 = q;
            const int m = r - 1;
            if (m < ib || m >= ie) return;
            // (masked: the FC_DEEP cells only)
            const bool d0 = !((K == 3 || K == 5) && A.fc) || (cd.x & FC_DEEP) != 0;
            const bool d1 = !((K == 3 || K == 5) && A.fc) || (cd.y & FC_DEEP) != 0;
            const int gi = g.i0 + m;
            const bool hW = gi > 0, hE = gi < g.nx - 1;
            const double hx = c.hx[gi], fw = c.fwx[gi], fe = c.fex[gi];
            if (K == 3) {
                // Div_V: u faces along x from the window, v faces along y from the lanes
                const double2 vv = x;
                const double vs0 = lane_up1(vv.y), vn1 = lane_dn1(vv.x);
                double val[2];
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    const double uc = e ? W1.y : W1.x, uw = e ? W0.y : W0.x, ue = e ? W2.y : W2.x;
                    const double vc = e ? vv.y : vv.x, vs = e ? vv.x : vs0, vn = e ? vn1 : vv.y;
                    const double V0 = face_val(uc, uw, hW, fw, ghost_v(g, uc, 0, 0));
                    const double V1 = face_val(uc, ue, hE, fe, ghost_v(g, uc, 1, 0));
                    const double V2 = face_val(vc, vs, e ? s1 : s0, e ? fs1 : fs0, ghost_v(g, vc, 2, 1));
                    const double V3 = face_val(vc, vn, e ? n1 : n0, e ? fn1 : fn0, ghost_v(g, vc, 3, 1));
                    val[e] = ((V1 - V0) / hx + (V3 - V2) / (e ? hy1 : hy0)) / A.dt;
                }
                if (wr) {   // (an odd ny's last pair: column ny is row padding, left untouched)
                    if (v1 && d0 && d1) st_stream(A.o0 + (ptrdiff_t)m * ld + c0, make_double2(val[0], val[1]), false);
                    else {
                        if (d0) A.o0[(ptrdiff_t)m * ld + c0] = val[0];
                        if (v1 && d1) A.o0[(ptrdiff_t)m * ld + c1] = val[1];
                    }
                }
                if (o0 && d0) { acc[0] += val[0]; acc[1] += val[0] * val[0]; }
                if (o1 && d1) { acc[0] += val[1]; acc[1] += val[1] * val[1]; }
            } else if (K == 7) {
                // k_apply<0, TopoRect>'s sum in its order (W, E, S, N): pn (x_nb - x_c), 0 across a
                // wall / inlet face, (ghost - x_c) / h^2 across a NEUMANN one, ghost = 2.5 x_c -
                // 2 x_1 + 0.5 x_2 (x_1, x_2 inward: the window row, one extra row load on the side's row)
                const double xs0 = lane_up1(W1.y), xn1 = lane_dn1(W1.x);
                const double xs1 = lane_up1(W1.x), xn2 = lane_dn1(W1.y);   // columns c0 - 2, c1 + 2
                const double pw = c.pw[gi], pe = c.pe[gi], wx = 1.0 / (hx * hx);
                double2 X2 = {0.0, 0.0};   // row m + 2 (W side) or m - 2 (E side) of a NEUMANN x side
                const bool nW = !hW && g.neu[0], nE = !hE && g.neu[1];
                if (nW || nE) X2 = *reinterpret_cast<const double2*>(A.a0 + (ptrdiff_t)(nW ? m + 2 : m - 2) * ld + lc);
                double val[2];
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    const double xc = e ? W1.y : W1.x, xw = e ? W0.y : W0.x, xe = e ? W2.y : W2.x;
                    const double x2 = e ? X2.y : X2.x;
                    const double xs = e ? W1.x : xs0, xn = e ? xn1 : W1.y;
                    const double xss = e ? xs0 : xs1, xnn = e ? xn2 : xn1;
                    const double hyc = e ? hy1 : hy0, wy = 1.0 / (hyc * hyc);
                    double sm = 0.0;
                    sm += hW ? pw * (xw - xc) : (g.neu[0] ? (2.5 * xc - 2.0 * xe + 0.5 * x2 - xc) * wx : 0.0);
                    sm += hE ? pe * (xe - xc) : (g.neu[1] ? (2.5 * xc - 2.0 * xw + 0.5 * x2 - xc) * wx : 0.0);
                    sm += (e ? s1 : s0) ? (e ? ps1 : ps0) * (xs - xc) : (g.neu[2] ? (2.5 * xc - 2.0 * xn + 0.5 * xnn - xc) * wy : 0.0);
                    sm += (e ? n1 : n0) ? (e ? pn1c : pn0c) * (xn - xc) : (g.neu[3] ? (2.5 * xc - 2.0 * xs + 0.5 * xss - xc) * wy : 0.0);
                    val[e] = sm;
                }
                if (wr) {
                    if (v1) st_stream(A.o0 + (ptrdiff_t)m * ld + c0, make_double2(val[0], val[1]), false);
                    else A.o0[(ptrdiff_t)m * ld + c0] = val[0];
                }
                const double q0 = A.a1 ? x.x : 0.0, q1 = A.a1 ? x.y : 0.0;
                if (o0) { acc[0] += val[0]; acc[1] += q0 * val[0]; }
                if (o1) { acc[0] += val[1]; acc[1] += q1 * val[1]; }
            } else {
                // GradP (phi ghost = phi at wall / inlet faces: 0.5 (p + p); a NEUMANN side's
                // extrapolated ghost goes through k_correct) and the correction
                const double ps0 = lane_up1(W1.y), pn1 = lane_dn1(W1.x);
                double un[2], vn[2];
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    const double pc = e ? W1.y : W1.x, pw = e ? W0.y : W0.x, pe = e ? W2.y : W2.x;
                    const double ps = e ? W1.x : ps0, pn = e ? pn1 : W1.y;
                    // (r6: corr1, the expression K1's deferred correction shares)
                    corr1(e ? x.y : x.x, e ? y.y : y.x, pc, pw, pe, ps, pn, hW, hE, e ? s1 : s0, e ? n1 : n0, fw, fe,
                          e ? fs1 : fs0, e ? fn1 : fn0, CORR_H(c.rhx[gi], hx), CORR_H(e ? c.rhy[k1] : c.rhy[k0], e ? hy1 : hy0),
                          A.dt, un[e], vn[e]);
                }
                if (wr && v1 && d0 && d1) {
                    st_stream(A.o0 + (ptrdiff_t)m * ld + c0, make_double2(un[0], un[1]), K5_NT);
                    st_stream(A.o1 + (ptrdiff_t)m * ld + c0, make_double2(vn[0], vn[1]), K5_NT);
                } else if (wr) {
                    if (d0) {
                        A.o0[(ptrdiff_t)m * ld + c0] = un[0];
                        A.o1[(ptrdiff_t)m * ld + c0] = vn[0];
                    }
                    if (v1 && d1) {
                        A.o0[(ptrdiff_t)m * ld + c1] = un[1];
                        A.o1[(ptrdiff_t)m * ld + c1] = vn[1];
                    }
                }
                if (K == 6) {
                    // the next step's Poisson guess from this step's phi (the window's row m) and the
                    // history rows -- extrapolate_phi's combination, which then only rotates planes
                    const double g0 = extrap_comb(A.gc0, W1.x, A.gc1, h1.x, A.gc2, A.h2, h2.x, A.gc3, A.h3, h3.x);
                    const double g1 = extrap_comb(A.gc0, W1.y, A.gc1, h1.y, A.gc2, A.h2, h2.y, A.gc3, A.h3, h3.y);
                    if (wr && v1) st_stream(A.gout + (ptrdiff_t)m * ld + c0, make_double2(g0, g1), false);
                    else if (wr) A.gout[(ptrdiff_t)m * ld + c0] = g0;
                }
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    if (!(e ? o1 && d1 : o0 && d0)) continue;
                    // NaN-propagating min so a blown-up step is visible in the stats
                    acc[0] = fmin(acc[0], un[e] != un[e] ? -INFINITY : un[e]);
                    acc[1] = fmin(acc[1], un[e] != un[e] ? -INFINITY : -un[e]);
                    acc[2] = fmin(acc[2], vn[e] != vn[e] ? -INFINITY : vn[e]);
                    acc[3] = fmin(acc[3], vn[e] != vn[e] ? -INFINITY : -vn[e]);
                }
            }
        };
        const int r0 = ib - 1, r1 = ie;
#pragma unroll
        for (int q = 0; q < SDK; q++) load(r0 + q, Q[q], X[q], Y[q], H1[q % SH], H2[q % SH], H3[q % SH], CD[q % SM]);
        for (int r = r0; r <= r1; r += SDK) {
#pragma unroll
            for (int q = 0; q < SDK; q++) {
                if (r + q <= r1) step(Q[q], X[q], Y[q], H1[q % SH], H2[q % SH], H3[q % SH], CD[q % SM], r + q);
                load(r + q + SDK, Q[q], X[q], Y[q], H1[q % SH], H2[q % SH], H3[q % SH], CD[q % SM]);
            }
        }
    }
    constexpr int NV = K5 ? 4 : 2;
#pragma unroll
    for (int k = 0; k < NV; k++)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const double o = __shfl_xor(acc[k], off, 64);
            acc[k] = K5 ? fmin(acc[k], o) : acc[k] + o;
        }
    if (lane == 0 && w < nstr)
#pragma unroll
        for (int k = 0; k < NV; k++) A.part[NV * wid + k] = acc[k];
}

// ------------------------------------------------ K2 / K4: two sweeps per HBM pass
// Temporal blocking of k_sweep<RB>: the row pipeline carries four stages -- red of
// sweep 1 at row r-1, black 1 at r-2, red 2 at r-3, black 2 at r-4 -- so one read of
// phi and b and one write of phi give two full red-black sweeps.  The dependency cone
// widens by one cell per half-sweep, so strips overlap by 4 columns on each side
// (128 loaded, 120 written) and read rows ib-4 .. ie+3.  Every value is computed with
// the same arithmetic as two k_sweep launches (bit-identical).
//
// RES: a fifth stage at row r-5 takes the residual of the finished values (partials of
// r^2 per strip: the solver's convergence check sees the pass's OUTPUT, not its input).
// The cone grows by one more cell: rows ib-5 .. ie+4, 116 written columns, and the
// black-2 stage also runs (unstored) on rows ib-1 and ie.
// FUSE_R (the last pre-smoothing pass of a V-cycle): the same fifth stage, and the
// residual restricted (k_restrict's area-weighted 2 x 2 sum, same order) into the coarse
// rhs, so the restriction costs no HBM pass of its own.
// FUSE_P (the first post-smoothing pass): every phi row entering the pipeline gets the
// bilinear prolongation of the coarse correction added (k_prolong's formula): coarse
// rows I = r/2 and its neighbour row are loaded with the row, coarse columns J +- 1
// come from the adjacent lanes (the outermost lanes' missing neighbours fall outside
// the written cone of the same 116-column layout).
constexpr int SW2 = 120;
// Helmholtz wall bands (k_helm_band): tile size and rows per thread (A/B: make variant DEFS="-DBAND_BT=52 -DBAND_SEG=8")
#ifndef BAND_BT
#define BAND_BT 32
#endif
#ifndef BAND_SEG
#define BAND_SEG 4
#endif
constexpr int BT = BAND_BT;
constexpr int SW2X = 116;
// rows in flight per wave (prefetch depth) per pass type: each row costs 8 VGPRs (phi, b);
// the Helmholtz pass (136 VGPRs at 3 rows) and FUSE_P (154) stay at 3 waves/SIMD up to 168
// VGPRs, FUSE_R (164) does not
#ifndef SD2_HELM
#define SD2_HELM 3
#endif
#ifndef SD2_HELMR
#define SD2_HELMR SD2_HELM
#endif
#ifndef SD2_PLAIN
#define SD2_PLAIN 3
#endif
#ifndef SD2_FP
#define SD2_FP 4   // (3: 97.4-98.4 us per 4096^2 FUSE_P pass, 4: 95.2-95.8, interleaved A/B)
#endif
#ifndef SD2_FPR
#define SD2_FPR 2
#endif
#ifndef SD2_GIN
#define SD2_GIN 2   // FUSE_R with the guess input (GIN): rows in flight
#endif
template <int OP, bool RES, int FUSE>
constexpr int sd2_of() {
    // (FUSE_P with the output residual: 172 VGPRs at 3 rows in flight = 2 waves/SIMD, 147 us per
    // pass at 4096^2 against 98 without it; 2 rows keep 3 waves)
    return FUSE == 1 ? 3 : FUSE == 2 ? (RES ? SD2_FPR : SD2_FP) : OP == 1 ? (RES ? SD2_HELMR : SD2_HELM) : SD2_PLAIN;
}
// FUSE_UV: no transfer fused; two fields (the multi-rank Helmholtz pair pass, u and v) in one launch
constexpr int FUSE_NONE = 0, FUSE_R = 1, FUSE_P = 2, FUSE_UV = 3;

// Strips of a workgroup (k_sweep2 / k_sweep3).  WG2X2 = 0: the four waves take four strips side
// by side (w = 4 t + wave).  WG2X2 = 1: a 2 x 2 block -- strip rows 2k, 2k+1 and strip columns
// 2m, 2m+1.  Strip row 2k walks down and 2k+1 up (sweep2_body), so the 5-6 halo rows the two
// share are read by both at the END of their walks; in different workgroups their progress drifts
// apart over the pass and the second read misses L2, in one workgroup (one CU) they read them
// together.  The start-of-walk halos (2k+1 / 2k+2) are read at the kernel's start by workgroups
// launched together.  Returns whether the wave has a strip; FUSE_UV: the second field's
// workgroups (or waves) switch `af` to in2 / out2 / b2 / part2.
#ifndef WG2X2
#define WG2X2 1
#endif
template <bool UV>
__device__ __forceinline__ bool strip_of(const StreamArgs& a, StreamArgs& af, int& run, int& sj) {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int t = xcd_swizzle(blockIdx.x, gridDim.x);
    if (WG2X2) {
        const int h = (a.nsj + 1) >> 1, nt = h * ((a.nrun + 1) >> 1);
        if (UV && t >= nt) {
            t -= nt;
            af.in = a.in2; af.out = a.out2; af.b = a.b2; af.part = a.part2;
        }
        const int tr = t / h, tj = t - tr * h;
        run = 2 * tr + (wv >> 1);
        sj = 2 * tj + (wv & 1);
        return run < a.nrun && sj < a.nsj;
    }
    const int nstr = a.nsj * a.nrun;
    int w = t * 4 + wv;
    if (UV && w >= nstr) {
        w -= nstr;
        af.in = a.in2; af.out = a.out2; af.b = a.b2; af.part = a.part2;
    }
    run = w / a.nsj;
    sj = w - run * a.nsj;
    return w < nstr;
}
#ifndef XR_BUF
#define XR_BUF 0   // FUSE_R's coarse stores through buffers too (1: 172 VGPRs, 2 waves/SIMD, slower)
#endif
#ifndef XR_UP
#define XR_UP 0    // FUSE_R's odd strips walk upwards too (A/B builds)
#endif
#ifndef XR_BF
#define XR_BF 0    // FUSE_R with the branch-free row loop (A/B builds)
#endif

// BF_STAGE: the pipeline stages of k_sweep2 / k_sweep3 relax every row they see -- a row outside a
// stage's range [lo, hi] is read by no row inside the next stage's range (each range is the
// previous one shrunk by a row; the stores and the residual stage take only the strip's rows) --
// and keep ghost rows / columns outside the domain by selects: no branch in a stage but the
// row colour's (wave-uniform).  Bit-identical to the guarded stages (relax rounds alike in every
// instantiation: explicit fmas)
#ifndef BF_STAGE
#define BF_STAGE 1
#endif
// a value the compiler must materialise here: a select on it stays a v_cndmask instead of
// becoming a branch around the value's computation
__device__ __forceinline__ double keep(double x) {
    asm volatile("" : "+v"(x));
    return x;
}

// UNI: a strip whose staged rows (its own and its read cone) all share one row sum -- every strip
// of a uniform grid but those within a cone of the top / bottom wall -- takes each lane's diagonal
// and omega / diagonal of its two columns from registers formed once per strip, instead of per
// stage (1 add, 1 fma, rcp + 4 fma, 1 mul).  Same expressions, so bit-identical results.
#ifndef DIAGC
#define DIAGC 1
#endif
struct DiagC {
    double d0, d1, w0, w1;
    double cw, ce, hx;   // the shared row coefficients (no LDS read per stage either)
};
template <int OP>
__device__ __forceinline__ DiagC diag_cache(const double* rm, double cd0, double cd1, double alpha, double omega) {
    DiagC c;
    const double rdc = rm[2];
    c.cw = rm[0];
    c.ce = rm[1];
    c.hx = rm[3];
    c.d0 = diag<OP>(rdc, cd0, alpha);
    c.d1 = diag<OP>(rdc, cd1, alpha);
    c.w0 = omega * rcp_nr(c.d0);
    c.w1 = omega * rcp_nr(c.d1);
    return c;
}
// the diagonal and omega / diagonal of one column of a row (row sum rd, column sum cd)
template <int OP, bool UNI>
__device__ __forceinline__ void diag_w(const DiagC& c, int col, double rd, double cd, double alpha, double omega,
                                       double& d, double& w) {
    if (UNI) {
        d = col ? c.d1 : c.d0;
        w = col ? c.w1 : c.w0;
    } else {
        d = diag<OP>(rd, cd, alpha);
        w = omega * rcp_nr(d);
    }
}
// whether every staged row of this wave's table (n rows) has the coefficients (weights, row sum,
// spacing) of row `mid` (UNI)
__device__ __forceinline__ bool rows_uniform(const double (*rc)[4], int n, int mid, int lane) {
    if (!DIAGC) return false;
    bool ok = true;
    for (int t = lane; t < n; t += 64)
        ok = ok && rc[t][0] == rc[mid][0] && rc[t][1] == rc[mid][1] && rc[t][2] == rc[mid][2] && rc[t][3] == rc[mid][3];
    return __builtin_amdgcn_ballot_w64(!ok) == 0;
}

// one strip of k_sweep2, walked downwards (DIR = 1) or upwards (DIR = -1); returns the
// strip's residual partial (R5)
// (two instantiations: runtime window selects would cost ~50 VGPRs)
// ZIN (FUSE_R only): the input iterate is identically zero -- a coarse level's first pass of a
// V-cycle, whose phi the restriction above no longer stores as zeros: no phi read at all (the
// same values as reading the zeros)
template <int OP, bool RES, int FUSE, int DIR, bool ZIN = false, bool UNI = false, bool GIN = false>
__device__ __forceinline__ double sweep2_strip(const StreamArgs& a, const double (*rc)[4], int ib, int ie, int sj,
                                              int lane) {
    constexpr int SD2 = GIN ? SD2_GIN : sd2_of<OP, RES, FUSE>();
    constexpr bool XR = FUSE == FUSE_R, XP = FUSE == FUSE_P;
    constexpr bool R5 = RES || XR;
    // the residual stage needs one more finished row on each side (EXT: rows), the prolongation's
    // coarse column neighbours one more column (EXTC: the written width)
    constexpr int EXT = R5 ? 1 : 0, EXTC = (R5 || XP) ? 1 : 0;
    constexpr int SWc = EXTC ? SW2X : SW2;
    // BF: the branch-free row loop (buffer stores, no tail guard; Helmholtz 95 -> 88 us, FUSE_P
    // 107 -> 104 us at 4096^2).  FUSE_R keeps plain stores: its deeper pipeline needed 172 VGPRs
    // (2 waves/SIMD, 112 -> 160 us), and at 3 waves it spilled and still lost 3 us
    constexpr bool BF = !XR || XR_BF;
    double res = 0.0;
    const int jb = sj * SWc;
    const int ny = a.ny, ld = a.ld;
    const int c0 = jb - 4 - 2 * EXTC + 2 * lane, c1 = c0 + 1;
    const int lc = min(max(c0, 0), ld - 2);
    const bool v0 = c0 >= 0 && c0 < ny, v1 = c1 >= 0 && c1 < ny;
    const bool wr = lane >= 2 + EXTC && lane <= 61 - EXTC && c0 < ny;
    const bool o0 = wr && v0, o1 = wr && v1;
    const int k0 = min(max(c0, 0), ny - 1), k1 = min(max(c1, 0), ny - 1);
    const double cs0 = a.cs[k0], cn0 = a.cn[k0], cd0 = cs0 + cn0 + (OP == 1 ? a.by[k0] : 0.0);
    const double cs1 = a.cs[k1], cn1 = a.cn[k1], cd1 = cs1 + cn1 + (OP == 1 ? a.by[k1] : 0.0);
    const double shift = (OP == 0 && a.shift) ? a.shift[0] : 0.0;
    const double alpha = a.alpha, omega = a.omega;
    const int rlo = -HALO, rhi = a.nxl + HALO - 1;

    // stores go through buffer resources based at this strip's first rows (wave-uniform,
    // 32-bit offsets): a lane / row that must not write gets an out-of-range offset, so the
    // row loop has no memory operation inside a branch (k_jacobi_s explains why that matters)
    const int rb = __builtin_amdgcn_readfirstlane(ib - 1 - EXT);
    const __amdgpu_buffer_rsrc_t out = __builtin_amdgcn_make_buffer_rsrc(
        a.out + (ptrdiff_t)rb * ld, (short)0, (int)((unsigned)(a.L + 2 * EXT + 2) * ld * 8u), 0x00020000);
    const int rbc = __builtin_amdgcn_readfirstlane(ib >> 1);
    const __amdgpu_buffer_rsrc_t bco = __builtin_amdgcn_make_buffer_rsrc(
        XR ? a.bc + (ptrdiff_t)rbc * a.ldc : a.out, (short)0, XR ? (int)((unsigned)((a.L >> 1) + 2) * a.ldc * 8u) : 0,
        0x00020000);
    const __amdgpu_buffer_rsrc_t pco = __builtin_amdgcn_make_buffer_rsrc(
        XR ? a.pc + (ptrdiff_t)rbc * a.ldc : a.out, (short)0, XR ? (int)((unsigned)((a.L >> 1) + 2) * a.ldc * 8u) : 0,
        0x00020000);
    double2 Q[SD2], QB[SD2];
    double QE[SD2];
    constexpr int SG = GIN ? SD2 : 1;   // GIN: the history planes' rows, prefetched alike
    double2 G1[SG], G2[SG], G3[SG];
    // phi rows ib-4-EXT .. ie+3+EXT and b rows ib-3-EXT .. ie+2+EXT (the first red
    // stage's) are read; the rest are clamped onto fetched rows (see k_sweep)
    const int r0 = ib - 4 - EXT, r1 = ie + 3 + EXT;
    // DIR < 0 walks the strip upwards: the prefetch overrun and the rows before the first
    // red stage's are then at the other end
    const int phi_lo = DIR > 0 ? rlo : max(r0, rlo), phi_hi = DIR > 0 ? min(r1, rhi) : rhi;
    const int b_lo = DIR > 0 ? max(ib - 3 - EXT, rlo) : rlo, b_hi = DIR > 0 ? rhi : min(ie + 2 + EXT, rhi);
    // FUSE_P: this lane's coarse column (its pair c0, c1 = 2J, 2J+1) and whether J -+ 1
    // exist (a missing one is replaced by J: the wall reflection of k_prolong)
    const int Jc = c0 >> 1;
    const int Jl = XP ? min(max(Jc, 0), a.ncy - 1) : 0;
    const bool jm_ok = Jc - 1 >= 0, jp_ok = Jc + 1 < a.ncy;
    // FUSE_P: fine row r needs coarse rows I = r >> 1 and its neighbour In (I + 1 for odd r, I - 1
    // for even r, I at a wall).  Along the walk consecutive rows share one of them, so a row
    // loads only In and takes I from the previous row's pair (`ep`): one coarse load per row
    // instead of two, each coarse row fetched about once per strip
    auto nbr = [&](int lp) {
        const int I = lp >> 1;                      // floor, also for ghost rows
        const int In = (lp & 1) ? I + 1 : I - 1;
        return (a.ci0 + In < 0 || a.ci0 + In >= a.ncx) ? I : In;
    };
    auto load = [&](int slot_r, double2& p, double2& bb, double& ee, double2& g1, double2& g2, double2& g3) {
        const int lp = min(max(slot_r, phi_lo), phi_hi), lb = min(max(slot_r - DIR, b_lo), b_hi);
        p = ZIN ? make_double2(0.0, 0.0) : ld_stream(a.in + (ptrdiff_t)lp * ld + lc, XP ? 1 : 0);   // (no branch)
        bb = *reinterpret_cast<const double2*>(a.b + (ptrdiff_t)lb * ld + lc);
        if (XP) ee = a.ec[(ptrdiff_t)nbr(lp) * a.ldc + Jl];
        if (GIN) {
            g1 = *reinterpret_cast<const double2*>(a.gh1 + (ptrdiff_t)lp * ld + lc);
            if (a.gh2) g2 = *reinterpret_cast<const double2*>(a.gh2 + (ptrdiff_t)lp * ld + lc);
            if (a.gh3) g3 = *reinterpret_cast<const double2*>(a.gh3 + (ptrdiff_t)lp * ld + lc);
        }
    };
    // windows (3 rows each) of the stages' inputs, rhs rows r-1 .. r-5
    double2 P0 = {0, 0}, P1 = {0, 0}, P2 = {0, 0};     // old:           rows r-2 .. r
    double2 A0 = {0, 0}, A1 = {0, 0}, A2 = {0, 0};     // after red 1:   rows r-3 .. r-1
    double2 C0 = {0, 0}, C1 = {0, 0}, C2 = {0, 0};     // after black 1: rows r-4 .. r-2
    double2 E0 = {0, 0}, E1 = {0, 0}, E2 = {0, 0};     // after red 2:   rows r-5 .. r-3
    double2 F0 = {0, 0}, F1 = {0, 0}, F2 = {0, 0};     // after black 2: rows r-6 .. r-4 (XR)
    double2 B1 = {0, 0}, B2 = {0, 0}, B3 = {0, 0}, B4 = {0, 0}, B5 = {0, 0};
    // XR: this lane's column spacings, the even row's partial sum and spacing
    const double hy0 = XR ? a.hy[k0] : 0.0, hy1 = XR ? a.hy[k1] : 0.0;
    double xs = 0.0, hxe = 0.0, ro0 = 0.0, ro1 = 0.0, hxo = 0.0;
    const DiagC dcc = UNI ? diag_cache<OP>(rc[RC_OFF + ((ie - ib) >> 1)], cd0, cd1, alpha, omega) : DiagC{};

    // one colour update of row `row` (window W0 above, W1 the row, W2 below); colour
    // parity: update c0 when (gi + c0) % 2 == par
    auto half = [&](const double2& W0, const double2& W1, const double2& W2, const double2& B, int row,
                    int par) -> double2 {
        double2 o = W1;
        const int gi = a.i0 + row;
        if (!BF_STAGE && (gi < 0 || gi >= a.nx)) return o;
        const double* rw = rc[BF_STAGE ? min(max(row - ib + RC_OFF, 0), RC_MAX - 1) : row - ib + RC_OFF];
        const double cw = UNI ? dcc.cw : rw[0], ce = UNI ? dcc.ce : rw[1];
        double rr;
        // BF_STAGE: a ghost row or a column outside the domain keeps its value through a select
        const bool in = !BF_STAGE || (gi >= 0 && gi < a.nx);
        // the row's colour is in one of the lane's two columns (wave-uniform): only that
        // column's diagonal, reciprocal and j-neighbour shuffle are formed
        if ((gi & 1) == par) {
            const double lf = lane_up1(W1.y);
            double d, w;
            diag_w<OP, UNI>(dcc, 0, rw[2], cd0, alpha, omega, d, w);
            if (BF_STAGE) {
                const double n = keep(relax<OP>(W1.x, W0.x, W2.x, lf, W1.y, B.x, cw, ce, cs0, cn0, d, w, alpha, rr));
                o.x = (in && v0) ? n : W1.x;
            } else if (v0) o.x = relax<OP>(W1.x, W0.x, W2.x, lf, W1.y, B.x, cw, ce, cs0, cn0, d, w, alpha, rr);
        } else {
            const double rt = lane_dn1(W1.x);
            double d, w;
            diag_w<OP, UNI>(dcc, 1, rw[2], cd1, alpha, omega, d, w);
            if (BF_STAGE) {
                const double n = keep(relax<OP>(W1.y, W0.y, W2.y, W1.x, rt, B.y, cw, ce, cs1, cn1, d, w, alpha, rr));
                o.y = (in && v1) ? n : W1.y;
            } else if (v1) o.y = relax<OP>(W1.y, W0.y, W2.y, W1.x, rt, B.y, cw, ce, cs1, cn1, d, w, alpha, rr);
        }
        return o;
    };

    double2 ep = {0, 0};   // FUSE_P: (e(I), e(In)) of the previous row of the walk
    auto step = [&](double2 p, const double2 bb, const double ce, const double2 g1, const double2 g2,
                    const double2 g3, int r) {
        if (GIN) {
            // the Poisson guess of this row: extrapolate_phi's combination (k_axpby, bit-identical)
            p.x = extrap_comb(a.gc0, p.x, a.gc1, g1.x, a.gc2, a.gh2, g2.x, a.gc3, a.gh3, g3.x);
            p.y = extrap_comb(a.gc0, p.y, a.gc1, g1.y, a.gc2, a.gh2, g2.y, a.gc3, a.gh3, g3.y);
        }
        if (XP) {
            // rows with a new neighbour row (odd r walking down, even r walking up) take it from
            // the load; the others reuse the previous row's two coarse rows, swapped
            // (at a wall the neighbour is I itself: k_prolong's reflection)
            const bool fresh = ((r & 1) != 0) == (DIR > 0), wall = nbr(r) == (r >> 1);
            const double2 ee = fresh ? make_double2(ep.x, ce) : make_double2(ep.y, wall ? ep.y : ep.x);
            ep = ee;
            // a side with face Dirichlet data (the outflow preconditioner) extends e oddly
            // (0 on the face) instead of reflecting it; rows outside the domain keep their
            // ghost data
            const double ey = (wall && (a.dsx & ((r & 1) ? 2 : 1))) ? -ee.y : ee.y;
            // phi += P(e): e(I, J) = ee.x, e(In, J) = ey, column neighbours from lanes -+ 1
            double m0 = lane_up1(ee.x), m1 = lane_up1(ey);
            double q0 = lane_dn1(ee.x), q1 = lane_dn1(ey);
            if (!jm_ok) { m0 = ee.x; m1 = ey; }
            if (!jp_ok) { q0 = ee.x; q1 = ey; }
            if (a.i0 + r >= 0 && a.i0 + r < a.nx) {
                p.x += (9.0 * ee.x + 3.0 * ey + 3.0 * m0 + m1) * 0.0625;
                p.y += (9.0 * ee.x + 3.0 * ey + 3.0 * q0 + q1) * 0.0625;
            }
        }
        P0 = P1; P1 = P2; P2 = (XP || !BF) ? p : vcopy(p);   // (XP: p is already a new value)
        B5 = B4; B4 = B3; B3 = B2; B2 = B1;
        B1 = make_double2(bb.x - shift, bb.y - shift);
        // stage 1: red of sweep 1 at m = r-1
        // (windows run oldest -> newest; half() wants rows i-1, i, i+1: swapped when DIR < 0)
        const int m = r - DIR;
        double2 n1 = P1;
        if (BF_STAGE || (m >= ib - 3 - EXT && m <= ie + 2 + EXT)) n1 = DIR > 0 ? half(P0, P1, P2, B1, m, 0) : half(P2, P1, P0, B1, m, 0);
        A0 = A1; A1 = A2; A2 = n1;
        // stage 2: black of sweep 1 at r-2
        double2 n2 = A1;
        const int m2 = r - 2 * DIR;
        if (BF_STAGE || (m2 >= ib - 2 - EXT && m2 <= ie + 1 + EXT)) n2 = DIR > 0 ? half(A0, A1, A2, B2, m2, 1) : half(A2, A1, A0, B2, m2, 1);
        C0 = C1; C1 = C2; C2 = n2;
        // stage 3: red of sweep 2 at r-3
        double2 n3 = C1;
        const int m3 = r - 3 * DIR;
        if (BF_STAGE || (m3 >= ib - 1 - EXT && m3 <= ie + EXT)) n3 = DIR > 0 ? half(C0, C1, C2, B3, m3, 0) : half(C2, C1, C0, B3, m3, 0);
        E0 = E1; E1 = E2; E2 = n3;
        // stage 4: black of sweep 2 at r-4, stored on the strip's rows
        const int k = r - 4 * DIR;
        double2 n4 = E1;
        if (!BF) {
            if (k >= ib - EXT && k < ie + EXT) {
                n4 = DIR > 0 ? half(E0, E1, E2, B4, k, 1) : half(E2, E1, E0, B4, k, 1);
                if (k >= ib && k < ie && wr) st_stream(a.out + (ptrdiff_t)k * ld + c0, n4, a.nt);
            }
        } else {
            if (BF_STAGE || (k >= ib - EXT && k < ie + EXT)) n4 = DIR > 0 ? half(E0, E1, E2, B4, k, 1) : half(E2, E1, E0, B4, k, 1);
            const unsigned off = (k >= ib && k < ie && wr) ? ((unsigned)(k - rb) * (unsigned)ld + (unsigned)c0) * 8u : OOB;
            const nsu4 d = {(unsigned)__double2loint(n4.x), (unsigned)__double2hiint(n4.x),
                            (unsigned)__double2loint(n4.y), (unsigned)__double2hiint(n4.y)};
            __builtin_amdgcn_raw_buffer_store_b128(d, out, (int)off, 0, 2);
        }
        unsigned coff = OOB;   // XR: the coarse cell this step completes (else dropped)
        double cval = 0.0;
        if (R5) {
            // stage 5: residual of the finished row r-5 (FUSE_R: restricted in row pairs)
            F0 = F1; F1 = F2; F2 = n4;
            const int m5 = r - 5 * DIR;
            const double2 Fm = DIR > 0 ? F0 : F2, Fp = DIR > 0 ? F2 : F0;   // rows m5 - 1, m5 + 1
            if (m5 >= ib && m5 < ie) {
                const double lf = lane_up1(F1.y), rt = lane_dn1(F1.x);
                const double* rw = rc[m5 - ib + RC_OFF];
                const double cw = UNI ? dcc.cw : rw[0], ce = UNI ? dcc.ce : rw[1], hxr = UNI ? dcc.hx : rw[3];
                const double d0 = UNI ? dcc.d0 : diag<OP>(rw[2], cd0, alpha), d1 = UNI ? dcc.d1 : diag<OP>(rw[2], cd1, alpha);
                double r0, r1;
                relax<OP>(F1.x, Fm.x, Fp.x, lf, F1.y, B5.x, cw, ce, cs0, cn0, d0, 0.0, alpha, r0);
                relax<OP>(F1.y, Fm.y, Fp.y, F1.x, rt, B5.y, cw, ce, cs1, cn1, d1, 0.0, alpha, r1);
                res += (o0 ? r0 * r0 : 0.0) + (o1 ? r1 * r1 : 0.0);
                if (!XR) {
                } else if (DIR < 0) {
                    // upwards: the odd row of a pair arrives first; the sum keeps k_restrict's
                    // order (even row, then odd row)
                    if ((a.i0 + m5) & 1) {
                        ro0 = r0; ro1 = r1; hxo = hxr;
                    } else {
                        xs = (hxr * hy0) * r0;
                        xs = xs + (hxr * hy1) * r1;
                        xs = xs + (hxo * hy0) * ro0;
                        xs = xs + (hxo * hy1) * ro1;
                        if (XR_BUF) {
                            if (wr) coff = ((unsigned)((m5 >> 1) - rbc) * (unsigned)a.ldc + (unsigned)(c0 >> 1)) * 8u;
                            cval = xs / ((hxr + hxo) * (hy0 + hy1));
                        } else if (wr) {
                            const ptrdiff_t o = (ptrdiff_t)(m5 >> 1) * a.ldc + (c0 >> 1);
                            a.bc[o] = xs / ((hxr + hxo) * (hy0 + hy1));
                            if (a.pc) a.pc[o] = 0.0;   // (null: the coarse pass reads zeros implicitly)
                        }
                    }
                } else if (((a.i0 + m5) & 1) == 0) {
                    xs = (hxr * hy0) * r0;
                    xs = xs + (hxr * hy1) * r1;
                    hxe = hxr;
                } else {
                    xs = xs + (hxr * hy0) * r0;
                    xs = xs + (hxr * hy1) * r1;
                    if (XR_BUF) {
                        if (wr) coff = ((unsigned)((m5 >> 1) - rbc) * (unsigned)a.ldc + (unsigned)(c0 >> 1)) * 8u;
                        cval = xs / ((hxe + hxr) * (hy0 + hy1));
                    } else if (wr) {
                        const ptrdiff_t o = (ptrdiff_t)(m5 >> 1) * a.ldc + (c0 >> 1);
                        a.bc[o] = xs / ((hxe + hxr) * (hy0 + hy1));
                        if (a.pc) a.pc[o] = 0.0;
                    }
                }
            }
        }
        if (XR && XR_BUF) {
            __builtin_amdgcn_raw_buffer_store_b64(
                (nsu2){(unsigned)__double2loint(cval), (unsigned)__double2hiint(cval)}, bco, (int)coff, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b64((nsu2){0u, 0u}, pco, (int)coff, 0, 0);
        }
    };

    const int rs = DIR > 0 ? r0 : r1, nr = r1 - r0 + 1;
    if (XP) {   // the coarse pair of the row before the walk's first
        const int lp = rs - DIR;
        ep = make_double2(a.ec[(ptrdiff_t)(lp >> 1) * a.ldc + Jl], a.ec[(ptrdiff_t)nbr(lp) * a.ldc + Jl]);
    }
#pragma unroll
    for (int q = 0; q < SD2; q++) {
        load(rs + DIR * q, Q[q], QB[q], QE[q], G1[q % SG], G2[q % SG], G3[q % SG]);
        if (BF) asm volatile("" ::: "memory");   // keep the slots' issue order (the loop's vmcnt bookkeeping)
    }
    for (int t = 0; t < nr; t += SD2) {
#pragma unroll
        for (int q = 0; q < SD2; q++) {
            if (BF || t + q < nr)   // (BF: steps past the strip store nothing)
                step(Q[q], QB[q], QE[q], G1[q % SG], G2[q % SG], G3[q % SG], rs + DIR * (t + q));
            load(rs + DIR * (t + q + SD2), Q[q], QB[q], QE[q], G1[q % SG], G2[q % SG], G3[q % SG]);
        }
    }
    return res;
}

// ------------------------------------------------ K2: three Helmholtz sweeps per HBM pass
// The Helmholtz solve needs 7 RB-SOR sweeps per component at 4096^2 (rtol 1e-8; the pairs of
// k_sweep2 made that 8).  k_sweep3 carries six stages (red / black of sweeps 1-3) in the same
// register pipeline: 7 sweeps = 3 + 2 + 2, three HBM passes instead of four.  Helmholtz
// operator only, no residual stage (the pass is never a batch's last: helm_sweeps), strips of
// 116 written columns (a 6-column cone on each side), rows ib-6 .. ie+5 read; every value is
// the same arithmetic as three single sweeps (bit-identical).  FUSE_UV: u and v in one launch.
// RES: a seventh stage at row r-7 takes the residual of the finished values (the batch's last
// pass: its partials of r^2 per strip are the convergence check's); the cone grows by one cell:
// rows ib-7 .. ie+6, 112 written columns (SW3R), 7 ghost rows (HALO = 7: slabs too; FUSE_UV + RES is
// the multi-rank batch end, u and v in one launch, v's partials at part2)
constexpr int SW3R = SW2X - 4;

template <int DIR, bool RES, int SD3, bool UNI = false>
__device__ __forceinline__ double sweep3_strip(const StreamArgs& a, const double (*rc)[4], int ib, int ie, int sj,
                                               int lane) {
    // SD3: rows in flight (round 2: 3 needed 174 VGPRs then; with the wave-uniform strip index the
    // pass takes 140-152 at 2, so 3 fits 3 waves / SIMD too: NSGPU_SD3=3, A/B)
    constexpr int EXT = RES ? 1 : 0;
    const int jb = sj * (RES ? SW3R : SW2X);
    const int ny = a.ny, ld = a.ld;
    const int c0 = jb - 6 - 2 * EXT + 2 * lane, c1 = c0 + 1;
    const int lc = min(max(c0, 0), ld - 2);
    const bool v0 = c0 >= 0 && c0 < ny, v1 = c1 >= 0 && c1 < ny;
    const bool wr = lane >= 3 + EXT && lane <= 60 - EXT && c0 < ny;
    const bool o0 = wr && v0, o1 = wr && v1;
    double res = 0.0;
    const int k0 = min(max(c0, 0), ny - 1), k1 = min(max(c1, 0), ny - 1);
    const double cs0 = a.cs[k0], cn0 = a.cn[k0], cd0 = cs0 + cn0 + a.by[k0];
    const double cs1 = a.cs[k1], cn1 = a.cn[k1], cd1 = cs1 + cn1 + a.by[k1];
    const double alpha = a.alpha, omega = a.omega;
    const int rlo = -HALO, rhi = a.nxl + HALO - 1;
    const int rb = __builtin_amdgcn_readfirstlane(ib - 1 - EXT);
    const __amdgpu_buffer_rsrc_t out = __builtin_amdgcn_make_buffer_rsrc(
        a.out + (ptrdiff_t)rb * ld, (short)0, (int)((unsigned)(a.L + 2 + 2 * EXT) * ld * 8u), 0x00020000);
    const DiagC dcc = UNI ? diag_cache<1>(rc[RC_OFF3 + ((ie - ib) >> 1)], cd0, cd1, alpha, omega) : DiagC{};
    double2 Q[SD3], QB[SD3];
    // q rows ib-6-EXT .. ie+5+EXT and b rows ib-5-EXT .. ie+4+EXT (the first red stage's) are read
    const int r0 = ib - 6 - EXT, r1 = ie + 5 + EXT;
    const int phi_lo = DIR > 0 ? rlo : max(r0, rlo), phi_hi = DIR > 0 ? min(r1, rhi) : rhi;
    const int b_lo = DIR > 0 ? max(ib - 5 - EXT, rlo) : rlo, b_hi = DIR > 0 ? rhi : min(ie + 4 + EXT, rhi);
    auto load = [&](int slot_r, double2& p, double2& bb) {
        const int lp = min(max(slot_r, phi_lo), phi_hi), lb = min(max(slot_r - DIR, b_lo), b_hi);
        p = ld_stream(a.in + (ptrdiff_t)lp * ld + lc, 0);
        bb = *reinterpret_cast<const double2*>(a.b + (ptrdiff_t)lb * ld + lc);
    };
    // windows (3 rows each) of the six stages' inputs; rhs rows r-1 .. r-6
    double2 P0 = {0, 0}, P1 = {0, 0}, P2 = {0, 0};
    double2 A0 = {0, 0}, A1 = {0, 0}, A2 = {0, 0};
    double2 C0 = {0, 0}, C1 = {0, 0}, C2 = {0, 0};
    double2 E0 = {0, 0}, E1 = {0, 0}, E2 = {0, 0};
    double2 G0 = {0, 0}, G1 = {0, 0}, G2 = {0, 0};
    double2 H0 = {0, 0}, H1 = {0, 0}, H2 = {0, 0};
    double2 F0 = {0, 0}, F1 = {0, 0}, F2 = {0, 0};   // RES: after black 3, rows r-8 .. r-6
    double2 B1 = {0, 0}, B2 = {0, 0}, B3 = {0, 0}, B4 = {0, 0}, B5 = {0, 0}, B6 = {0, 0}, B7 = {0, 0};
    auto half = [&](const double2& W0, const double2& W1, const double2& W2, const double2& B, int row,
                    int par) -> double2 {
        double2 o = W1;
        const int gi = a.i0 + row;
        if (!BF_STAGE && (gi < 0 || gi >= a.nx)) return o;
        const double* rw = rc[BF_STAGE ? min(max(row - ib + RC_OFF3, 0), RC_MAX3 - 1) : row - ib + RC_OFF3];
        const double cw = UNI ? dcc.cw : rw[0], ce = UNI ? dcc.ce : rw[1];
        double rr;
        // BF_STAGE: no branch but the colour's: a ghost row or a column outside the domain keeps
        // its value through a select (the relaxation is computed anyway)
        const bool in = !BF_STAGE || (gi >= 0 && gi < a.nx);
        if ((gi & 1) == par) {
            const double lf = lane_up1(W1.y);
            double d, w;
            diag_w<1, UNI>(dcc, 0, rw[2], cd0, alpha, omega, d, w);
            if (BF_STAGE) {
                const double n = keep(relax<1>(W1.x, W0.x, W2.x, lf, W1.y, B.x, cw, ce, cs0, cn0, d, w, alpha, rr));
                o.x = (in && v0) ? n : W1.x;
            } else if (v0) o.x = relax<1>(W1.x, W0.x, W2.x, lf, W1.y, B.x, cw, ce, cs0, cn0, d, w, alpha, rr);
        } else {
            const double rt = lane_dn1(W1.x);
            double d, w;
            diag_w<1, UNI>(dcc, 1, rw[2], cd1, alpha, omega, d, w);
            if (BF_STAGE) {
                const double n = keep(relax<1>(W1.y, W0.y, W2.y, W1.x, rt, B.y, cw, ce, cs1, cn1, d, w, alpha, rr));
                o.y = (in && v1) ? n : W1.y;
            } else if (v1) o.y = relax<1>(W1.y, W0.y, W2.y, W1.x, rt, B.y, cw, ce, cs1, cn1, d, w, alpha, rr);
        }
        return o;
    };
    // one pipeline stage: colour `par` at row m if m lies in [lo, hi] (else the value passes on).
    // BF_STAGE: every row is relaxed -- a row outside [lo, hi] is read by no row inside the next
    // stage's range (each stage's range is the previous one's shrunk by a row), and the stores
    // and the residual stage take only the strip's rows
    auto stage = [&](const double2& W0, const double2& W1, const double2& W2, const double2& B, int m, int lo,
                     int hi, int par) -> double2 {
        if (!BF_STAGE && (m < lo || m > hi)) return W1;
        return DIR > 0 ? half(W0, W1, W2, B, m, par) : half(W2, W1, W0, B, m, par);
    };
    auto step = [&](double2 p, const double2 bb, int r) {
        P0 = P1; P1 = P2; P2 = vcopy(p);
        if (RES) B7 = B6;
        B6 = B5; B5 = B4; B4 = B3; B3 = B2; B2 = B1;
        B1 = bb;
        const double2 n1 = stage(P0, P1, P2, B1, r - DIR, ib - 5 - EXT, ie + 4 + EXT, 0);       // red 1
        A0 = A1; A1 = A2; A2 = n1;
        const double2 n2 = stage(A0, A1, A2, B2, r - 2 * DIR, ib - 4 - EXT, ie + 3 + EXT, 1);   // black 1
        C0 = C1; C1 = C2; C2 = n2;
        const double2 n3 = stage(C0, C1, C2, B3, r - 3 * DIR, ib - 3 - EXT, ie + 2 + EXT, 0);   // red 2
        E0 = E1; E1 = E2; E2 = n3;
        const double2 n4 = stage(E0, E1, E2, B4, r - 4 * DIR, ib - 2 - EXT, ie + 1 + EXT, 1);   // black 2
        G0 = G1; G1 = G2; G2 = n4;
        const double2 n5 = stage(G0, G1, G2, B5, r - 5 * DIR, ib - 1 - EXT, ie + EXT, 0);       // red 3
        H0 = H1; H1 = H2; H2 = n5;
        // black 3 at r-6, stored on the strip's rows (out-of-range offset: dropped)
        const int k = r - 6 * DIR;
        const double2 n6 = stage(H0, H1, H2, B6, k, ib - EXT, ie - 1 + EXT, 1);
        const unsigned off = (k >= ib && k < ie && wr) ? ((unsigned)(k - rb) * (unsigned)ld + (unsigned)c0) * 8u : OOB;
        const nsu4 d = {(unsigned)__double2loint(n6.x), (unsigned)__double2hiint(n6.x),
                        (unsigned)__double2loint(n6.y), (unsigned)__double2hiint(n6.y)};
        __builtin_amdgcn_raw_buffer_store_b128(d, out, (int)off, 0, 2);
        if (RES) {
            // stage 7: residual of the finished row r-7 (k_sweep2's fifth stage)
            F0 = F1; F1 = F2; F2 = n6;
            const int m7 = r - 7 * DIR;
            const double2 Fm = DIR > 0 ? F0 : F2, Fp = DIR > 0 ? F2 : F0;   // rows m7 - 1, m7 + 1
            if (m7 >= ib && m7 < ie) {
                const double lf = lane_up1(F1.y), rt = lane_dn1(F1.x);
                const double* rw = rc[m7 - ib + RC_OFF3];
                const double cw = UNI ? dcc.cw : rw[0], ce = UNI ? dcc.ce : rw[1];
                const double d0 = UNI ? dcc.d0 : diag<1>(rw[2], cd0, alpha), d1 = UNI ? dcc.d1 : diag<1>(rw[2], cd1, alpha);
                double q0, q1;
                relax<1>(F1.x, Fm.x, Fp.x, lf, F1.y, B7.x, cw, ce, cs0, cn0, d0, 0.0, alpha, q0);
                relax<1>(F1.y, Fm.y, Fp.y, F1.x, rt, B7.y, cw, ce, cs1, cn1, d1, 0.0, alpha, q1);
                if (m7 >= a.sr0 && m7 < a.sr1) res += (o0 ? q0 * q0 : 0.0) + (o1 ? q1 * q1 : 0.0);
            }
        }
    };
    const int rs = DIR > 0 ? r0 : r1, nr = r1 - r0 + 1;
#pragma unroll
    for (int q = 0; q < SD3; q++) {
        load(rs + DIR * q, Q[q], QB[q]);
        asm volatile("" ::: "memory");
    }
    for (int t = 0; t < nr; t += SD3) {
#pragma unroll
        for (int q = 0; q < SD3; q++) {
            step(Q[q], QB[q], rs + DIR * (t + q));
            load(rs + DIR * (t + q + SD3), Q[q], QB[q]);
        }
    }
    return res;
}

template <int FUSE, bool RES = false, int SD3 = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SD3 == 3 ? 3 : 1))) void k_sweep3(StreamArgs a) {
    __shared__ double rcs[4][RC_MAX3][4];
    double (*rc)[4] = rcs[threadIdx.x >> 6];
    StreamArgs af = a;
    int run, sj;
    const bool live = strip_of<FUSE == FUSE_UV>(a, af, run, sj);
    const int lane = threadIdx.x & 63;
    const int ib = run < a.slo ? a.rb0 + run * a.L : a.rb1 + (run - a.slo) * a.L;
    const int ie = min(ib + a.L, a.rend);
    const int si = a.pbase + run;
    if (live) stage_rows<1, RC_OFF3, L3_MAX>(af, rc, ib, lane);
    __syncthreads();
    double res = 0.0;
    if (live) {
        const bool uni = rows_uniform(rc, min(ie - ib + 2 * RC_OFF3, RC_MAX3), RC_OFF3 + ((ie - ib) >> 1), lane);
        if (si & 1) res = uni ? sweep3_strip<-1, RES, SD3, true>(af, rc, ib, ie, sj, lane)
                              : sweep3_strip<-1, RES, SD3>(af, rc, ib, ie, sj, lane);
        else res = uni ? sweep3_strip<1, RES, SD3, true>(af, rc, ib, ie, sj, lane)
                       : sweep3_strip<1, RES, SD3>(af, rc, ib, ie, sj, lane);
    }
    if (RES) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) res += __shfl_xor(res, off, 64);
        if (lane == 0 && live) af.part[si * a.nsj + sj] = res;
    }
}

template <int OP, bool RES, int FUSE, bool ZIN = false, bool GIN = false>
__device__ __forceinline__ void sweep2_body(const StreamArgs& a) {
    constexpr bool XR = FUSE == FUSE_R;
    constexpr bool R5 = RES || XR;                 // the fifth (output residual) stage
    __shared__ double rcs[4][RC_MAX][4];
    const int lane = threadIdx.x & 63;
    double (*rc)[4] = rcs[threadIdx.x >> 6];
    // this wave's strip (plan_strips2: the launch may cover a subset of the pass's rows) and
    // field (FUSE_UV: the second field's workgroups take in2 / out2 / b2 / part2)
    StreamArgs af = a;
    int run, sj;
    const bool live = strip_of<FUSE == FUSE_UV>(a, af, run, sj);
    const int ib = run < a.slo ? a.rb0 + run * a.L : a.rb1 + (run - a.slo) * a.L;
    const int ie = min(ib + a.L, a.rend);
    const int si = a.pbase + run, wid = si * a.nsj + sj;
    if (live) stage_rows<OP>(af, rc, ib, lane);
    __syncthreads();
    double res = 0.0;
    if (live) {
        // odd strips walk upwards: the halo rows two strips share are then read by both at about
        // the same time -- an L2 hit for the second (Helmholtz pass 86.5 -> 84 us at 4096^2).
        // The restriction pass walks downwards only: upwards, its fused restriction rounds some
        // coarse sums differently, and its values would depend on how a pass is cut into strips
        // (the overlapped exchange's split, the slab height)
        const bool uni = rows_uniform(rc, min(ie - ib + 2 * RC_OFF, RC_MAX), RC_OFF + ((ie - ib) >> 1), lane);
        if ((FUSE != FUSE_R || XR_UP) && (si & 1))
            res = uni ? sweep2_strip<OP, RES, FUSE, -1, ZIN, true, GIN>(af, rc, ib, ie, sj, lane)
                      : sweep2_strip<OP, RES, FUSE, -1, ZIN, false, GIN>(af, rc, ib, ie, sj, lane);
        else
            res = uni ? sweep2_strip<OP, RES, FUSE, 1, ZIN, true, GIN>(af, rc, ib, ie, sj, lane)
                      : sweep2_strip<OP, RES, FUSE, 1, ZIN, false, GIN>(af, rc, ib, ie, sj, lane);
    }
    if (R5) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) res += __shfl_xor(res, off, 64);
        if (lane == 0 && live) af.part[wid] = res;
    }
}

template <int OP, bool RES, int FUSE, bool ZIN = false>
__global__ __launch_bounds__(256) void k_sweep2(StreamArgs a) { sweep2_body<OP, RES, FUSE, ZIN>(a); }
// the first restriction pass of a Poisson solve with the phi extrapolation formed on the fly (GIN)
__global__ __launch_bounds__(256) void k_sweep2_gin(StreamArgs a) { sweep2_body<0, false, FUSE_R, false, true>(a); }
// FP_W4 (A/B): the finest prolongation pass held to 4 waves / SIMD (128 VGPRs; with SD2_FP = 2)
#ifndef FP_W4
#define FP_W4 0
#endif
template <bool RES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_sweep2_fp4(StreamArgs a) {
    sweep2_body<0, RES, FUSE_P>(a);
}

// ------------------------------------------------ K4: a V-cycle boundary in one HBM pass (r4)
// Between two V-cycles the finest level runs FUSE_P of cycle c (prolongation + 2 RB sweeps) and
// then FUSE_R of cycle c + 1 (2 RB sweeps + residual + restriction): two passes over phi and b
// (~90 us each at 4096^2), latency-bound rather than bandwidth-bound.  When cycle c's output is not
// checked (the solver predicts the check point), k_sweep4 does both in ONE pass: the prolongation
// on each row entering the pipeline, eight stages (red / black of four sweeps), the output stored
// after the eighth and the residual of the finished rows restricted in row pairs into the coarse
// rhs -- k_sweep2<FUSE_P>'s input stage and k_sweep2<FUSE_R>'s output stages around k_sweep2's
// stages, the same arithmetic in the same order, so bit-identical to the two passes.  Walks
// downwards (FUSE_R's restriction sums must not depend on the walk); one rank / replicated levels
// only (the cone reads 9 rows beyond the strip: more than HALO; walls clamp onto ghost rows).
// Strips: 108 written columns of 128 (prolongation 1 + 8 stages + residual 1 on each side).
constexpr int SW4 = 108;
constexpr int RC_OFF4 = 9;               // table row of strip row ib: stage 1 reads rows ib-8 .. ie+7
constexpr int L4_MAX = 128;
constexpr int RC_MAX4 = L4_MAX + 2 * RC_OFF4;
#ifndef SD4
#define SD4 3                            // rows in flight (1 / 2 / 3: 179 / 140 / 129 us per pass at 4096^2)
#endif
template <bool UNI>
__device__ __forceinline__ double sweep4_strip(const StreamArgs& a, const double (*rc)[4], int ib, int ie, int sj,
                                               int lane) {
    double res = 0.0;
    const int jb = sj * SW4;
    const int ny = a.ny, ld = a.ld;
    const int c0 = jb - 10 + 2 * lane, c1 = c0 + 1;
    const int lc = min(max(c0, 0), ld - 2);
    const bool v0 = c0 >= 0 && c0 < ny, v1 = c1 >= 0 && c1 < ny;
    const bool wr = lane >= 5 && lane <= 58 && c0 < ny;
    const bool o0 = wr && v0, o1 = wr && v1;
    const int k0 = min(max(c0, 0), ny - 1), k1 = min(max(c1, 0), ny - 1);
    const double cs0 = a.cs[k0], cn0 = a.cn[k0], cd0 = cs0 + cn0;
    const double cs1 = a.cs[k1], cn1 = a.cn[k1], cd1 = cs1 + cn1;
    const double shift = a.shift ? a.shift[0] : 0.0;
    const double omega = a.omega;
    const int rlo = -HALO, rhi = a.nxl + HALO - 1;
    const int rb = __builtin_amdgcn_readfirstlane(ib);
    const __amdgpu_buffer_rsrc_t out = __builtin_amdgcn_make_buffer_rsrc(
        a.out + (ptrdiff_t)rb * ld, (short)0, (int)((unsigned)a.L * ld * 8u), 0x00020000);
    double2 Q[SD4], QB[SD4];
    double QE[SD4];
    // phi rows ib-9 .. ie+8 and b rows ib-8 .. ie+7 are read (the rest clamp onto fetched rows)
    const int r0 = ib - 9, r1 = ie + 8;
    const int phi_lo = rlo, phi_hi = min(r1, rhi);
    const int b_lo = max(ib - 8, rlo), b_hi = rhi;
    const int Jc = c0 >> 1;
    const int Jl = min(max(Jc, 0), a.ncy - 1);
    const bool jm_ok = Jc - 1 >= 0, jp_ok = Jc + 1 < a.ncy;
    auto nbr = [&](int lp) {
        const int I = lp >> 1;
        const int In = (lp & 1) ? I + 1 : I - 1;
        return (a.ci0 + In < 0 || a.ci0 + In >= a.ncx) ? I : In;
    };
    auto load = [&](int slot_r, double2& p, double2& bb, double& ee) {
        const int lp = min(max(slot_r, phi_lo), phi_hi), lb = min(max(slot_r - 1, b_lo), b_hi);
        p = ld_stream(a.in + (ptrdiff_t)lp * ld + lc, 1);
        bb = *reinterpret_cast<const double2*>(a.b + (ptrdiff_t)lb * ld + lc);
        ee = a.ec[(ptrdiff_t)nbr(lp) * a.ldc + Jl];
    };
    // windows of the nine stages' inputs (3 rows each), rhs rows r-1 .. r-9
    double2 W[9][3];
#pragma unroll
    for (int s = 0; s < 9; s++) W[s][0] = W[s][1] = W[s][2] = make_double2(0.0, 0.0);
    double2 B[9];
#pragma unroll
    for (int s = 0; s < 9; s++) B[s] = make_double2(0.0, 0.0);
    const double hy0 = a.hy[k0], hy1 = a.hy[k1];
    double xs = 0.0, hxe = 0.0;
    const DiagC dcc = UNI ? diag_cache<0>(rc[RC_OFF4 + ((ie - ib) >> 1)], cd0, cd1, 0.0, omega) : DiagC{};
    auto half = [&](const double2& W0, const double2& W1, const double2& W2, const double2& Bv, int row,
                    int par) -> double2 {
        double2 o = W1;
        const int gi = a.i0 + row;
        const double* rw = rc[min(max(row - ib + RC_OFF4, 0), RC_MAX4 - 1)];
        const double cw = UNI ? dcc.cw : rw[0], ce = UNI ? dcc.ce : rw[1];
        double rr;
        const bool in = gi >= 0 && gi < a.nx;
        if ((gi & 1) == par) {
            const double lf = lane_up1(W1.y);
            double d, w;
            diag_w<0, UNI>(dcc, 0, rw[2], cd0, 0.0, omega, d, w);
            const double n = keep(relax<0>(W1.x, W0.x, W2.x, lf, W1.y, Bv.x, cw, ce, cs0, cn0, d, w, 0.0, rr));
            o.x = (in && v0) ? n : W1.x;
        } else {
            const double rt = lane_dn1(W1.x);
            double d, w;
            diag_w<0, UNI>(dcc, 1, rw[2], cd1, 0.0, omega, d, w);
            const double n = keep(relax<0>(W1.y, W0.y, W2.y, W1.x, rt, Bv.y, cw, ce, cs1, cn1, d, w, 0.0, rr));
            o.y = (in && v1) ? n : W1.y;
        }
        return o;
    };
    double2 ep = {0, 0};   // (e(I), e(In)) of the previous row of the walk (k_sweep2<FUSE_P>)
    auto step = [&](double2 p, const double2 bb, const double ce, int r) {
        {
            // phi += P(e) on the entering row (k_sweep2<FUSE_P>'s input stage, walking down)
            const bool fresh = (r & 1) != 0, wall = nbr(r) == (r >> 1);
            const double2 ee = fresh ? make_double2(ep.x, ce) : make_double2(ep.y, wall ? ep.y : ep.x);
            ep = ee;
            const double ey = (wall && (a.dsx & ((r & 1) ? 2 : 1))) ? -ee.y : ee.y;
            double m0 = lane_up1(ee.x), m1 = lane_up1(ey);
            double q0 = lane_dn1(ee.x), q1 = lane_dn1(ey);
            if (!jm_ok) { m0 = ee.x; m1 = ey; }
            if (!jp_ok) { q0 = ee.x; q1 = ey; }
            if (a.i0 + r >= 0 && a.i0 + r < a.nx) {
                p.x += (9.0 * ee.x + 3.0 * ey + 3.0 * m0 + m1) * 0.0625;
                p.y += (9.0 * ee.x + 3.0 * ey + 3.0 * q0 + q1) * 0.0625;
            }
        }
#pragma unroll
        for (int s = 8; s > 0; s--) B[s] = B[s - 1];
        B[0] = make_double2(bb.x - shift, bb.y - shift);
        W[0][0] = W[0][1]; W[0][1] = W[0][2]; W[0][2] = p;
        // stages 1 .. 8 at rows r-1 .. r-8 (red, black, ...): stage s reads window s-1, writes window s
#pragma unroll
        for (int s = 1; s <= 8; s++) {
            const double2 n = half(W[s - 1][0], W[s - 1][1], W[s - 1][2], B[s - 1], r - s, (s + 1) & 1);
            W[s][0] = W[s][1]; W[s][1] = W[s][2]; W[s][2] = n;
        }
        // the eighth stage's row r-8 is the pass's output (strip rows only; else the offset drops it)
        const int k = r - 8;
        const double2 n8 = W[8][2];
        const unsigned off = (k >= ib && k < ie && wr) ? ((unsigned)(k - rb) * (unsigned)ld + (unsigned)c0) * 8u : OOB;
        const nsu4 d = {(unsigned)__double2loint(n8.x), (unsigned)__double2hiint(n8.x),
                        (unsigned)__double2loint(n8.y), (unsigned)__double2hiint(n8.y)};
        __builtin_amdgcn_raw_buffer_store_b128(d, out, (int)off, 0, 2);
        // residual of the finished row r-9, restricted in row pairs (k_sweep2<FUSE_R>'s fifth stage)
        const int m9 = r - 9;
        if (m9 >= ib && m9 < ie) {
            const double2 F1 = W[8][1], Fm = W[8][0], Fp = W[8][2];
            const double lf = lane_up1(F1.y), rt = lane_dn1(F1.x);
            const double* rw = rc[m9 - ib + RC_OFF4];
            const double cw = UNI ? dcc.cw : rw[0], ce = UNI ? dcc.ce : rw[1], hxr = UNI ? dcc.hx : rw[3];
            const double d0 = UNI ? dcc.d0 : diag<0>(rw[2], cd0, 0.0), d1 = UNI ? dcc.d1 : diag<0>(rw[2], cd1, 0.0);
            double q0, q1;
            relax<0>(F1.x, Fm.x, Fp.x, lf, F1.y, B[8].x, cw, ce, cs0, cn0, d0, 0.0, 0.0, q0);
            relax<0>(F1.y, Fm.y, Fp.y, F1.x, rt, B[8].y, cw, ce, cs1, cn1, d1, 0.0, 0.0, q1);
            res += (o0 ? q0 * q0 : 0.0) + (o1 ? q1 * q1 : 0.0);
            if (((a.i0 + m9) & 1) == 0) {
                xs = (hxr * hy0) * q0;
                xs = xs + (hxr * hy1) * q1;
                hxe = hxr;
            } else {
                xs = xs + (hxr * hy0) * q0;
                xs = xs + (hxr * hy1) * q1;
                if (wr) {
                    const ptrdiff_t o = (ptrdiff_t)(m9 >> 1) * a.ldc + (c0 >> 1);
                    a.bc[o] = xs / ((hxe + hxr) * (hy0 + hy1));
                    if (a.pc) a.pc[o] = 0.0;
                }
            }
        }
    };
    {   // the coarse pair of the row before the walk's first
        const int lp = r0 - 1;
        ep = make_double2(a.ec[(ptrdiff_t)(lp >> 1) * a.ldc + Jl], a.ec[(ptrdiff_t)nbr(lp) * a.ldc + Jl]);
    }
    const int nr = r1 - r0 + 1;
#pragma unroll
    for (int q = 0; q < SD4; q++) {
        load(r0 + q, Q[q], QB[q], QE[q]);
        asm volatile("" ::: "memory");
    }
    for (int t = 0; t < nr; t += SD4) {
#pragma unroll
        for (int q = 0; q < SD4; q++) {
            step(Q[q], QB[q], QE[q], r0 + t + q);   // (steps past the strip store nothing)
            load(r0 + t + q + SD4, Q[q], QB[q], QE[q]);
        }
    }
    return res;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_sweep4(StreamArgs a) {
    __shared__ double rcs[4][RC_MAX4][4];
    double (*rc)[4] = rcs[threadIdx.x >> 6];
    StreamArgs af = a;
    int run, sj;
    const bool live = strip_of<false>(a, af, run, sj);
    const int lane = threadIdx.x & 63;
    const int ib = run < a.slo ? a.rb0 + run * a.L : a.rb1 + (run - a.slo) * a.L;
    const int ie = min(ib + a.L, a.rend);
    const int si = a.pbase + run, wid = si * a.nsj + sj;
    if (live) stage_rows<0, RC_OFF4, L4_MAX>(af, rc, ib, lane);
    __syncthreads();
    double res = 0.0;
    if (live) {
        const bool uni = rows_uniform(rc, min(ie - ib + 2 * RC_OFF4, RC_MAX4), RC_OFF4 + ((ie - ib) >> 1), lane);
        res = uni ? sweep4_strip<true>(af, rc, ib, ie, sj, lane) : sweep4_strip<false>(af, rc, ib, ie, sj, lane);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) res += __shfl_xor(res, off, 64);
    if (lane == 0 && live && af.part) af.part[wid] = res;
}

// ------------------------------------------------ K4 small levels: LDS-tiled fused passes
// The multigrid levels below the streaming kernels' range (< 2048^2 cells: 1024^2 .. 128^2
// at 4096^2) are latency-bound: a row pipeline of L rows costs L dependent steps whatever
// the level's size.  Here one 256-thread workgroup owns a TT x TT output tile, stages phi
// and b over the tile plus the dependency cone in LDS with ONE round of loads, and runs the
// four half-sweeps of two red-black sweeps there (red, black, red, black; the updated
// region shrinks by one cell per half-sweep):
//   FUSE_R (cone 5): + the residual of the finished tile, restricted to the coarse rhs
//                    (+ coarse phi := 0) and r^2 partials -- k_sweep2<XR>'s pass;
//   FUSE_P (cone 4): every staged phi gets the bilinear prolongation of the coarse
//                    correction first -- k_sweep2<FUSE_P>'s pass.
// Same arithmetic as k_sweep2 (relax<0>, the Newton reciprocal of the diagonal, the
// restriction's summation order), so the two are interchangeable level by level.
// TT = 32, or 16 on the levels that would have fewer than 512 tiles of 32 (<= 512^2): four
// times the workgroups and a quarter of the work per half-sweep -- these levels are latency-bound,
// so the larger cone overhead costs nothing (128^2 / 256^2: 8.2 -> 5.4 us per FUSE_R pass, 512^2:
// 8.8 -> 7.6 us; at 1024^2 16 x 16 tiles measured 0.3 % slower overall, so 32 stays there)
// ZIN (FUSE_R): the input iterate is identically zero (see sweep2_strip): no phi load
template <int FUSE, int TT, bool RES = false, bool ZIN = false>
__global__ __launch_bounds__(256) void k_tile2(StreamArgs a, int tiles_j) {
    constexpr bool XR = FUSE == FUSE_R, XP = FUSE == FUSE_P;
    constexpr bool R5 = XR || RES;   // the output residual (RES: FUSE_P's, partials only)
    constexpr int R = R5 ? 5 : 4;
    constexpr int E = TT + 2 * R;
    constexpr int NQ = (E * E + 255) / 256;     // staged cells per thread
    constexpr int CE = E / 2 + 3;                // XP: staged coarse rows / columns
    constexpr int NC = (CE * CE + 255) / 256;
    __shared__ double sp[E][E];
    __shared__ double sb[E][E];
    __shared__ double rw[E][4];   // per staged row: cw, ce, cw + ce, hx
    __shared__ double cl[E][4];   // per staged column: cs, cn, cs + cn, hy
    __shared__ double se[XP ? CE : 1][XP ? CE : 1];
    const int t = xcd_swizzle(blockIdx.x, gridDim.x);
    const int ti = t / tiles_j, tj = t - ti * tiles_j;
    const int li0 = ti * TT, j0 = tj * TT;
    const int ld = a.ld, ny = a.ny;
    const int rlo = -HALO, rhi = a.nxl + HALO - 1;
    // every global load first (one latency for the whole stage-in): phi and b over the cone,
    // the row / column coefficients, and (XP) the coarse correction over its parent rows
    // Ilo-1 .. (whole level: ci0 = 0; rows clamped into the allocation -- a clamped row only
    // feeds cells outside the cone)
    double pv[NQ], bv[NQ], ev[NC];
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const int q = threadIdx.x + 256 * k;
        if (q < E * E) {
            const int r = q / E, cc = q - r * E;
            const int li = min(max(li0 - R + r, rlo), rhi);
            const int j = min(max(j0 - R + cc, 0), ny - 1);
            pv[k] = ZIN ? 0.0 : a.in[(ptrdiff_t)li * ld + j];
            bv[k] = a.b[(ptrdiff_t)li * ld + j];
        }
    }
    const int Ilo = ((li0 - R) >> 1) - 1, Jlo = max(((j0 - R) >> 1) - 1, 0);
    if (XP) {
#pragma unroll
        for (int k = 0; k < NC; k++) {
            const int q = threadIdx.x + 256 * k;
            if (q < CE * CE) {
                const int r = q / CE, cc = q - r * CE;
                const int I = min(max(Ilo + r, -HALO), a.ncx + HALO - 1);
                const int J = min(Jlo + cc, a.ncy - 1);
                ev[k] = a.ec[(ptrdiff_t)I * a.ldc + J];
            }
        }
    }
    double c4[4] = {0.0, 0.0, 0.0, 0.0};
    if (threadIdx.x < E) {
        const int gi = min(max(a.i0 + li0 - R + (int)threadIdx.x, 0), a.nx - 1);
        c4[0] = a.cw[gi]; c4[1] = a.ce[gi]; c4[3] = XR ? a.hx[gi] : 0.0;
    } else if (threadIdx.x >= 64 && threadIdx.x < 64 + E) {
        const int j = min(max(j0 - R + (int)threadIdx.x - 64, 0), ny - 1);
        c4[0] = a.cs[j]; c4[1] = a.cn[j]; c4[3] = XR ? a.hy[j] : 0.0;
    }
    const double shift = a.shift ? a.shift[0] : 0.0;
    if (threadIdx.x < E) {
        rw[threadIdx.x][0] = c4[0]; rw[threadIdx.x][1] = c4[1]; rw[threadIdx.x][2] = c4[0] + c4[1];
        rw[threadIdx.x][3] = c4[3];
    } else if (threadIdx.x >= 64 && threadIdx.x < 64 + E) {
        const int q = threadIdx.x - 64;
        cl[q][0] = c4[0]; cl[q][1] = c4[1]; cl[q][2] = c4[0] + c4[1]; cl[q][3] = c4[3];
    }
    if (XP) {
#pragma unroll
        for (int k = 0; k < NC; k++) {
            const int q = threadIdx.x + 256 * k;
            if (q < CE * CE) se[q / CE][q - (q / CE) * CE] = ev[k];
        }
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const int q = threadIdx.x + 256 * k;
        if (q < E * E) {
            const int r = q / E, cc = q - r * E;
            double p = pv[k];
            if (XP) {
                // phi += P(e) (k_prolong / k_sweep2<FUSE_P>: the row's coarse row I and its
                // neighbour In on the child's side, the wall reflecting onto the parent)
                const int li = min(max(li0 - R + r, rlo), rhi);
                const int j = min(max(j0 - R + cc, 0), ny - 1);
                const int I = li >> 1, Jc = j >> 1;
                int In = (li & 1) ? I + 1 : I - 1;
                double wn = 1.0;   // -1: a face-Dirichlet side (Geo::dsx), odd instead of even
                if (a.ci0 + In < 0 || a.ci0 + In >= a.ncx) {
                    if (a.dsx & ((li & 1) ? 2 : 1)) wn = -1.0;
                    In = I;
                }
                int Jn = (j & 1) ? Jc + 1 : Jc - 1;
                if (Jn < 0 || Jn >= a.ncy) Jn = Jc;
                const int i1 = I - Ilo, i2 = In - Ilo, k1 = Jc - Jlo, k2 = Jn - Jlo;
                if (a.i0 + li >= 0 && a.i0 + li < a.nx)
                    p += (9.0 * se[i1][k1] + 3.0 * wn * se[i2][k1] + 3.0 * se[i1][k2] + wn * se[i2][k2]) * 0.0625;
            }
            sp[r][cc] = p;
            sb[r][cc] = bv[k] - shift;
        }
    }
    __syncthreads();
    const double omega = a.omega;
    const int gib = a.i0 + li0 - R, jb = j0 - R;   // global row / column of staged (0, 0)
#pragma unroll
    for (int h = 0; h < 4; h++) {
        const int par = h & 1;              // red ((gi + j) even), black, red, black
        const int W = E - 2 - 2 * h;         // the half-sweep's region: [h+1, E-2-h]^2
        const int hw = W / 2;
        for (int q = threadIdx.x; q < W * hw; q += 256) {
            const int r = h + 1 + q / hw;
            const int gi = gib + r;
            const int cc = h + 1 + 2 * (q - (q / hw) * hw) + ((par + gi + jb + h + 1) & 1);
            const int j = jb + cc;
            if (gi < 0 || gi >= a.nx || j < 0 || j >= ny) continue;
            const double dg = diag<0>(rw[r][2], cl[cc][2], 0.0), w = omega * rcp_nr(dg);
            double rr;
            sp[r][cc] = relax<0>(sp[r][cc], sp[r - 1][cc], sp[r + 1][cc], sp[r][cc - 1], sp[r][cc + 1], sb[r][cc],
                                 rw[r][0], rw[r][1], cl[cc][0], cl[cc][1], dg, w, 0.0, rr);
        }
        __syncthreads();
    }
    double res = 0.0;
    for (int q = threadIdx.x; q < TT * TT; q += 256) {
        const int r = R + q / TT, cc = R + (q & (TT - 1));
        const int li = li0 + r - R, j = j0 + cc - R;
        if (li >= a.nxl || j >= ny) continue;
        a.out[(ptrdiff_t)li * ld + j] = sp[r][cc];
        if (R5) {
            const double dg = diag<0>(rw[r][2], cl[cc][2], 0.0);
            double rr;
            relax<0>(sp[r][cc], sp[r - 1][cc], sp[r + 1][cc], sp[r][cc - 1], sp[r][cc + 1], sb[r][cc], rw[r][0],
                     rw[r][1], cl[cc][0], cl[cc][1], dg, 0.0, 0.0, rr);
            res += rr * rr;
            if (XR) sb[r][cc] = rr;   // this cell's own b is no longer needed
        }
    }
    if (RES && !XR && a.part) {
        double x[1] = {res};
        block_reduce_sum<1>(x, a.part + blockIdx.x);
    }
    if (XR) {
        __syncthreads();
        // one coarse cell per thread: k_restrict's area-weighted sum, same order
        const int Ic = threadIdx.x / (TT / 2), Jc = threadIdx.x - Ic * (TT / 2);
        const int li = li0 + 2 * Ic, j = j0 + 2 * Jc;
        if ((int)threadIdx.x < (TT / 2) * (TT / 2) && li < a.nxl && j < ny) {
            const int r = R + 2 * Ic, cc = R + 2 * Jc;
            double xs = (rw[r][3] * cl[cc][3]) * sb[r][cc];
            xs = xs + (rw[r][3] * cl[cc + 1][3]) * sb[r][cc + 1];
            xs = xs + (rw[r + 1][3] * cl[cc][3]) * sb[r + 1][cc];
            xs = xs + (rw[r + 1][3] * cl[cc + 1][3]) * sb[r + 1][cc + 1];
            const ptrdiff_t o = (ptrdiff_t)(li >> 1) * a.ldc + (j >> 1);
            a.bc[o] = xs / ((rw[r][3] + rw[r + 1][3]) * (cl[cc][3] + cl[cc + 1][3]));
            if (a.pc) a.pc[o] = 0.0;
        }
        if (a.part) {
            double x[1] = {res};
            block_reduce_sum<1>(x, a.part + blockIdx.x);
        }
    }
}

// ------------------------------------------------ K2 wall bands (before the global Helmholtz passes)
// The Helmholtz residual of the guess u^n lives in thin layers along the walls -- the lid's and
// the side walls' boundary layers: at 4096^2 > 99.9 % of ||r||^2 lies within 16 cells of a wall
// -- where the global RB-SOR sweeps converge at their asymptotic rate.  6 RB-SOR sweeps
// restricted to the cells within 128 of a wall (every other cell held; the solver's band_w /
// band_sweeps) first cut the global sweeps rtol 1e-8 needs from 7 to 3 at 4096^2
// (tools/helm_band_study.py): ONE HBM pass per component (k_sweep3 with its residual stage)
// instead of three (3 + 2 + 2).  A launch does 3 of the sweeps: one workgroup per BT x BT tile
// that touches the band stages the tile and its 6-cell dependency cone (one cell per half-sweep)
// in LDS -- k_tile2's temporal blocking -- so its band cells come out exactly as from the global
// masked sweeps, whatever the tiling (one rank and slabs agree).  The band cells are read from
// `qb` and written to `out`, the other cells read from `q` (never written): launch 1 reads the
// iterate and writes the scratch plane, launch 2 reads the scratch plane's band and writes the
// iterate -- no tile ever writes what another reads, and no copy-back.  Same arithmetic as the
// streaming passes (relax<1>, diag<1>, the Newton reciprocal: w = omega / d is formed once per
// cell, 0 off the band).  blockIdx.y: 0 u, 1 v.
struct BandArgs {
    const double* q[2];    // the iterates u, v (cells off the band; never written)
    const double* qb[2];   // the band cells' current values
    double* out[2];        // the band cells' new values
    const double* b[2];    // RHS_u, RHS_v
    const double *cw, *ce, *bx, *cs, *cn, *by;
    double alpha, omega;
    int nx, ny, i0, nxl, ld;
    int bw;                // band width (cells from a wall)
    int nti, ntj;          // tiles of the slab: rows, columns
    int fa, fb;            // tile rows [0, fa) and [fb, nti) touch the W / E bands: every column
    int ncl, ncr;          // other tile rows: columns [0, ncl) and [ncr, ntj) only
    int phase;             // exchange overlap (set_strip_phase): 1 the tiles that read no neighbour's
                           // ghost rows, 2 the others, 0 all
};
__device__ __forceinline__ void band_tile(int b, const BandArgs& t, int& ti, int& tj) {
    const int nf = t.fa * t.ntj, nl = (t.nti - t.fb) * t.ntj;
    if (b < nf) { ti = b / t.ntj; tj = b - ti * t.ntj; return; }
    b -= nf;
    if (b < nl) { ti = t.fb + b / t.ntj; tj = b - (b / t.ntj) * t.ntj; return; }
    b -= nl;
    const int k = t.ncl + t.ntj - t.ncr, c = b % k;
    ti = t.fa + b / k;
    tj = c < t.ncl ? c : t.ncr + (c - t.ncl);
}
// a band cell of the domain (global row gi, column j)
__device__ __forceinline__ bool in_band(int gi, int j, int nx, int ny, int bw) {
    return gi >= 0 && gi < nx && (gi < bw || gi >= nx - bw || j < bw || j >= ny - bw);
}

#ifndef BAND_TBL_FIRST
#define BAND_TBL_FIRST 1   // k_helm_band: the coefficient tables loaded before the tile, unconditionally (A/B: 0)
#endif
constexpr int BAND_NSW = 3;   // sweeps per launch: a 6-cell cone, within the slabs' 6 ghost rows
// Thread layout: the staged E x E region (E = BT + 12 = 44) is cut into 22 column pairs x 11
// segments of 4 rows; a thread keeps its 8 cells (value, rhs, weight) in registers and meets
// its neighbours in LDS only across the segment / pair edges: per update ~1.5 LDS reads instead
// of ~12.  A row of a pair holds one cell of each colour, and the colour's column in row s is
// (par + gi + j0) parity: uniform over the workgroup (every pair starts on an even column,
// every segment on an even row), so there is no divergence.  One barrier per half-sweep: a
// half-sweep reads only the other colour (stable) and publishes its own cells.
// (r6, k_helm_band6's body: BTT tile, NSW sweeps, SEGT rows per thread, NTH threads; the relaxation weights
// formed at each update -- the 512 threads must fit 128 VGPRs for 2 workgroups a CU)
template <int BTT, int NSW, int SEGT, int NTH>
__device__ __forceinline__ void helm_band_body(const BandArgs& a, double* smem) {
    constexpr int R = 2 * NSW, E = BTT + 2 * R, NP = E / 2, SEG = SEGT, NSEG = E / SEG;
    constexpr int CO = (E + 63) / 64 * 64;   // the column tables' loaders: threads CO .. CO + E - 1
    static_assert(E % SEG == 0 && NP * NSEG <= NTH && CO + E <= NTH, "band tile layout");
    double (*sp)[E] = reinterpret_cast<double (*)[E]>(smem);
    double (*rw)[3] = reinterpret_cast<double (*)[3]>(smem + E * E);           // per staged row: cw, ce, cw + ce + bx
    double (*cl)[3] = reinterpret_cast<double (*)[3]>(smem + E * E + 3 * E);   // per staged column: cs, cn, cs + cn + by
    int ti, tj;
    band_tile(blockIdx.x, a, ti, tj);
    const int f = blockIdx.y;
    const double* q = a.q[f];
    const double* qb = a.qb[f];
    const double* b = a.b[f];
    const int li0 = ti * BTT, j0 = tj * BTT, ld = a.ld, ny = a.ny, nx = a.nx;
    if (a.phase) {   // (workgroup-uniform) does the staged region reach a neighbour rank's rows?
        const bool touch = (a.i0 > 0 && li0 - R < 0) || (a.i0 + a.nxl < nx && li0 + BTT + R > a.nxl);
        if (touch != (a.phase == 2)) return;
    }
    const int rlo = -HALO, rhi = a.nxl + HALO - 1;
    const int gib = a.i0 + li0 - R, jb = j0 - R;   // global row / column of staged (0, 0)
    const int t = threadIdx.x;
    const bool act = t < NP * NSEG;
    const int kp = act ? t % NP : 0, sg = act ? t / NP : 0;
    const int c0 = 2 * kp, r0 = SEG * sg;          // columns c0, c0 + 1; rows r0 .. r0 + SEG - 1
    double2 v[SEG], bq[SEG];
    int jj[2];
    bool jin[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const int j = jb + c0 + e;
        jin[e] = j >= 0 && j < ny;
        jj[e] = min(max(j, 0), ny - 1);
    }
#pragma unroll
    for (int s = 0; s < SEG; s++) {
        const int li = min(max(li0 - R + r0 + s, rlo), rhi);
        const ptrdiff_t o = (ptrdiff_t)li * ld;
        const bool b0 = in_band(a.i0 + li, jj[0], nx, ny, a.bw), b1 = in_band(a.i0 + li, jj[1], nx, ny, a.bw);
        v[s].x = (b0 ? qb : q)[o + jj[0]];
        v[s].y = (b1 ? qb : q)[o + jj[1]];
        bq[s].x = b[o + jj[0]];
        bq[s].y = b[o + jj[1]];
    }
    if (t < E) {
        const int gi = min(max(gib + t, 0), nx - 1);
        const double cw = a.cw[gi], ce = a.ce[gi];
        rw[t][0] = cw; rw[t][1] = ce; rw[t][2] = cw + ce + a.bx[gi];
    } else if (t >= CO && t < CO + E) {
        const int k = t - CO;
        const int j = min(max(jb + k, 0), ny - 1);
        const double cs = a.cs[j], cn = a.cn[j];
        cl[k][0] = cs; cl[k][1] = cn; cl[k][2] = cs + cn + a.by[j];
    }
    if (act) {
#pragma unroll
        for (int s = 0; s < SEG; s++) { sp[r0 + s][c0] = v[s].x; sp[r0 + s][c0 + 1] = v[s].y; }
    }
    __syncthreads();
    const double alpha = a.alpha, omega = a.omega;
    // this thread's column coefficients; the row's and the relaxation weight (0 on held cells: k_helm_band's
    // expression) at each update
    const double ccs0 = cl[c0][0], ccn0 = cl[c0][1], ccd0 = cl[c0][2];
    const double ccs1 = cl[c0 + 1][0], ccn1 = cl[c0 + 1][1], ccd1 = cl[c0 + 1][2];
    const int cpar = (gib + jb) & 1;   // colour parity of staged (0, 0)
    for (int h = 0; h < 2 * NSW; h++) {
        const int par = h & 1;                   // red ((gi + j) even), black, ...
        const int lo = h + 1, hi = E - 2 - h;    // the half-sweep's region: [lo, hi]^2
        if (act) {
#pragma unroll
            for (int s = 0; s < SEG; s++) {
                const int r = r0 + s;
                if (r < lo || r > hi) continue;
                // the colour's column in this row: c0 + e, e = (par + gi + j) parity, uniform
                const int e = (par + cpar + r) & 1;
                const int cc = c0 + e;
                if (cc < lo || cc > hi) continue;
                const double xm = s > 0 ? (e ? v[s - 1].y : v[s - 1].x) : sp[r - 1][cc];
                const double xp = s < SEG - 1 ? (e ? v[s + 1].y : v[s + 1].x) : sp[r + 1][cc];
                double rr;
                const double cws = rw[r][0], ces = rw[r][1], rds = rw[r][2];
                const double wc = ((e ? jin[1] : jin[0]) && in_band(gib + r, e ? jj[1] : jj[0], nx, ny, a.bw))
                                      ? omega * rcp_nr(diag<1>(rds, e ? ccd1 : ccd0, alpha)) : 0.0;
                if (e == 0) {
                    const double ym = sp[r][cc - 1], yp = v[s].y;
                    v[s].x = relax<1>(v[s].x, xm, xp, ym, yp, bq[s].x, cws, ces, ccs0, ccn0,
                                      diag<1>(rds, ccd0, alpha), wc, alpha, rr);
                    sp[r][cc] = v[s].x;
                } else {
                    const double ym = v[s].x, yp = sp[r][cc + 1];
                    v[s].y = relax<1>(v[s].y, xm, xp, ym, yp, bq[s].y, cws, ces, ccs1, ccn1,
                                      diag<1>(rds, ccd1, alpha), wc, alpha, rr);
                    sp[r][cc] = v[s].y;
                }
            }
        }
        __syncthreads();
    }
    if (act) {
        double* out = a.out[f];
#pragma unroll
        for (int s = 0; s < SEG; s++) {
            const int r = r0 + s, li = li0 + r - R;
            if (r < R || r >= R + BTT || li >= a.nxl) continue;
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const int cc = c0 + e, j = jb + cc;
                if (cc < R || cc >= R + BTT || j >= ny || !in_band(a.i0 + li, j, nx, ny, a.bw)) continue;
                out[(ptrdiff_t)li * ld + j] = e ? v[s].y : v[s].x;
            }
        }
    }
}
// (the 3-sweep launch: its own body -- the templated one above measured 48.5 -> 62.8 us here)
__global__ __launch_bounds__(256) void k_helm_band(BandArgs a) {
    constexpr int R = 2 * BAND_NSW, E = BT + 2 * R, NP = E / 2, SEG = BAND_SEG, NSEG = E / SEG;
    static_assert(E % SEG == 0 && NP * NSEG <= 256, "band tile layout");
    __shared__ double sp[E][E];
    __shared__ double rw[E][3];   // per staged row: cw, ce, cw + ce + bx
    __shared__ double cl[E][3];   // per staged column: cs, cn, cs + cn + by
    int ti, tj;
    band_tile(blockIdx.x, a, ti, tj);
    const int f = blockIdx.y;
    const double* q = a.q[f];
    const double* qb = a.qb[f];
    const double* b = a.b[f];
    const int li0 = ti * BT, j0 = tj * BT, ld = a.ld, ny = a.ny, nx = a.nx;
    if (a.phase) {   // (workgroup-uniform) does the staged region reach a neighbour rank's rows?
        const bool touch = (a.i0 > 0 && li0 - R < 0) || (a.i0 + a.nxl < nx && li0 + BT + R > a.nxl);
        if (touch != (a.phase == 2)) return;
    }
    const int rlo = -HALO, rhi = a.nxl + HALO - 1;
    const int gib = a.i0 + li0 - R, jb = j0 - R;   // global row / column of staged (0, 0)
    const int t = threadIdx.x;
    const bool act = t < NP * NSEG;
    const int kp = act ? t % NP : 0, sg = act ? t / NP : 0;
    const int c0 = 2 * kp, r0 = SEG * sg;          // columns c0, c0 + 1; rows r0 .. r0 + SEG - 1
    // (r6) the coefficient tables' loads first, unconditional in waves 0 (rows) and 1 (columns), so that they fly
    // with the tile's: in the branches below they had waited for the tile's loads and then one another (the ISA's
    // load / s_waitcnt vmcnt(0) pairs), two round trips more before the first barrier
#if BAND_TBL_FIRST
    double tb0 = 0.0, tb1 = 0.0, tb2 = 0.0;
    if (t < 128) {   // (wave-uniform)
        const bool rowt = t < 64;
        const int k = t & 63;
        const int ix = rowt ? min(max(gib + k, 0), nx - 1) : min(max(jb + k, 0), ny - 1);
        tb0 = (rowt ? a.cw : a.cs)[ix];
        tb1 = (rowt ? a.ce : a.cn)[ix];
        tb2 = (rowt ? a.bx : a.by)[ix];
    }
#endif
    double2 v[SEG], bq[SEG];
    int jj[2];
    bool jin[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const int j = jb + c0 + e;
        jin[e] = j >= 0 && j < ny;
        jj[e] = min(max(j, 0), ny - 1);
    }
#pragma unroll
    for (int s = 0; s < SEG; s++) {
        const int li = min(max(li0 - R + r0 + s, rlo), rhi);
        const ptrdiff_t o = (ptrdiff_t)li * ld;
        const bool b0 = in_band(a.i0 + li, jj[0], nx, ny, a.bw), b1 = in_band(a.i0 + li, jj[1], nx, ny, a.bw);
        v[s].x = (b0 ? qb : q)[o + jj[0]];
        v[s].y = (b1 ? qb : q)[o + jj[1]];
        bq[s].x = b[o + jj[0]];
        bq[s].y = b[o + jj[1]];
    }
#if BAND_TBL_FIRST
    if (t < E) {
        rw[t][0] = tb0; rw[t][1] = tb1; rw[t][2] = tb0 + tb1 + tb2;
    } else if (t >= 64 && t < 64 + E) {
        cl[t - 64][0] = tb0; cl[t - 64][1] = tb1; cl[t - 64][2] = tb0 + tb1 + tb2;
    }
#else
    if (t < E) {
        const int gi = min(max(gib + t, 0), nx - 1);
        const double cw = a.cw[gi], ce = a.ce[gi];
        rw[t][0] = cw; rw[t][1] = ce; rw[t][2] = cw + ce + a.bx[gi];
    } else if (t >= 64 && t < 64 + E) {
        const int k = t - 64;
        const int j = min(max(jb + k, 0), ny - 1);
        const double cs = a.cs[j], cn = a.cn[j];
        cl[k][0] = cs; cl[k][1] = cn; cl[k][2] = cs + cn + a.by[j];
    }
#endif
    if (act) {
#pragma unroll
        for (int s = 0; s < SEG; s++) { sp[r0 + s][c0] = v[s].x; sp[r0 + s][c0 + 1] = v[s].y; }
    }
    __syncthreads();
    const double alpha = a.alpha, omega = a.omega;
    // this thread's coefficients and relaxation weights (0 on held cells)
    double2 w[SEG];
    double rcw[SEG], rce[SEG], rd[SEG];
    const double ccs0 = cl[c0][0], ccn0 = cl[c0][1], ccd0 = cl[c0][2];
    const double ccs1 = cl[c0 + 1][0], ccn1 = cl[c0 + 1][1], ccd1 = cl[c0 + 1][2];
#pragma unroll
    for (int s = 0; s < SEG; s++) {
        const int r = r0 + s, gi = gib + r;
        rcw[s] = rw[r][0]; rce[s] = rw[r][1]; rd[s] = rw[r][2];
        w[s].x = (jin[0] && in_band(gi, jj[0], nx, ny, a.bw)) ? omega * rcp_nr(diag<1>(rd[s], ccd0, alpha)) : 0.0;
        w[s].y = (jin[1] && in_band(gi, jj[1], nx, ny, a.bw)) ? omega * rcp_nr(diag<1>(rd[s], ccd1, alpha)) : 0.0;
    }
    const int cpar = (gib + jb) & 1;   // colour parity of staged (0, 0)
    for (int h = 0; h < 2 * BAND_NSW; h++) {
        const int par = h & 1;                   // red ((gi + j) even), black, ...
        const int lo = h + 1, hi = E - 2 - h;    // the half-sweep's region: [lo, hi]^2
        if (act) {
#pragma unroll
            for (int s = 0; s < SEG; s++) {
                const int r = r0 + s;
                if (r < lo || r > hi) continue;
                // the colour's column in this row: c0 + e, e = (par + gi + j) parity, uniform
                const int e = (par + cpar + r) & 1;
                const int cc = c0 + e;
                if (cc < lo || cc > hi) continue;
                const double xm = s > 0 ? (e ? v[s - 1].y : v[s - 1].x) : sp[r - 1][cc];
                const double xp = s < SEG - 1 ? (e ? v[s + 1].y : v[s + 1].x) : sp[r + 1][cc];
                double rr;
                if (e == 0) {
                    const double ym = sp[r][cc - 1], yp = v[s].y;
                    v[s].x = relax<1>(v[s].x, xm, xp, ym, yp, bq[s].x, rcw[s], rce[s], ccs0, ccn0,
                                      diag<1>(rd[s], ccd0, alpha), w[s].x, alpha, rr);
                    sp[r][cc] = v[s].x;
                } else {
                    const double ym = v[s].x, yp = sp[r][cc + 1];
                    v[s].y = relax<1>(v[s].y, xm, xp, ym, yp, bq[s].y, rcw[s], rce[s], ccs1, ccn1,
                                      diag<1>(rd[s], ccd1, alpha), w[s].y, alpha, rr);
                    sp[r][cc] = v[s].y;
                }
            }
        }
        __syncthreads();
    }
    if (act) {
        double* out = a.out[f];
#pragma unroll
        for (int s = 0; s < SEG; s++) {
            const int r = r0 + s, li = li0 + r - R;
            if (r < R || r >= R + BT || li >= a.nxl) continue;
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const int cc = c0 + e, j = jb + cc;
                if (cc < R || cc >= R + BT || j >= ny || !in_band(a.i0 + li, j, nx, ny, a.bw)) continue;
                out[(ptrdiff_t)li * ld + j] = e ? v[s].y : v[s].x;
            }
        }
    }
}

// (r6) one rank: all 6 sweeps in ONE launch -- 64 x 64 tiles and their 12-cell cone (88 x 88
// staged, 66 KB of LDS: 2 workgroups a CU), the same (88/64)^2 read amplification as a 3-sweep
// 32 x 32 launch, so half the band traffic; the band cells land in `out` (the scratch plane) and
// k_band_copy brings them back.  Identical arithmetic (each band cell's value after 6 sweeps does
// not depend on the tiling).
constexpr int BAND6_BT = 64, BAND6_E = BAND6_BT + 24;
constexpr int BAND6_LDS = (BAND6_E * BAND6_E + 6 * BAND6_E) * 8;
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_helm_band6(BandArgs a) {
    extern __shared__ double smem6[];
    helm_band_body<BAND6_BT, 6, 8, 512>(a, smem6);
}

// the band cells of each tile: qb -> out (an odd number of band launches ends in the scratch plane)
template <int BTT>
__global__ __launch_bounds__(256) void k_band_copy(BandArgs a) {
    int ti, tj;
    band_tile(blockIdx.x, a, ti, tj);
    const int f = blockIdx.y;
    for (int t = threadIdx.x; t < BTT * BTT; t += 256) {
        const int li = ti * BTT + t / BTT, j = tj * BTT + t % BTT;
        if (li >= a.nxl || j >= a.ny || !in_band(a.i0 + li, j, a.nx, a.ny, a.bw)) continue;
        const ptrdiff_t o = (ptrdiff_t)li * a.ld + j;
        a.out[f][o] = a.qb[f][o];
    }
}

// ------------------------------------------------ K4 multigrid transfer kernels
// Cell-centred geometric multigrid for L phi = b (the Poisson solve of
// FluidSolver.cpp:551): each coarse cell is the union of 2 x 2 fine cells, the
// coarse operator is ConstructLHS's stencil rediscretised on the coarse spacings
// (hx_c = hx_2I + hx_2I+1), restriction is the area-weighted average of the fine
// residuals and prolongation is bilinear (9/16, 3/16, 3/16, 1/16; a missing coarse
// neighbour at a wall is replaced by the parent -- the zero-flux reflection).
// Both transfers are one HBM pass over the fine level (16 B/cell and 24 B/cell).

// residual b - shift - L phi at fine cell (li, j)
__device__ __forceinline__ double pois_residual(const Geo& g, const Coef& c, const double* phi, const double* b,
                                                double shift, int li, int j) {
    const int gi = g.i0 + li, ld = g.ld;
    const double cw = c.pw[gi], ce = c.pe[gi], cs = c.ps[j], cn = c.pn[j];
    const double q = ldf(phi, ld, li, j);
    const double s = cw * ldf(phi, ld, li - 1, j) + ce * ldf(phi, ld, li + 1, j) +
                     cs * ldf(phi, ld, li, max(j - 1, 0)) + cn * ldf(phi, ld, li, min(j + 1, g.ny - 1));
    const double dg = -((cw + ce) + (cs + cn));
    return (ldf(b, ld, li, j) - shift) - (s + dg * q);
}

// fine residual -> coarse rhs (area-weighted average), coarse phi := 0; partials of sum r^2 (fine)
__global__ __launch_bounds__(256) void k_restrict(Geo gf, Coef cf, const double* __restrict__ phi,
                                                  const double* __restrict__ b, const double* __restrict__ shiftp,
                                                  Geo gc, Coef cc, double* __restrict__ bc, double* __restrict__ pc,
                                                  double* __restrict__ part, int rows) {
    const int J = blockIdx.x * 64 + threadIdx.x;
    const int Iend = min((int)(blockIdx.y + 1) * 4 * rows, gc.nxl);
    double acc[1] = {0.0};
    for (int I = blockIdx.y * 4 * rows + threadIdx.y; I < Iend && J < gc.ny; I += 4) {
        const double shift = shiftp ? shiftp[0] : 0.0;
        double sum = 0.0;
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const int li = 2 * I + a, j = 2 * J + q;
                const double r = pois_residual(gf, cf, phi, b, shift, li, j);
                sum += (cf.hx[gf.i0 + li] * cf.hy[j]) * r;
                acc[0] += r * r;
            }
        const int gI = gc.i0 + I;
        bc[(ptrdiff_t)I * gc.ld + J] = sum / (cc.hx[gI] * cc.hy[J]);
        pc[(ptrdiff_t)I * gc.ld + J] = 0.0;
    }
    block_reduce_sum<1>(acc, part + (blockIdx.x + gridDim.x * blockIdx.y));
}

// fine phi += bilinear interpolation of the coarse correction
__global__ __launch_bounds__(256) void k_prolong(Geo gf, double* __restrict__ phi, Geo gc,
                                                 const double* __restrict__ ec, int rows) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int lend = min((int)(blockIdx.y + 1) * 4 * rows, gf.nxl);
    if (j >= gf.ny) return;
    for (int li = blockIdx.y * 4 * rows + threadIdx.y; li < lend; li += 4) {
    const int I = li >> 1, Jc = j >> 1;
    const int In = (li & 1) ? I + 1 : I - 1;        // coarse row on this child's side
    const int Jn = (j & 1) ? Jc + 1 : Jc - 1;
    const int gIn = gc.i0 + In;
    const int Iu = (gIn >= 0 && gIn < gc.nx) ? In : I;       // wall: reflect onto the parent
    const int Ju = (Jn >= 0 && Jn < gc.ny) ? Jn : Jc;
    // a face-Dirichlet side (Geo::dsx): e extended oddly (0 on the face) instead
    const double wn = (Iu == I && (gc.dsx & ((li & 1) ? 2 : 1))) ? -1.0 : 1.0;
    const double e = (9.0 * ldf(ec, gc.ld, I, Jc) + 3.0 * wn * ldf(ec, gc.ld, Iu, Jc) + 3.0 * ldf(ec, gc.ld, I, Ju) +
                      wn * ldf(ec, gc.ld, Iu, Ju)) * 0.0625;
    phi[(ptrdiff_t)li * gf.ld + j] += e;
    }
}

// ------------------------------------------------ K4 coarse levels: a whole V-cycle in LDS
// Levels from the coarsest global one (<= 64 x 64) down to <= 4 x 4 live in one
// workgroup's LDS; one launch runs `cycles` V-cycles over them (RB Gauss-Seidel
// smoothing, the same area-weighted restriction / bilinear prolongation as
// k_restrict / k_prolong, RB-SOR on the last level).  Replaces ~6 launches per level
// that are pure launch latency at these sizes.  Single rank (the level is whole).
constexpr int LV_MAX = 8;
constexpr int CV_THREADS = 1024;


struct LdsLv {
    int nx, ny, phi, b, idg, cw, ce, cs, cn, hx, hy;  // offsets in doubles
    float rny;                                          // 1/ny for the index split
    int dlo, dhi;   // a Dirichlet-centre closure (ghost value 0) on the x-low / x-high side
};

// a level's descriptor read from LDS, made wave-uniform (SGPRs instead of ~14 VGPRs per copy)
__device__ __forceinline__ LdsLv lv_uni(const LdsLv& s) {
    LdsLv v;
    v.nx = __builtin_amdgcn_readfirstlane(s.nx); v.ny = __builtin_amdgcn_readfirstlane(s.ny);
    v.phi = __builtin_amdgcn_readfirstlane(s.phi); v.b = __builtin_amdgcn_readfirstlane(s.b);
    v.idg = __builtin_amdgcn_readfirstlane(s.idg); v.cw = __builtin_amdgcn_readfirstlane(s.cw);
    v.ce = __builtin_amdgcn_readfirstlane(s.ce); v.cs = __builtin_amdgcn_readfirstlane(s.cs);
    v.cn = __builtin_amdgcn_readfirstlane(s.cn); v.hx = __builtin_amdgcn_readfirstlane(s.hx);
    v.hy = __builtin_amdgcn_readfirstlane(s.hy);
    v.rny = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(s.rny)));
    v.dlo = __builtin_amdgcn_readfirstlane(s.dlo); v.dhi = __builtin_amdgcn_readfirstlane(s.dhi);
    return v;
}

// k -> (k / ny, k % ny) without an integer division: float estimate + one correction
__device__ __forceinline__ void lv_split(const LdsLv& v, int k, int& i, int& j) {
    i = __float2int_rz(__int2float_rn(k) * v.rny);
    j = k - i * v.ny;
    if (j < 0) { i--; j += v.ny; }
    else if (j >= v.ny) { i++; j -= v.ny; }
}

__device__ __forceinline__ double lv_lap(const double* L, const LdsLv& v, int i, int j) {
    const int ny = v.ny, k = i * ny + j;
    const double* p = L + v.phi;
    // (a wall's weight is 0; a Dirichlet-centre side's ghost holds 0: the correction's data)
    const double pw = i > 0 ? p[k - ny] : (v.dlo ? 0.0 : p[k]);
    const double pe = i < v.nx - 1 ? p[k + ny] : (v.dhi ? 0.0 : p[k]);
    const double s = L[v.cw + i] * pw + L[v.ce + i] * pe +
                     L[v.cs + j] * p[k - (j > 0 ? 1 : 0)] + L[v.cn + j] * p[k + (j < ny - 1 ? 1 : 0)];
    const double dg = -((L[v.cw + i] + L[v.ce + i]) + (L[v.cs + j] + L[v.cn + j]));
    return s + dg * p[k];
}

__device__ __forceinline__ void lv_rb(double* L, const LdsLv& v, double omega, int sweeps) {
    const bool even = (v.ny & 1) == 0;
    const int cnt = even ? v.nx * v.ny / 2 : v.nx * v.ny;
    for (int s = 0; s < sweeps; s++)
        for (int color = 0; color < 2; color++) {
            for (int t = threadIdx.x; t < cnt; t += CV_THREADS) {
                // even ny: the t-th cell of this colour in row-major order; odd ny (last
                // level only): every cell, filtered by colour
                int i, j;
                lv_split(v, even ? 2 * t : t, i, j);
                if (even) j += ((i + j + color) & 1);
                else if ((i + j + color) & 1) continue;
                const int c = i * v.ny + j;
                const double r = L[v.b + c] - lv_lap(L, v, i, j);
                L[v.phi + c] += omega * r * L[v.idg + c];
            }
            __syncthreads();
        }
}

// the coarsest level's RB-SOR solve (citers sweeps): when it has <= 64 cells of a colour,
// wave 0 alone runs it -- its lanes' LDS accesses stay in program order, so a wave barrier
// (no workgroup barrier) separates the half-sweeps: 2 * citers workgroup barriers saved
__device__ __forceinline__ void lv_rb_last(double* L, const LdsLv& v, double omega, int sweeps) {
    const bool even = (v.ny & 1) == 0;
    const int cnt = even ? v.nx * v.ny / 2 : v.nx * v.ny;
    if (cnt > 64) {
        lv_rb(L, v, omega, sweeps);
        return;
    }
    if (threadIdx.x < 64) {
        const int t = threadIdx.x;
        int i = 0, j = 0;
        if (t < cnt) lv_split(v, even ? 2 * t : t, i, j);
        for (int s = 0; s < sweeps; s++)
            for (int color = 0; color < 2; color++) {
                if (t < cnt) {
                    int jj = j;
                    bool on = true;
                    if (even) jj += ((i + j + color) & 1);
                    else on = ((i + j + color) & 1) == 0;
                    if (on) {
                        const int c = i * v.ny + jj;
                        const double r = L[v.b + c] - lv_lap(L, v, i, jj);
                        L[v.phi + c] += omega * r * L[v.idg + c];
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
    }
    __syncthreads();
}

// The smoothing, residual / restriction and prolongation of a level with even nx, ny in 2 x 2
// blocks: thread t < (nx/2)(ny/2) owns block (a, b) = cells (2a + Q/2, 2b + Q%2), Q = 0..3 --
// one cell of each colour per row, and exactly the four children of coarse cell (a, b).  Its
// cells' phi, b and 1/diag stay in registers for the level's visit, so a half-sweep reads two
// neighbours and the four weights per cell from LDS (the other two neighbours are the thread's
// own) and writes the cell back: ~7 LDS accesses per update instead of ~12.  Same expressions in the same
// order as lv_lap / lv_rb / the restriction and prolongation loops.
struct CvBlk {
    double idg[4], b[4], p[4];
    int i0, j0;
    bool act;
};
__device__ __forceinline__ void blk_load(const double* L, const LdsLv& v, CvBlk& B) {
    const int nby = v.ny >> 1, t = threadIdx.x;
    B.act = t < (v.nx >> 1) * nby;
    if (!B.act) return;
    const int a = t / nby;
    B.i0 = 2 * a;
    B.j0 = 2 * (t - a * nby);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int k = (B.i0 + (q >> 1)) * v.ny + B.j0 + (q & 1);
        B.idg[q] = L[v.idg + k]; B.b[q] = L[v.b + k]; B.p[q] = L[v.phi + k];
    }
}
template <int Q>
__device__ __forceinline__ double blk_lap(const double* L, const LdsLv& v, const CvBlk& B) {
    constexpr int di = Q >> 1, dj = Q & 1;
    const int i = B.i0 + di, j = B.j0 + dj, ny = v.ny, k = i * ny + j;
    const double* p = L + v.phi;
    const double pc = B.p[Q];
    double pw, pe, ps, pn;
    if constexpr (di == 1) pw = B.p[Q - 2]; else pw = i > 0 ? p[k - ny] : (v.dlo ? 0.0 : pc);
    if constexpr (di == 0) pe = B.p[Q + 2]; else pe = i < v.nx - 1 ? p[k + ny] : (v.dhi ? 0.0 : pc);
    if constexpr (dj == 1) ps = B.p[Q - 1]; else ps = j > 0 ? p[k - 1] : pc;
    if constexpr (dj == 0) pn = B.p[Q + 1]; else pn = j < ny - 1 ? p[k + 1] : pc;
    const double cw = L[v.cw + i], ce = L[v.ce + i], cs = L[v.cs + j], cn = L[v.cn + j];
    const double s = cw * pw + ce * pe + cs * ps + cn * pn;
    const double dg = -((cw + ce) + (cs + cn));
    return s + dg * pc;
}
template <int Q>
__device__ __forceinline__ void blk_upd(double* L, const LdsLv& v, CvBlk& B, double omega) {
    const double r = B.b[Q] - blk_lap<Q>(L, v, B);
    B.p[Q] += omega * r * B.idg[Q];
    L[v.phi + (B.i0 + (Q >> 1)) * v.ny + B.j0 + (Q & 1)] = B.p[Q];
}
// prolongation into block cell Q (the cell loop's k_prolong formula; a face-Dirichlet side,
// v.dlo / v.dhi, extends the correction oddly)
template <int Q>
__device__ __forceinline__ void blk_prolong(double* L, const LdsLv& f, const LdsLv& v, CvBlk& B) {
    const int I = B.i0 >> 1, J = B.j0 >> 1;
    const double* e = L + v.phi;
    int In = (Q >> 1) ? I + 1 : I - 1, Jn = (Q & 1) ? J + 1 : J - 1;
    double wn = 1.0;
    if (In < 0 || In >= v.nx) {
        if (In < 0 ? v.dlo : v.dhi) wn = -1.0;
        In = I;
    }
    if (Jn < 0 || Jn >= v.ny) Jn = J;
    B.p[Q] += (9.0 * e[I * v.ny + J] + 3.0 * wn * e[In * v.ny + J] + 3.0 * e[I * v.ny + Jn] + wn * e[In * v.ny + Jn]) *
              0.0625;
    L[f.phi + (B.i0 + (Q >> 1)) * f.ny + B.j0 + (Q & 1)] = B.p[Q];
}
__device__ __forceinline__ void blk_rb(double* L, const LdsLv& v, CvBlk& B, double omega, int sweeps) {
    for (int s = 0; s < sweeps; s++) {
        if (B.act) { blk_upd<0>(L, v, B, omega); blk_upd<3>(L, v, B, omega); }
        __syncthreads();
        if (B.act) { blk_upd<1>(L, v, B, omega); blk_upd<2>(L, v, B, omega); }
        __syncthreads();
    }
}
// the area-weighted residual sum of the block = coarse cell (I, J)'s rhs (k_restrict's order),
// the coarse iterate zeroed
__device__ __forceinline__ void blk_restrict(double* L, const LdsLv& f, const LdsLv& v, const CvBlk& B) {
    if (!B.act) return;
    double sum = 0.0;
    double r = B.b[0] - blk_lap<0>(L, f, B);
    sum += (L[f.hx + B.i0] * L[f.hy + B.j0]) * r;
    r = B.b[1] - blk_lap<1>(L, f, B);
    sum += (L[f.hx + B.i0] * L[f.hy + B.j0 + 1]) * r;
    r = B.b[2] - blk_lap<2>(L, f, B);
    sum += (L[f.hx + B.i0 + 1] * L[f.hy + B.j0]) * r;
    r = B.b[3] - blk_lap<3>(L, f, B);
    sum += (L[f.hx + B.i0 + 1] * L[f.hy + B.j0 + 1]) * r;
    const int I = B.i0 >> 1, J = B.j0 >> 1, t = I * v.ny + J;
    L[v.b + t] = sum / (L[v.hx + I] * L[v.hy + J]);
    L[v.phi + t] = 0.0;
}
__device__ __forceinline__ void blk_prolong_all(double* L, const LdsLv& f, const LdsLv& v, CvBlk& B) {
    if (!B.act) return;
    blk_prolong<0>(L, f, v, B);
    blk_prolong<1>(L, f, v, B);
    blk_prolong<2>(L, f, v, B);
    blk_prolong<3>(L, f, v, B);
}

// LDS footprint (doubles) of the levels from (nx, ny) down; fills lv when non-null
__host__ __device__ inline int lv_layout(int nx, int ny, LdsLv* lv, int* nlev) {
    int off = 0, k = 0;
    for (;;) {
        if (lv) {
            LdsLv& v = lv[k];
            v.nx = nx; v.ny = ny; v.rny = 1.0f / (float)ny;
            v.phi = off; v.b = off + nx * ny; v.idg = off + 2 * nx * ny;
            v.cw = off + 3 * nx * ny; v.ce = v.cw + nx; v.hx = v.ce + nx;
            v.cs = v.hx + nx; v.cn = v.cs + ny; v.hy = v.cn + ny;
        }
        off += 3 * nx * ny + 3 * nx + 3 * ny;
        off = (off + 1) & ~1;
        k++;
        if (k == LV_MAX || !mg_can_coarsen(nx, ny)) break;
        nx /= 2; ny /= 2;
    }
    if (nlev) *nlev = k;
    return off;
}

// the last LDS level is solved directly when it has <= CV_DIRECT cells: x = M b with M the
// inverse of its operator (a Dirichlet-closed side) or, pure Neumann, the n x n block of the
// inverse of the bordered system [A 1; w^T 0] (w = cell areas, the left null vector): A x =
// b - (w.b / w.1) and w.x = 0 -- what the 2n+10 RB-SOR sweeps of the old last-level solve
// converged to up to a constant, in one LDS phase instead of 4n+20 (cv_image builds M)
constexpr int CV_DIRECT = 64;

// the LDS image's size in doubles (levels, then M if the last level is solved directly) and
// the direct solve's size dn (0: RB-SOR sweeps)
__host__ __device__ inline int cv_image_size(int nx, int ny, int* dn) {
    LdsLv lv[LV_MAX];
    int nl = 0;
    const int off = lv_layout(nx, ny, lv, &nl);
    const int n = lv[nl - 1].nx * lv[nl - 1].ny;
    *dn = n <= CV_DIRECT ? n : 0;
    return off + *dn * *dn;
}

#ifndef CV_PROF
#define CV_PROF 0   // (A/B builds: thread 0 prints the phase times of a few launches)
#endif
#if CV_PROF
__device__ int cv_prof_count = 0;
#define CV_T(k) do { if (threadIdx.x == 0 && (k) < 48) tp[(k)] = wall_clock64(); } while (0)
#else
#define CV_T(k) do {} while (0)
#endif

// img: the host-built LDS image (cv_image) of every level's tables (idg, cw, ce, hx, cs, cn,
// hy; phi and b zero) and M; one copy into LDS replaces ~3 barriers of table arithmetic per
// level.  Level 0's phi and b come from the global coarsest level.
template <bool BLK>
__global__ __launch_bounds__(CV_THREADS) void k_coarse_vcycle(Geo g, const double* __restrict__ img, int img_n,
                                                              int dn, double* __restrict__ phi,
                                                              const double* __restrict__ b, int cycles, int pre,
                                                              int post, int citers, double comega, double somega,
                                                              int dlo, int dhi, int zin) {
    extern __shared__ __attribute__((aligned(16))) double L[];
    __shared__ LdsLv lv[LV_MAX];
    __shared__ int nlev;
#if CV_PROF
    unsigned long long tp[48];
    int np = 0;
    CV_T(np); np++;
#endif
    if (threadIdx.x == 0) {
        lv_layout(g.nx, g.ny, lv, &nlev);
        for (int k = 0; k < nlev; k++) { lv[k].dlo = dlo; lv[k].dhi = dhi; }
    }
    {
        // the image from level 0's idg on (16 B per lane; the offsets are even), then level 0's
        // phi and b from the global level
        const int n0 = g.nx * g.ny, from = 2 * n0;
        const double2* src = reinterpret_cast<const double2*>(img + from);
        double2* dst = reinterpret_cast<double2*>(L + from);
        const int n2 = (img_n - from) >> 1;
#pragma unroll 8
        for (int t = threadIdx.x; t < n2; t += CV_THREADS) dst[t] = src[t];
        if (((img_n - from) & 1) && threadIdx.x == 0) L[img_n - 1] = img[img_n - 1];
        LdsLv v;
        v.ny = g.ny;
        v.rny = 1.0f / (float)g.ny;
#if CV_PROF
        __syncthreads();
        CV_T(np); np++;
#endif
        for (int t = threadIdx.x; t < n0; t += CV_THREADS) {
            int i, j;
            lv_split(v, t, i, j);
            L[t] = zin ? 0.0 : ldf(phi, g.ld, i, j);   // (zin: the level's phi is implicitly zero)
            L[n0 + t] = ldf(b, g.ld, i, j);
        }
    }
    __syncthreads();
#if CV_PROF
    CV_T(np); np++;
#endif
    const int nl = nlev;
    for (int cyc = 0; cyc < cycles; cyc++) {
        for (int k = 0; k < nl - 1; k++) {
            const LdsLv f = lv_uni(lv[k]), v = lv_uni(lv[k + 1]);
            if (BLK) {
                CvBlk B;
                blk_load(L, f, B);
                blk_rb(L, f, B, somega, pre);
#if CV_PROF
                CV_T(np); np++;
#endif
                blk_restrict(L, f, v, B);
                __syncthreads();
#if CV_PROF
                CV_T(np); np++;
#endif
                continue;
            }
            lv_rb(L, f, somega, pre);
#if CV_PROF
            CV_T(np); np++;
#endif
            for (int t = threadIdx.x; t < v.nx * v.ny; t += CV_THREADS) {
                int I, J;
                lv_split(v, t, I, J);
                double sum = 0.0;
#pragma unroll
                for (int a = 0; a < 2; a++)
#pragma unroll
                    for (int q = 0; q < 2; q++) {
                        const int i = 2 * I + a, j = 2 * J + q;
                        const double r = L[f.b + i * f.ny + j] - lv_lap(L, f, i, j);
                        sum += (L[f.hx + i] * L[f.hy + j]) * r;
                    }
                L[v.b + t] = sum / (L[v.hx + I] * L[v.hy + J]);
                L[v.phi + t] = 0.0;
            }
            __syncthreads();
#if CV_PROF
            CV_T(np); np++;
#endif
        }
        if (dn > 0) {
            // x = M b (M after the levels in the image)
            const LdsLv v = lv_uni(lv[nl - 1]);
            if ((int)threadIdx.x < dn) {
                const double* M = L + (img_n - dn * dn) + threadIdx.x * dn;
                double x = 0.0;
                for (int k = 0; k < dn; k++) x += M[k] * L[v.b + k];
                L[v.phi + threadIdx.x] = x;
            }
            __syncthreads();
        } else {
            lv_rb_last(L, lv[nl - 1], comega, citers);
        }
#if CV_PROF
        CV_T(np); np++;
#endif
        for (int k = nl - 2; k >= 0; k--) {
            const LdsLv f = lv_uni(lv[k]), v = lv_uni(lv[k + 1]);
            if (BLK) {
                CvBlk B;
                blk_load(L, f, B);
                blk_prolong_all(L, f, v, B);
                __syncthreads();
#if CV_PROF
                CV_T(np); np++;
#endif
                blk_rb(L, f, B, somega, post);
#if CV_PROF
                CV_T(np); np++;
#endif
                continue;
            }
            for (int t = threadIdx.x; t < f.nx * f.ny; t += CV_THREADS) {
                int i, j;
                lv_split(f, t, i, j);
                const int I = i >> 1, J = j >> 1;
                int In = (i & 1) ? I + 1 : I - 1, Jn = (j & 1) ? J + 1 : J - 1;
                double wn = 1.0;   // a face-Dirichlet side (dlo / dhi): e extended oddly
                if (In < 0 || In >= v.nx) {
                    if (In < 0 ? dlo : dhi) wn = -1.0;
                    In = I;
                }
                if (Jn < 0 || Jn >= v.ny) Jn = J;
                const double* e = L + v.phi;
                L[f.phi + t] += (9.0 * e[I * v.ny + J] + 3.0 * wn * e[In * v.ny + J] + 3.0 * e[I * v.ny + Jn] +
                                 wn * e[In * v.ny + Jn]) * 0.0625;
            }
            __syncthreads();
#if CV_PROF
            CV_T(np); np++;
#endif
            lv_rb(L, f, somega, post);
#if CV_PROF
            CV_T(np); np++;
#endif
        }
    }
    {
        const LdsLv v = lv_uni(lv[0]);
        for (int t = threadIdx.x; t < v.nx * v.ny; t += CV_THREADS) {
            int i, j;
            lv_split(v, t, i, j);
            phi[(ptrdiff_t)i * g.ld + j] = L[v.phi + t];
        }
    }
#if CV_PROF
    CV_T(np); np++;
    if (threadIdx.x == 0) {
        const int c = atomicAdd(&cv_prof_count, 1);
        if (c >= 20 && c < 23) {
            printf("cvprof nl=%d n0=%dx%d img=%d dn=%d :", nl, g.nx, g.ny, img_n, dn);
            for (int k = 1; k < np && k < 48; k++) printf(" %.2f", (tp[k] - tp[k - 1]) * 0.01);
            printf(" total %.2f us\n", (tp[np - 1] - tp[0]) * 0.01);
        }
    }
#endif
}


// ---------------------------------------------------------------- reductions
// the 1024 threads' tree sum sh[t] += sh[t + w], w = 512 ... 1, in that pairing: the four levels across waves through
// the LDS, the last six inside wave 0 by shuffles (the same additions in the same order -- bit-identical to the
// all-LDS tree -- with 6 barriers fewer per value).  Thread 0's return value is the sum; the LDS can take the next
// value at once (wave 0 reads only sh[0, 64), which no other wave writes)
__device__ __forceinline__ double tree_sum_1024(double s, double* sh) {
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int w = 512; w >= 64; w >>= 1) {
        if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    double x = threadIdx.x < 64 ? sh[threadIdx.x] : 0.0;
#pragma unroll
    for (int w = 32; w > 0; w >>= 1) x += __shfl_down(x, w, 64);
    return x;
}
__device__ __forceinline__ void reduce_sum_body(const double* __restrict__ p, int n, int nv, double* __restrict__ out,
                                                double* sh) {
    for (int v = 0; v < nv; v++) {
        double s = 0.0;
        for (int k = threadIdx.x; k < n; k += 1024) s += p[(size_t)k * nv + v];
        s = tree_sum_1024(s, sh);
        if (threadIdx.x == 0) out[v] = s;
    }
}
__global__ __launch_bounds__(1024) void k_reduce_sum(const double* __restrict__ p, int n, int nv,
                                                     double* __restrict__ out) {
    __shared__ double sh[1024];
    reduce_sum_body(p, n, nv, out, sh);
}

// nseg contiguous segments of n partials -> out[seg]: one launch instead of nseg, each segment
// summed exactly as k_reduce_sum (nv = 1) sums it
__global__ __launch_bounds__(1024) void k_reduce_sum_segs(const double* __restrict__ p, int n, int nseg,
                                                          double* __restrict__ out) {
    __shared__ double sh[1024];
    for (int g = 0; g < nseg; g++) {
        const double* q = p + (size_t)g * n;
        double s = 0.0;
        for (int k = threadIdx.x; k < n; k += 1024) s += q[k];
        s = tree_sum_1024(s, sh);
        if (threadIdx.x == 0) out[g] = s;
    }
}

__device__ __forceinline__ void reduce_min_body(const double* __restrict__ p, int n, int nv, double* __restrict__ out,
                                                double (*sh)[4]) {
    // all nv (<= 4) minima in one pass: per-thread registers, a wave's shuffles, the 16 waves'
    // results through LDS (2 barriers instead of 11 per value; fmin is order-independent)
    double m[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
    for (int k = threadIdx.x; k < n; k += 1024)
#pragma unroll
        for (int v = 0; v < 4; v++)
            if (v < nv) m[v] = fmin(m[v], p[(size_t)k * nv + v]);
#pragma unroll
    for (int v = 0; v < 4; v++)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) m[v] = fmin(m[v], __shfl_xor(m[v], off, 64));
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0)
#pragma unroll
        for (int v = 0; v < 4; v++) sh[wv][v] = m[v];
    __syncthreads();
    if (threadIdx.x < 4 && (int)threadIdx.x < nv) {
        double r = sh[0][threadIdx.x];
        for (int w = 1; w < 16; w++) r = fmin(r, sh[w][threadIdx.x]);
        out[threadIdx.x] = r;
    }
}
__global__ __launch_bounds__(1024) void k_reduce_min(const double* __restrict__ p, int n, int nv,
                                                     double* __restrict__ out) {
    __shared__ double sh[16][4];
    reduce_min_body(p, n, nv, out, sh);
}
// (r6) k_reduce_sum and k_reduce_min of two partial sets in one launch (workgroup 0 / 1): K1' leaves both
__global__ __launch_bounds__(1024) void k_reduce_sum_min(const double* __restrict__ ps, int ns, int nvs,
                                                         double* __restrict__ outs, const double* __restrict__ pm,
                                                         int nm, int nvm, double* __restrict__ outm) {
    __shared__ double sh[1024];
    if (blockIdx.x == 0) reduce_sum_body(ps, ns, nvs, outs, sh);
    else reduce_min_body(pm, nm, nvm, outm, reinterpret_cast<double (*)[4]>(sh));
}

// one rank: k_reduce_sum of the (sum, sum^2) partials and k_finish_mean in one launch (no
// all-reduce between them; the same arithmetic in the same order)
__global__ __launch_bounds__(1024) void k_reduce_sum_mean(const double* __restrict__ p, int n,
                                                          double* __restrict__ sums, double nc,
                                                          double* __restrict__ out) {
    __shared__ double sh[1024];
    double r[2];
    for (int v = 0; v < 2; v++) {
        double s = 0.0;
        for (int k = threadIdx.x; k < n; k += 1024) s += p[(size_t)k * 2 + v];
        r[v] = tree_sum_1024(s, sh);   // (thread 0's is the sum)
        if (threadIdx.x == 0) sums[v] = r[v];
    }
    if (threadIdx.x == 0) {
        const double s = r[0], s2 = r[1];
        out[0] = s / nc;
        out[1] = fmax(s2 - s * s / nc, 0.0);
    }
}
__global__ void k_finish_mean(const double* __restrict__ sums, double n, double* __restrict__ out) {
    const double s = sums[0], s2 = sums[1];
    out[0] = s / n;                 // MatNullSpaceRemove: subtract the plain mean (FluidSolver.cpp:550)
    out[1] = fmax(s2 - s * s / n, 0.0);  // ||rhs - mean||^2
}

// multi-rank scalar bus (r5, ns_solver.cpp bus()): g holds P rank slots of nv values each; value t
// of every slot is folded over the ranks in rank order -- a sum for t < nsum, a min after -- into
// out[dst[t]] (the same result on every rank, whatever the collective's internal order)
struct BusDst {
    int d[16];
};
__global__ void k_bus_reduce(const double* __restrict__ g, int P, int nv, int nsum, BusDst dst,
                             double* __restrict__ out) {
    const int t = threadIdx.x;
    if (t >= nv) return;
    double a = g[t];
    for (int q = 1; q < P; q++) {
        const double x = g[(size_t)q * nv + t];
        a = t < nsum ? a + x : fmin(a, x);
    }
    out[dst.d[t]] = a;
}

// (sum f, sum f^2) block partials over the slab's own cells
__global__ __launch_bounds__(256) void k_sums(Geo g, const double* __restrict__ f, double* __restrict__ part,
                                              int rows) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int lend = min((int)(blockIdx.y + 1) * 4 * rows, g.nxl);
    double acc[2] = {0.0, 0.0};
    for (int li = blockIdx.y * 4 * rows + threadIdx.y; li < lend && j < g.ny; li += 4) {
        const double x = ldf(f, g.ld, li, j);
        acc[0] += x;
        acc[1] += x * x;
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

// out = a x + b y (+ c z) over the slab's own cells (the Poisson initial-guess extrapolation)
__global__ __launch_bounds__(256) void k_axpby(Geo g, double a, const double* __restrict__ x, double b,
                                               const double* __restrict__ y, double c, const double* __restrict__ z,
                                               double d, const double* __restrict__ w, double e,
                                               const double* __restrict__ v, double* __restrict__ out) {
    // (one column per thread: 103.8 us per cubic guess at 4096^2 against 105.3 with 16-B loads and
    // stores and 110.5 with non-temporal 16-B stores, kernel traces gpurun_out/ab_trace)
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int li = blockIdx.y * 4 + threadIdx.y;
    if (j >= g.ny || li >= g.nxl) return;
    const ptrdiff_t o = (ptrdiff_t)li * g.ld + j;
    double r = extrap_comb(a, x[o], b, y[o], c, z, z ? z[o] : 0.0, d, w, w ? w[o] : 0.0);
    if (v) r = fma(e, v[o], r);
    out[o] = r;
}

// ------------------------------------------------ NEUMANN outflow: BiCGStab pieces
// With an outflow side the Poisson matrix is no longer the wall-closure L the smoothers
// relax: AddGhostStencils (FluidSolver.cpp:147-163) adds, per outflow face, w (ghost_p - x_c)
// with w = 1/h^2 (:124-127) and the ghost 2.5 x_c - 2 x_1 + 0.5 x_2 (:98-101) -- a row that
// reaches two cells inward and is not diagonally dominant.  The solver then runs BiCGStab on
// the true operator (the reference's KSPBCGSL, :73-82), right-preconditioned by one V-cycle
// of the wall-closure multigrid (ns_solver.cpp pois_solve_krylov).
//
// y = A x over own cells; block partials (sum y, sum q*y) (q may be null).
// OP 0: the Poisson matrix LHS_phi (ConstructLHS + AddGhostStencils, :105-163);
// OP 1: the Helmholtz matrix (I - alpha L_V) (:140-141) with L_V's boundary faces
//       w (wself q_c - q_c), wself = 1 (NEUMANN) / -1 (walls, inlets; ghost[0].weights, :87-99).
template <int OP, class T>
__global__ __launch_bounds__(256) void k_apply(Geo g, Coef c, double alpha, const double* __restrict__ x,
                                               double* __restrict__ y, const double* __restrict__ q,
                                               double* __restrict__ part, int rows, const double* stop) {
    if (stop && *stop != 0.0) return;   // (r5: a converged Krylov batch's remaining launches)
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int lend = min((int)(blockIdx.y + 1) * 4 * rows, g.nxl);
    double acc[2] = {0.0, 0.0};
    for (int li = blockIdx.y * 4 * rows + threadIdx.y; li < lend && j < g.ny; li += 4) {
        const T t(g, li, j);
        const int gi = g.i0 + li, ld = g.ld;
        const ptrdiff_t o = (ptrdiff_t)li * ld + j;
        if (!t.cell()) { y[o] = 0.0; continue; }
        const double xc = x[o], hx = c.hx[gi], hy = c.hy[j];
        const double w2[4] = {1.0 / (hx * hx), 1.0 / (hx * hx), 1.0 / (hy * hy), 1.0 / (hy * hy)};
        const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
        const double pn[4] = {c.pw[gi], c.pe[gi], c.ps[j], c.pn[j]};
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (t.in(di[k], dj[k])) {
                s += pn[k] * (x[o + di[k] * ld + dj[k]] - xc);
            } else {
                const EdgeDev E = t.edge(k);
                if (OP == 0) s += E.neu ? (ghost_p_e(g, E, x, li, j, xc) - xc) * w2[k] : 0.0;
                else s += E.neu ? 0.0 : -2.0 * xc * w2[k];
            }
        }
        const double val = OP == 0 ? s : xc - alpha * s;
        y[o] = val;
        acc[0] += val;
        if (q) acc[1] += q[o] * val;
    }
    block_reduce_sum<2>(acc, part + 2 * (blockIdx.x + gridDim.x * blockIdx.y));
}

// (r5) the masked domain's Helmholtz solve by red-black SOR (one rank; ns_solver.cpp helm_solve), k_apply<1, T>'s
// operator on x (rhs b) and, if x2 is not null, x2 (rhs b2) in the same pass -- the topology decoded once for u
// and v: par 0 / 1 relaxes the cells of that colour ((gi + j) parity) in place, x += omega (b - A x) / d, a
// half-sweep reading only the other colour, one thread per cell OF THAT COLOUR (j = 2 jx + parity); par 2 leaves
// x and writes the block partials of ||b - A x||^2 (and ||b2 - A x2||^2: 2 per block)
template <class T>
__global__ __launch_bounds__(256) void k_helm_rb_mask(Geo g, Coef c, double alpha, double omega, double* __restrict__ x,
                                                      const double* __restrict__ b, double* __restrict__ x2,
                                                      const double* __restrict__ b2, int par, double* __restrict__ part,
                                                      int rows) {
    const int jx = blockIdx.x * 64 + threadIdx.x;
    const int lend = min((int)(blockIdx.y + 1) * 4 * rows, g.nxl);
    double acc[2] = {0.0, 0.0};
    for (int li = blockIdx.y * 4 * rows + threadIdx.y; li < lend; li += 4) {
        const int gi = g.i0 + li, ld = g.ld;
        const int j = par < 2 ? 2 * jx + ((par + gi) & 1) : jx;
        if (j >= g.ny) continue;
        const T t(g, li, j);
        if (!t.cell()) continue;
        const ptrdiff_t o = (ptrdiff_t)li * ld + j;
        const double hx = c.hx[gi], hy = c.hy[j];
        const double w2[4] = {1.0 / (hx * hx), 1.0 / (hx * hx), 1.0 / (hy * hy), 1.0 / (hy * hy)};
        const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
        const double pn[4] = {c.pw[gi], c.pe[gi], c.ps[j], c.pn[j]};
        // the stencil as weights: A x = x - alpha (sum_k wk x_nb(k) - wc x_c), wk = 0 where the face has no neighbour
        double wk[4], wc = 0.0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            wk[k] = 0.0;
            if (t.in(di[k], dj[k])) {
                wk[k] = pn[k];
                wc += pn[k];
            } else if (!t.edge(k).neu) {
                wc += 2.0 * w2[k];
            }
        }
        const double dinv = omega / (1.0 + alpha * wc);
        auto relax = [&](double* __restrict__ xf, const double* __restrict__ bf, double& a) {
            const double xc = xf[o];
            double s = -wc * xc;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (wk[k] != 0.0) s = fma(wk[k], xf[o + di[k] * ld + dj[k]], s);
            const double r = bf[o] - (xc - alpha * s);
            if (par < 2) xf[o] = fma(dinv, r, xc);
            else a += r * r;
        };
        relax(x, b, acc[0]);
        if (x2) relax(x2, b2, acc[1]);
    }
    if (par == 2) block_reduce_sum<2>(acc, part + 2 * (blockIdx.x + gridDim.x * blockIdx.y));
}

// (r5) one whole red-black SOR sweep of k_helm_rb_mask's operator on u and v per launch, out of place (u, v ->
// uo, vo): a tile of RTM x 64 cells staged in LDS with a 2-cell ring; red relaxed over the tile and its 1-cell ring
// (the ring's red values the tile's black cells need), then black over the tile, from the same old values a
// red launch and a black launch would read -- the same arithmetic, half the launches and HBM passes
constexpr int RTM = 8;
__global__ __launch_bounds__(256) void k_helm_rbt_mask(Geo g, Coef c, double alpha, double omega,
                                                       const double* __restrict__ u, const double* __restrict__ v,
                                                       const double* __restrict__ bu, const double* __restrict__ bv,
                                                       double* __restrict__ uo, double* __restrict__ vo) {
    constexpr int EI = RTM + 4, EJ = 64 + 4, NQ = (EI * EJ + 255) / 256;
    __shared__ double su[EI][EJ], sv[EI][EJ];
    const int li0 = blockIdx.y * RTM, j0 = blockIdx.x * 64, ld = g.ld;
    const int tid = threadIdx.x + 64 * threadIdx.y;
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const int q = tid + 256 * k;
        if (q < EI * EJ) {
            const int r = q / EJ, cc = q - r * EJ;
            const int li = min(max(li0 - 2 + r, -HALO), g.nxl + HALO - 1);
            const int j = min(max(j0 - 2 + cc, 0), g.ny - 1);
            su[r][cc] = ldf(u, ld, li, j);
            sv[r][cc] = ldf(v, ld, li, j);
        }
    }
    // the 1-cell ring's codes and the tile's spacing / coefficient tables in LDS too
    constexpr int RI = RTM + 2, RJ = 66, NB = (RI * RJ + 255) / 256;
    __shared__ int scode[RI][RJ];
    __shared__ double trow[3][RI], tcol[3][RJ];   // hx, pw, pe of rows li0 - 1 ..; hy, ps, pn of columns j0 - 1 ..
#pragma unroll
    for (int k = 0; k < NB; k++) {
        const int q = tid + 256 * k;
        if (q < RI * RJ) {
            const int r = q / RJ, cc = q - r * RJ, li = li0 - 1 + r, j = j0 - 1 + cc;
            // (one rank: ring cells outside the slab are outside the box -- code 0)
            const bool ok = j >= 0 && j < g.ny && li >= -1 && li <= g.nxl;
            const ptrdiff_t o = (ptrdiff_t)li * ld + j;
            scode[r][cc] = ok ? g.fc[o] : 0;
        }
    }
    if (tid < RI) {
        const int gi = min(max(g.i0 + li0 - 1 + tid, 0), g.nx - 1);
        trow[0][tid] = c.hx[gi]; trow[1][tid] = c.pw[gi]; trow[2][tid] = c.pe[gi];
    } else if (tid >= 64 && tid < 64 + RJ) {
        const int k = tid - 64, j = min(max(j0 - 1 + k, 0), g.ny - 1);
        tcol[0][k] = c.hy[j]; tcol[1][k] = c.ps[j]; tcol[2][k] = c.pn[j];
    }
    __syncthreads();
    // relax the cell at ring coordinates (r1, c1) (LDS su / sv at (r1 + 1, c1 + 1)) if in the domain: k_helm_rb_mask's
    // arithmetic in its order
    auto relax = [&](int r1, int c1) {
        const int code = scode[r1][c1];
        if (!(code & FC_IN)) return;
        const double hx = trow[0][r1], hy = tcol[0][c1];
        const double w2[4] = {1.0 / (hx * hx), 1.0 / (hx * hx), 1.0 / (hy * hy), 1.0 / (hy * hy)};
        const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
        const double pn[4] = {trow[1][r1], trow[2][r1], tcol[1][c1], tcol[2][c1]};
        double wk[4], wc = 0.0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            wk[k] = 0.0;
            if (fc_edge(code, k) == FC_INT) {
                wk[k] = pn[k];
                wc += pn[k];
            } else if (!g.et[fc_edge(code, k)].neu) {
                wc += 2.0 * w2[k];
            }
        }
        const double dinv = omega / (1.0 + alpha * wc);
        const int R = r1 + 1, C = c1 + 1;
        auto one = [&](double (*sx)[EJ], double b) {
            const double xc = sx[R][C];
            double s = -wc * xc;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (wk[k] != 0.0) s = fma(wk[k], sx[R + di[k]][C + dj[k]], s);
            const double r = b - (xc - alpha * s);
            sx[R][C] = fma(dinv, r, xc);
        };
        // (the right-hand sides from global memory: staged too, the tile's 47 KB of LDS left 3 workgroups per CU and
        // the launch two rounds of them -- 26 us at 1024^2)
        const ptrdiff_t o = (ptrdiff_t)(li0 - 1 + r1) * ld + (j0 - 1 + c1);
        one(su, bu[o]);
        one(sv, bv[o]);
    };
    // red (colour 0) over rows li0 - 1 .. li0 + RTM, columns j0 - 1 .. j0 + 64: 33 red cells in each ring row, one
    // per thread
    for (int q = tid; q < RI * 33; q += 256) {
        const int r1 = q / 33, k = q - r1 * 33;
        relax(r1, 2 * k + ((g.i0 + li0 - 1 + r1 + j0 - 1) & 1));
    }
    __syncthreads();
    // black (colour 1) over the tile: 32 in each row
    for (int q = tid; q < RTM * 32; q += 256) {
        const int r = q >> 5, k = q & 31;
        if (li0 + r < g.nxl) relax(r + 1, 2 * k + ((g.i0 + li0 + r + j0 + 1) & 1) + 1);
    }
    const int j = j0 + threadIdx.x;
    __syncthreads();
    for (int r = threadIdx.y; r < RTM; r += 4) {
        const int li = li0 + r;
        if (li < g.nxl && j < g.ny) {
            const ptrdiff_t o = (ptrdiff_t)li * ld + j;
            uo[o] = su[r + 2][threadIdx.x + 2];
            vo[o] = sv[r + 2][threadIdx.x + 2];
        }
    }
}

// (r6) NSW whole red-black SOR sweeps of k_helm_rb_mask's operator on u and v in ONE launch (temporal blocking,
// k_helm_band's idea on the masked domain): a TI x 64 tile is staged with its R-cell cone (R = 2 NSW, + 1 with
// the residual) -- u, v and the cell codes in LDS, the right-hand sides read from global memory (L2) -- each
// half-sweep relaxes one colour over a region one ring smaller, so the tile's cells come out exactly as after NSW
// global sweeps, in the same arithmetic order as k_helm_rb_mask / k_helm_rbt_mask (bit-identical fields).  RES:
// the tile's residuals of both fields after the last sweep (k_helm_rb_mask par 2's expression) into part --
// the batch's check without a pass of its own.  One rank (the cone reaches R > HALO rows past the tile).
// Per NSW sweeps: u, v, code read ~(1 + 2R/TI)(1 + 2R/64) x 20 B + b 16 + write 16 -- against 52 B per sweep.
template <int NSW>
struct MtTile {   // (two workgroups per CU by LDS: 4 sweeps with the residual take 24-row tiles)
    static constexpr int TI = NSW >= 4 ? 24 : MT_TI, TJ = MT_TJ, NTH = 512;
};
// BAND (r6, the wall bands of a masked domain): only the cells flagged FC_BAND (within the band width of a
// boundary face along a row or column) are relaxed, the rest held; one workgroup per tile of the list `tiles`;
// band cells read from qbu / qbv, the others from u / v, and only band cells written (k_helm_band's scheme: two
// launches U -> TU, then (U, TU) -> U, no tile writes what another reads, no copy-back)
template <int NSW, bool RES, bool BAND>
__global__ __launch_bounds__(512) void k_helm_mt_mask(Geo g, Coef c, double alpha, double omega,
                                                       const double* __restrict__ u, const double* __restrict__ v,
                                                       const double* __restrict__ qbu, const double* __restrict__ qbv,
                                                       const double* __restrict__ bu, const double* __restrict__ bv,
                                                       double* __restrict__ uo, double* __restrict__ vo,
                                                       double* __restrict__ part, const int2* __restrict__ tiles) {
    constexpr int TI = MtTile<NSW>::TI, TJ = MtTile<NSW>::TJ, NTH = MtTile<NSW>::NTH;
    constexpr int R = 2 * NSW + (RES ? 1 : 0), EI = TI + 2 * R, EJ = TJ + 2 * R, NE = EI * EJ;
    // LDS: u, v, the codes, and per row hx, pw, pe, 1 / hx^2, per column hy, ps, pn, 1 / hy^2 (20 B per staged
    // cell: two workgroups per CU, one loading while the other relaxes -- with the weights staged too (36 B) one
    // workgroup per CU left the memory idle during its sweeps: 540 vs 3 x 194 us for 3 sweeps)
    extern __shared__ double smt[];
    double* su = smt;
    double* sv = smt + NE;
    double* trow = smt + 2 * NE;            // [4][EI]
    double* tcol = trow + 4 * EI;           // [4][EJ]
    int* sc = reinterpret_cast<int*>(tcol + 4 * EJ);
    int li0 = blockIdx.y * TI, j0 = blockIdx.x * TJ;
    if (BAND) {
        const int2 t = tiles[blockIdx.x];
        li0 = t.x;
        j0 = t.y;
    }
    const int ld = g.ld;
    const int tid = threadIdx.x;
    // the cells this launch relaxes
    auto live = [](int code) { return (code & FC_IN) && (!BAND || (code & FC_BAND)); };
    // the edge tags' NEUMANN flags as a mask (the table is padded to 32 entries)
    const unsigned long long neub = __ballot((tid & 63) < 32 && g.et[tid & 31].neu != 0);
    const unsigned neum = (unsigned)neub;
    const int base = (g.i0 + li0 - R + j0 - R) & 1;   // colour of staged (0, 0)
    // staging: every load of the thread's cells issued before the first LDS store (one memory round trip, not
    // one per cell: with one workgroup per CU nothing else hides it)
    constexpr int NQ = (NE + NTH - 1) / NTH;
    double lu[NQ], lv[NQ], lbu[BAND ? NQ : 1], lbv[BAND ? NQ : 1];
    int lc[NQ];
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const int q = min(tid + k * NTH, NE - 1);
        const int r = q / EJ, cc = q - r * EJ;
        const int li = li0 - R + r, j = j0 - R + cc;
        const bool in = li >= 0 && li < g.nxl && j >= 0 && j < g.ny;
        const ptrdiff_t o = (ptrdiff_t)min(max(li, -HALO), g.nxl + HALO - 1) * ld + min(max(j, 0), g.ny - 1);
        lc[k] = in ? g.fc[o] : 0;   // (one rank: cells off the slab are off the box)
        lu[k] = u[o];
        lv[k] = v[o];
        if (BAND) {   // (both planes: the select waits for the code)
            lbu[BAND ? k : 0] = qbu[o];
            lbv[BAND ? k : 0] = qbv[o];
        }
    }
    // the right-hand sides of a half-sweep's cells are loaded one half-sweep ahead (a load per half-sweep, behind
    // a barrier, would expose its latency 2 NSW times)
    constexpr int MAXIT = ((EI - 2) * (EJ - 2) / 2 + EI + NTH - 1) / NTH;
    double pbu[MAXIT], pbv[MAXIT];
    auto load_b = [&](int h) {
        const int par = h & 1, lo = h + 1, hr = EI - 2 - h, hc = EJ - 2 - h;
        const int npr = (hc - lo) / 2 + 1, cnt = (hr - lo + 1) * npr;
#pragma unroll
        for (int it = 0; it < MAXIT; it++) {
            const int q = tid + it * NTH;
            const int rq = q / npr, r = lo + rq;
            const int cc = min(lo + ((par + base + r + lo) & 1) + 2 * (q - rq * npr), hc);
            const int li = min(max(li0 - R + r, 0), g.nxl - 1), j = min(max(j0 - R + cc, 0), g.ny - 1);
            const ptrdiff_t o = (ptrdiff_t)li * ld + j;
            pbu[it] = q < cnt ? bu[o] : 0.0;
            pbv[it] = q < cnt ? bv[o] : 0.0;
        }
    };
    load_b(0);
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const int q = tid + k * NTH;
        if (q >= NE) continue;
        const bool fb = BAND && (lc[k] & FC_BAND);
        su[q] = fb ? lbu[BAND ? k : 0] : lu[k];
        sv[q] = fb ? lbv[BAND ? k : 0] : lv[k];
        sc[q] = lc[k];
    }
    if (tid < EI) {
        const int gi = min(max(g.i0 + li0 - R + tid, 0), g.nx - 1);
        const double hx = c.hx[gi];
        trow[tid] = hx; trow[EI + tid] = c.pw[gi]; trow[2 * EI + tid] = c.pe[gi]; trow[3 * EI + tid] = 1.0 / (hx * hx);
    } else if (tid >= 128 && tid < 128 + EJ) {
        const int k = tid - 128, j = min(max(j0 - R + k, 0), g.ny - 1);
        const double hy = c.hy[j];
        tcol[k] = hy; tcol[EJ + k] = c.ps[j]; tcol[2 * EJ + k] = c.pn[j]; tcol[3 * EJ + k] = 1.0 / (hy * hy);
    }
    __syncthreads();
    // k_helm_rb_mask's weights in its order: the off-diagonal of face k is its coefficient when the face is
    // interior, else 0 (a wall's 2 / h^2 goes to the diagonal unless NEUMANN)
    auto pn_of = [&](int k, int r, int cc) {
        return k == 0 ? trow[EI + r] : k == 1 ? trow[2 * EI + r] : k == 2 ? tcol[EJ + cc] : tcol[2 * EJ + cc];
    };
    // (branch-free: a term that k_helm_rb_mask skips is added as an exact 0 here -- wc + 0.0 and
    // fma(0.0, x, s) leave the sums' values unchanged, so the result is the same bit for bit -- and every
    // neighbour is loaded: the iterations of a half-sweep interleave instead of waiting on each other)
    auto wsum = [&](int code, int r, int cc, double (&pk)[4]) {
        const double w2[4] = {trow[3 * EI + r], trow[3 * EI + r], tcol[3 * EJ + cc], tcol[3 * EJ + cc]};
        double wc = 0.0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int e = fc_edge(code, k);
            const double p = pn_of(k, r, cc);
            pk[k] = e == FC_INT ? p : 0.0;
            wc += e == FC_INT ? p : (((neum >> e) & 1u) ? 0.0 : 2.0 * w2[k]);
        }
        return wc;
    };
    // the residual b - (I - alpha L_V) x at staged cell x (row r, column cc)
    auto resid = [&](const double* sx, int x, const double (&pk)[4], double wc, double b) {
        const double xc = sx[x];
        double s = -wc * xc;
        const int nb[4] = {x - EJ, x + EJ, x - 1, x + 1};
#pragma unroll
        for (int k = 0; k < 4; k++) s = fma(pk[k], sx[nb[k]], s);
        return b - (xc - alpha * s);
    };
#pragma unroll
    for (int h = 0; h < 2 * NSW; h++) {
        const int par = h & 1, lo = h + 1, hr = EI - 2 - h, hc = EJ - 2 - h;
        const int npr = (hc - lo) / 2 + 1, cnt = (hr - lo + 1) * npr;
        double cbu[MAXIT], cbv[MAXIT];
#pragma unroll
        for (int it = 0; it < MAXIT; it++) { cbu[it] = pbu[it]; cbv[it] = pbv[it]; }
        if (h + 1 < 2 * NSW) load_b(h + 1);
#pragma unroll
        for (int it = 0; it < MAXIT; it++) {
            const int q = tid + it * NTH;
            const int rq = min(q / npr, hr - lo), k = q - (q / npr) * npr, r = lo + rq;
            const int cc0 = lo + ((par + base + r + lo) & 1) + 2 * k;
            const int cc = min(cc0, hc);
            const int x = r * EJ + cc, code = sc[x];
            double pk[4];
            const double wc = wsum(code, r, cc, pk);
            const double di = omega / (1.0 + alpha * wc), xu = su[x], xv = sv[x];
            const double ru = resid(su, x, pk, wc, cbu[it]), rv = resid(sv, x, pk, wc, cbv[it]);
            if (q < cnt && cc0 <= hc && live(code)) {
                su[x] = fma(di, ru, xu);
                sv[x] = fma(di, rv, xv);
            }
        }
        __syncthreads();
    }
    double acc[2] = {0.0, 0.0};
    for (int q = tid; q < TI * TJ; q += NTH) {
        const int r = q / TJ, cc = q - r * TJ, li = li0 + r, j = j0 + cc;
        if (li >= g.nxl || j >= g.ny) continue;
        const int x = (r + R) * EJ + cc + R;
        const ptrdiff_t o = (ptrdiff_t)li * ld + j;
        if (BAND && !live(sc[x])) continue;
        uo[o] = su[x];
        vo[o] = sv[x];
        if (RES) {
            const int code = sc[x];
            if (code & FC_IN) {
                double pk[4];
                const double wc = wsum(code, r + R, cc + R, pk);
                const double ru = resid(su, x, pk, wc, bu[o]);
                const double rv = resid(sv, x, pk, wc, bv[o]);
                acc[0] += ru * ru;
                acc[1] += rv * rv;
            }
        }
    }
    if (RES) block_reduce_sum<2>(acc, part + 2 * (blockIdx.x + gridDim.x * blockIdx.y));
}

// z = q / diag(A) (the Jacobi preconditioner of the masked-domain Krylov solves; the
// outflow rows' diagonal -(sum p) + 1.5 w, oracle diag_poisson / diag_helmholtz)
template <int OP, class T>
__global__ __launch_bounds__(256) void k_diag_pc(Geo g, Coef c, double alpha, const double* __restrict__ qv,
                                                 double* __restrict__ z, const double* stop) {
    if (stop && *stop != 0.0) return;
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int li = blockIdx.y * 4 + threadIdx.y;
    if (j >= g.ny || li >= g.nxl) return;
    const T t(g, li, j);
    const ptrdiff_t o = (ptrdiff_t)li * g.ld + j;
    if (!t.cell()) { z[o] = 0.0; return; }
    const int gi = g.i0 + li;
    const double hx = c.hx[gi], hy = c.hy[j];
    const double w2[4] = {1.0 / (hx * hx), 1.0 / (hx * hx), 1.0 / (hy * hy), 1.0 / (hy * hy)};
    const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
    const double pn[4] = {c.pw[gi], c.pe[gi], c.ps[j], c.pn[j]};
    double d = 0.0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (t.in(di[k], dj[k])) d -= pn[k];
        else if (OP == 0) d += t.edge(k).neu ? 1.5 * w2[k] : 0.0;
        else d -= t.edge(k).neu ? 0.0 : 2.0 * w2[k];
    }
    if (OP == 1) d = 1.0 - alpha * d;
    z[o] = d != 0.0 ? qv[o] / d : qv[o];
}

// BiCGStab vector updates; coefficients from the device scalars k_bicg_scal leaves in sc,
// each fused with the dot products the next scalar stage needs (block partials, 3 per block):
//   KV_INIT: r = (b - shift) - (y - mean_y), r0 = r, p = v = 0     partials (r.r, r0.r, sum r)
//   KV_P:    p = r + beta (p - omega v)
//   KV_V:    v = y - mean_y (in place), s = r - alpha v
//   KV_T:    t = y - mean_y (in place)                             partials (t.s, t.t, -)
//   KV_X:    x += alpha ph + omega sh, r = s - omega t             partials (r.r, r0.r, sum r)

template <int MODE>
__global__ __launch_bounds__(256) void k_bicg_vec(KrylovArgs a) {
    if (a.sc[KS_STOP] != 0.0) return;   // (r5: frozen -- the partials stay unread, every scalar stage is frozen too)
    const Geo& g = a.g;
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int lend = min((int)(blockIdx.y + 1) * 4 * a.rows, g.nxl);
    double acc[3] = {0.0, 0.0, 0.0};
    const double alpha = a.sc[KS_ALPHA], beta = a.sc[KS_BETA], omega = a.sc[KS_OMEGA], my = a.sc[KS_MEAN];
    const double shift = a.shift ? a.shift[0] : 0.0;
    for (int li = blockIdx.y * 4 * a.rows + threadIdx.y; li < lend && j < g.ny; li += 4) {
        const ptrdiff_t o = (ptrdiff_t)li * g.ld + j;
        // outside a masked domain: every vector stays 0 (kv planes zeroed at ns_create, never written
        // here).  Invariant the box preconditioners rely on (fps_precond, ns_solver.cpp): the vectors they
        // are handed -- p and s -- are mean-free over the domain (the mean projection below) and exactly
        // 0 outside it, so the bounding box's singular mode 0 sees a consistent right-hand side
        if (g.fc && !(g.fc[o] & FC_IN)) continue;
        if (MODE == KV_INIT) {
            const double r = (a.b[o] - shift) - (a.v[o] - my);
            a.r[o] = r; a.r0[o] = r; a.p[o] = 0.0; a.v[o] = 0.0;
            acc[0] += r * r; acc[1] += r * r; acc[2] += r;
        } else if (MODE == KV_P) {
            a.p[o] = a.r[o] + beta * (a.p[o] - omega * a.v[o]);
        } else if (MODE == KV_V) {
            const double v = a.v[o] - my;
            a.v[o] = v;
            a.s[o] = a.r[o] - alpha * v;
        } else if (MODE == KV_T) {
            const double t = a.t[o] - my;
            a.t[o] = t;
            acc[0] += t * a.s[o]; acc[1] += t * t;
        } else {
            a.x[o] += alpha * a.ph[o] + omega * a.sh[o];
            const double r = a.s[o] - omega * a.t[o];
            a.r[o] = r;
            acc[0] += r * r; acc[1] += a.r0[o] * r; acc[2] += r;
        }
    }
    if (MODE == KV_INIT || MODE == KV_T || MODE == KV_X)
        block_reduce_sum<3>(acc, a.part + 3 * (blockIdx.x + gridDim.x * blockIdx.y));
}

// the scalar recurrences of BiCGStab on one thread; d = the stage's reduced sums
//   KSC_RHO  (d = r.r, r0.r, sum r):   beta = (rho1/rho)(alpha/omega), rho = rho1
//   KSC_ALPHA (d = sum y, r0.y):       mean_y, alpha = rho / (r0.y - mean_y sum r0)
//   KSC_MEAN  (d = sum y):             mean_y
//   KSC_OMEGA (d = t.s, t.t):          omega = t.s / t.t
//   KSC_CHECK (d = r.r, ...):          the convergence test of the host loop's head (r5), in its order: divergence
//                                      (non-finite, or 1e16 b2), convergence (<= tol^2 b2, = 0), the cap, a breakdown
//   KSC_RESET:                         a restart after a breakdown (KS_STOP, KS_BRK cleared)
__global__ void k_bicg_scal(int stage, const double* __restrict__ d, double n, double* __restrict__ sc, double thr,
                            double b2, int maxit) {
    // a breakdown (a zero or non-finite denominator) zeroes the coefficient -- the vector
    // updates then leave x untouched -- and raises KS_BRK; the host restarts from x
    auto guard = [&](double v) {
        if (!isfinite(v)) { sc[KS_BRK] = 1.0; return 0.0; }
        return v;
    };
    if (stage == KSC_RESET) {
        sc[KS_STOP] = 0.0;
        sc[KS_BRK] = 0.0;
        if (maxit >= 0) {   // (a solve's start)
            sc[KS_IT] = 0.0; sc[KS_THR] = thr; sc[KS_B2] = b2; sc[KS_MAXIT] = maxit;
        }
        return;
    }
    if (sc[KS_STOP] != 0.0) return;
    if (stage == KSC_CHECK) {
        const double r2 = d[0], bb = sc[KS_B2];
        const bool stop = !isfinite(r2) || (bb > 0 && r2 > 1e16 * bb) || r2 <= sc[KS_THR] || r2 == 0.0 ||
                          sc[KS_IT] >= sc[KS_MAXIT] || sc[KS_BRK] != 0.0;
        if (stop) {
            sc[KS_STOP] = 1.0;
            sc[KS_R2] = r2;
        }
        return;
    }
    if (stage == KSC_INIT) {
        sc[KS_RHO] = 1.0; sc[KS_ALPHA] = 1.0; sc[KS_OMEGA] = 1.0; sc[KS_SUMR0] = d[2]; sc[KS_BRK] = 0.0;
    } else if (stage == KSC_RHO) {
        const double rho1 = d[1];
        sc[KS_BETA] = guard((rho1 / sc[KS_RHO]) * (sc[KS_ALPHA] / sc[KS_OMEGA]));
        if (rho1 == 0.0) sc[KS_BRK] = 1.0;
        sc[KS_RHO] = rho1;
    } else if (stage == KSC_ALPHA) {
        const double m = d[0] / n;
        sc[KS_MEAN] = m;
        sc[KS_ALPHA] = guard(sc[KS_RHO] / (d[1] - m * sc[KS_SUMR0]));
    } else if (stage == KSC_MEAN) {
        sc[KS_MEAN] = d[0] / n;
    } else {
        const double om = d[1] > 0.0 ? d[0] / d[1] : 0.0;
        sc[KS_OMEGA] = guard(om);
        if (om == 0.0) sc[KS_BRK] = 1.0;
        sc[KS_IT] += 1.0;   // (the iteration's last scalar stage)
    }
}

// ------------------------------------------------ stretched grids: a consistent Poisson rhs
// The Poisson operator conserves area-weighted sums (sum_c A_c (L phi)_c = 0 at walls and
// inlets), so L phi = b is solvable only if sum_c A_c b_c = 0.  div(u*) satisfies that, but the
// reference's PLAIN mean removal (MatNullSpaceRemove, FluidSolver.cpp:550) breaks it on a
// stretched grid and leaves its Krylov solve an inconsistent system.  The oracle's PCG
// converges to the area-projected solution (b - shift) - m / A_c with
// m = sum_c A_c (b_c - shift) / N; these two passes move the rhs there (in place; the shift
// stays the plain mean), so every solver sees a consistent system with that same solution.
__global__ __launch_bounds__(256) void k_area_sum(Geo g, Coef c, const double* __restrict__ b,
                                                  double* __restrict__ part, int rows) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int lend = min((int)(blockIdx.y + 1) * 4 * rows, g.nxl);
    double acc[1] = {0.0};
    for (int li = blockIdx.y * 4 * rows + threadIdx.y; li < lend && j < g.ny; li += 4)
        acc[0] += (c.hx[g.i0 + li] * c.hy[j]) * b[(ptrdiff_t)li * g.ld + j];   // 0 outside a mask
    block_reduce_sum<1>(acc, part + (blockIdx.x + gridDim.x * blockIdx.y));
}
// b_c -= m / A_c, m = (sum A b - shift * sum A) / N from the reduced sum sab and the shift;
// kshift = shift + mean(b - shift) afterwards = shift - m sum(1/A) / N (the mean-free shift of
// the Krylov solves; the plain mean of b - shift was 0 before the fix)
__global__ __launch_bounds__(256) void k_area_fix(Geo g, Coef c, double* __restrict__ b,
                                                  const double* __restrict__ sab, const double* __restrict__ shift,
                                                  double area, double inv_area, double n, double* __restrict__ kshift) {
    const int j = blockIdx.x * 64 + threadIdx.x;
    const int li = blockIdx.y * 4 + threadIdx.y;
    const double m = (sab[0] - shift[0] * area) / n;
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && threadIdx.y == 0) kshift[0] = shift[0] - m * inv_area / n;
    if (j >= g.ny || li >= g.nxl) return;
    const ptrdiff_t o = (ptrdiff_t)li * g.ld + j;
    if (g.fc && !(g.fc[o] & FC_IN)) return;
    b[o] -= m * (c.rhx[g.i0 + li] * c.rhy[j]);
}

// ---------------------------------------------------------------- launchers
static inline dim3 cell_grid(const Geo& g) { return dim3((g.ny + 63) / 64, (g.nxl + 3) / 4); }

// cell kernels walk `rows` 4-row groups per 64 x 4 block: one block reduction (and one
// partial) per 64 x 4*rows cells instead of per 256; still >= 2048 blocks per launch
static inline int cell_rows(const Geo& g) {
    const long blocks = (long)((g.ny + 63) / 64) * ((g.nxl + 3) / 4);
    return (int)std::min(16L, std::max(1L, blocks / 2048));
}
static inline dim3 cell_grid(const Geo& g, int rows) {
    return dim3((g.ny + 63) / 64, (g.nxl + 4 * rows - 1) / (4 * rows));
}

int max_partials(const Geo& g) {
    const dim3 cg = cell_grid(g);
    int n = (int)(cg.x * cg.y) * 4;
    const int tiles = ((g.nxl + 7) / 8) * ((g.ny + 63) / 64) * 2;   // tiled sweeps
    const int strips = ((g.nxl + 3) / 4) * ((g.ny + 115) / 116) * 2;  // streaming sweeps, strip rows >= 4
    return std::max(n, std::max(tiles, strips));
}

}  // namespace nsg

namespace nsg {

// Kernel timing with the dispatch's own timestamps: time_next_launch(a, b) makes the next launch
// go through hipExtLaunchKernel with start / stop events a, b, which the runtime stamps at the
// kernel's begin and end (the same interval rocprofv3's kernel trace reports).  HIP marker
// events recorded around a launch also count its dispatch latency (~3 us at 4096^2).
static thread_local hipEvent_t g_tev[2] = {nullptr, nullptr};
void time_next_launch(hipEvent_t a, hipEvent_t b) { g_tev[0] = a; g_tev[1] = b; }
bool time_next_launch_pending() {
    const bool p = g_tev[0] != nullptr;
    g_tev[0] = g_tev[1] = nullptr;
    return p;
}
bool take_launch_timing(hipEvent_t& a, hipEvent_t& b) {
    if (!g_tev[0]) return false;
    a = g_tev[0];
    b = g_tev[1];
    g_tev[0] = g_tev[1] = nullptr;
    return true;
}
#define NS_LAUNCH(kern, grid, block, shmem, st, ...)                                                     \
    do {                                                                                              \
        if (::nsg::g_tev[0]) {                                                                        \
            hipExtLaunchKernelGGL(kern, grid, block, shmem, st, ::nsg::g_tev[0], ::nsg::g_tev[1], 0, __VA_ARGS__); \
            ::nsg::g_tev[0] = ::nsg::g_tev[1] = nullptr;                                              \
        } else {                                                                                      \
            hipLaunchKernelGGL(kern, grid, block, shmem, st, __VA_ARGS__);                            \
        }                                                                                             \
    } while (0)
static hipError_t launch_raw(const void* k, dim3 grid, dim3 block, void** args, size_t shmem, hipStream_t st) {
    if (g_tev[0]) {
        const hipError_t e = hipExtLaunchKernel(k, grid, block, args, shmem, st, g_tev[0], g_tev[1], 0);
        g_tev[0] = g_tev[1] = nullptr;
        return e;
    }
    return hipLaunchKernel(k, grid, block, args, shmem, st);
}

static long resident_waves(const void* k);
static int strip_rows(int nxl, long nsj, long cap, int lmin, int lmax = 64);

int launch_rhs(const Geo& g, const Coef& c, double dt, double re, const double* u, const double* v,
               const double* phi, double* cu, double* cv, double* ru, double* rv, double* part, hipStream_t st,
               int depth, double* uo, double* vo, double* mm) {
    const char* e = getenv("NSGPU_RHS");   // NSGPU_RHS=global: the global-load K1 (A/B)
    // (r6) uo: the previous step's correction folded in (k_rhs_sc) -- the streaming kernel only, rectangles without
    // NEUMANN sides, hy uniform (the solver asks for it only there)
    if (uo && (e || g.fc || !c.yuni || g.neu[0] || g.neu[1] || g.neu[2] || g.neu[3])) return -1;
    // (the grid kernels cannot split: the interior phase launches nothing, the edge phase all;
    // K1 updates cu / cv in place, so no cell may run twice)
    if (g.fc) {   // masked domain: the grid kernel with the polygon's topology
        if (e && std::strcmp(e, "global") == 0) {   // (A/B: r1-r4's global-load kernel)
            const int rows = cell_rows(g);
            const dim3 cg = cell_grid(g, rows);
            if (g_phase != 1)
                NS_LAUNCH(k_rhs<TopoMask>, cg, dim3(64, 4), 0, st, g, c, dt, re, u, v, phi, cu, cv, ru, rv, part, rows);
            return (int)(cg.x * cg.y);
        }
        // (r5) LDS tiles for the FC_DEEP cells (k_rhs_lds<true>), then the listed others (k_rhs_cells); the whole
        // slab in one pass (no phase split, as above)
        const int nti = (g.nxl + RT - 1) / RT, nb = ((g.ny + 63) / 64) * nti, ne = (g.necell + 255) / 256;
        if (g_phase != 1) {
            NS_LAUNCH(k_rhs_lds<true>, dim3((g.ny + 63) / 64, nti), dim3(64, 4), 0, st, g, c, dt, re, u, v, phi, cu, cv,
                      ru, rv, part, nti, nti);
            if (ne > 0) NS_LAUNCH(k_rhs_cells, dim3(ne), dim3(256), 0, st, g, c, dt, re, u, v, phi, cu, cv, ru, rv,
                                  part + 2 * nb);
        }
        return nb + ne;
    }
    if (!e) {
        // the streaming inner kernel (k_rhs_s) with its wall ring (extra workgroups of the same launch)
        RhsStreamArgs A{};
        A.g = g; A.c = c; A.dt = dt; A.re = re; A.u = u; A.v = v; A.phi = phi; A.cu = cu; A.cv = cv; A.ru = ru;
        A.rv = rv; A.part = part;
        A.uo = uo; A.vo = vo; A.mm = mm;
        A.jhi = std::max(2, (g.ny - 2) & ~1);
        A.ilo = std::max(0, std::min(2 - g.i0, g.nxl));
        A.ihi = std::max(A.ilo, std::min(g.nx - 2 - g.i0, g.nxl));
        A.nsj = (g.ny + SW - 1) / SW;
        const char* w3 = getenv("NSGPU_K1S");
        const int kv = w3 ? std::atoi(w3) : 0;
        // (r5) uniform hy: k_rhs_su, the column tables in SGPRs -- 164 VGPRs, three waves per SIMD, no spill
        // (NSGPU_K1S=32; 33: three rows in flight, spills).  Measured slower (driver form, interleaved:
        // 243-246 us vs k_rhs_s's 230 us; profiles/r05/k1_waves.log): K1 moves its bytes at ~0.8 of the
        // measured HBM copy rate already (4 streams read, 4 written), more waves only shorten the strips
        const bool uy = c.yuni && (kv == 32 || kv == 33);
        const void* kk = uo ? (const void*)k_rhs_sc<true, 2>
                       : uy ? (kv == 33 ? (const void*)k_rhs_su<true, 3> : (const void*)k_rhs_su<true, 2>)
                       : kv == 3 ? (const void*)k_rhs_s3<true>
                       : kv == 24 ? (const void*)k_rhs_s<true, 4> : (const void*)k_rhs_s<true, 2>;
        {
            // the fewest rows that keep every strip in ONE resident round (strip_rows caps at 64:
            // 4096^2 at 2 waves / SIMD then left 128 of 2176 strips to a second round)
            const long nsi = std::max(1L, resident_waves(kk) / A.nsj);
            int L = std::min(std::max((int)((g.nxl + nsi - 1) / nsi + 1) & ~1, 8), K1_LMAX);
            // (r6, A/B) NSGPU_K1_L: rows per strip (several resident rounds of shorter strips)
            static const int k1l = getenv("NSGPU_K1_L") ? std::atoi(getenv("NSGPU_K1_L")) : 0;
            if (k1l >= 4) L = std::min(k1l & ~1, K1_LMAX);
            A.nstr = A.nsj * plan_rows(g.nxl, L, depth, &A.P, K1_ESPLIT);   // u, v rows ib-2 .. ie+1
        }
        const bool inner = A.jhi > 2 && A.ihi > A.ilo;
        if (!inner) A.P.nrun = 0;
        RhsRingArgs& R = A.R;
        R.jhi = A.jhi;
        for (int li = 0; li < g.nxl; li++)
            if ((li < A.ilo || li >= A.ihi) && R.nfull < 4) R.fr[R.nfull++] = li;
        R.rlo = A.ilo;
        R.rhi = A.ihi;
        R.ncol = A.jhi <= 2 ? g.ny : 2 + (g.ny - A.jhi);   // (tiny grids: whole rows)
        R.n = R.nfull * g.ny + (R.rhi - R.rlo) * R.ncol;
        const int nring = (R.n + 255) / 256;
        // the ring reads phi's and u, v's ghost rows (wall terms, MUSCL): with the edge phase
        A.nring = g_phase != 1 ? nring : 0;
        A.nsblk = (A.nsj * A.P.nrun + 3) / 4;
        if (!inner && g_phase != 1) {
            (void)hipMemsetAsync(part, 0, 2 * sizeof(double) * A.nstr, st);   // (no inner cells: zero partials)
            if (mm) {   // (min / max partials of no cell: +inf)
                static const std::vector<double> inf(4 * 4096, INFINITY);
                if (4 * (size_t)A.nstr > inf.size()) return -1;
                (void)hipMemcpyAsync(mm, inf.data(), 4 * sizeof(double) * A.nstr, hipMemcpyHostToDevice, st);
            }
        }
        if (A.nsblk + A.nring > 0) {
            void* args[] = {&A};
            if (launch_raw(kk, dim3(A.nsblk + A.nring), dim3(256), args, 0, st) != hipSuccess) return -1;
        }
        return A.nstr + nring;
    }
    if (std::strcmp(e, "global") != 0) {   // NSGPU_RHS=lds: the LDS-tiled K1 (A/B)
        const int nti = (g.nxl + RT - 1) / RT;
        int tlo, thi0;
        const int nrun = phase_range(g.nxl, RT, nti, 2, &tlo, &thi0);   // MUSCL: rows li0-2 .. li0+RT+1
        const int nb = ((g.ny + 63) / 64) * nti;
        if (nrun > 0)
            NS_LAUNCH(k_rhs_lds<false>, dim3((g.ny + 63) / 64, nrun), dim3(64, 4), 0, st, g, c, dt, re, u, v, phi,
                               cu, cv, ru, rv, part, tlo, thi0);
        const int nbc = (2 * g.nxl + 2 * g.ny + 255) / 256;
        // the wall terms read phi's ghost rows: with the edge phase
        if (g_phase != 1)
            NS_LAUNCH(k_rhs_bc, dim3(nbc), dim3(256), 0, st, g, c, dt, re, phi, ru, rv, part + 2 * nb);
        return nb + nbc;
    }
    const int rows = cell_rows(g);
    const dim3 cg = cell_grid(g, rows);
    if (g_phase != 1)
        NS_LAUNCH(k_rhs<TopoRect>, cg, dim3(64, 4), 0, st, g, c, dt, re, u, v, phi, cu, cv, ru, rv, part, rows);
    return (int)(cg.x * cg.y);
}

template <int K>
static int launch_cell_s(CellStreamArgs A, hipStream_t st) {
    A.nsj = (A.g.ny + SW - 1) / SW;
    const int L = strip_rows(A.g.nxl, A.nsj, resident_waves((const void*)k_cell_s<K>), 4);
    int nstr;
    if (K == 3) {
        // K3's (sum, sum^2) partials set the null-space mean (values, not just a norm): the same
        // strips in both overlap phases (phase_range), so the overlapped exchange stays bit-identical
        const int nsi = (A.g.nxl + L - 1) / L;
        int lo = 0, hi0 = 0;
        const int nrun = phase_range(A.g.nxl, L, nsi, 1, &lo, &hi0);
        A.P.L = L; A.P.rb0 = 0; A.P.rend = A.P.rend0 = A.g.nxl;
        A.P.nrun = nrun;
        A.P.slo = lo;
        A.P.rb1 = hi0 * L;   // launch strip row k >= lo is strip row hi0 + (k - lo)
        A.P.pbase = -1;      // (partial slots: that strip-row numbering)
        nstr = A.nsj * nsi;
    } else {
        nstr = A.nsj * plan_rows(A.g.nxl, L, 1, &A.P);   // window rows ib-1 .. ie
    }
    if (A.P.nrun > 0) NS_LAUNCH(k_cell_s<K>, dim3((A.nsj * A.P.nrun + 3) / 4), dim3(256), 0, st, A);
    return nstr;
}

static bool cell_streaming() {
    const char* e = getenv("NSGPU_CELL");   // NSGPU_CELL=grid: the thread-per-cell K3 / K5 (A/B)
    return !(e && std::strcmp(e, "grid") == 0);
}

// (r6) a masked domain on one rank: the streaming K3 / K5 on its FC_DEEP cells + the listed cells (NSGPU_MASK_CELL=0:
// the thread-per-cell k_div / k_correct<TopoMask>)
static bool mask_cell_streams(const Geo& g) {
    const char* e = getenv("NSGPU_MASK_CELL");   // (read per launch: the tests switch it)
    const bool on = !(e && std::atoi(e) == 0);
    return on && g.fc && g.ecell && g.nxl == g.nx && cell_streaming();
}

int launch_div(const Geo& g, const Coef& c, double dt, const double* u, const double* v, double* rp, double* part,
               hipStream_t st) {
    if (cell_streaming() && !g.fc) {
        CellStreamArgs A{};
        A.g = g; A.c = c; A.dt = dt; A.a0 = u; A.a1 = v; A.o0 = rp; A.part = part;
        return launch_cell_s<3>(A, st);
    }
    if (mask_cell_streams(g)) {
        // (an overlapped exchange's interior phase launches nothing: all of it with the edge phase, whole -- the
        // same launches as without the exchange, so a loopback / slab run matches one rank bit for bit)
        if (g_phase == 1) return 0;
        const int ph = g_phase;
        g_phase = 0;
        CellStreamArgs A{};
        A.g = g; A.c = c; A.dt = dt; A.a0 = u; A.a1 = v; A.o0 = rp; A.part = part; A.fc = g.fc;
        const int n1 = launch_cell_s<3>(A, st);
        const int n2 = (g.necell + 255) / 256;
        NS_LAUNCH(k_div_cells, dim3(n2), dim3(256), 0, st, g, c, dt, u, v, rp, part + 2 * n1);
        g_phase = ph;
        return n1 + n2;
    }
    const int rows = cell_rows(g);
    const dim3 cg = cell_grid(g, rows);
    if (g_phase == 1) return (int)(cg.x * cg.y);   // (cannot split: all with the edge phase)
    if (g.fc) NS_LAUNCH(k_div<TopoMask>, cg, dim3(64, 4), 0, st, g, c, dt, u, v, rp, part, rows);
    else NS_LAUNCH(k_div<TopoRect>, cg, dim3(64, 4), 0, st, g, c, dt, u, v, rp, part, rows);
    return (int)(cg.x * cg.y);
}

int launch_apply(int op, const Geo& g, const Coef& c, double alpha, const double* x, double* y, const double* q,
                 double* part, hipStream_t st, const double* stop) {
    const char* ae = getenv("NSGPU_APPLY");   // NSGPU_APPLY=grid: k_apply only (A/B)
    if (op == 0 && !g.fc && cell_streaming() && !(ae && std::strcmp(ae, "grid") == 0)) {
        CellStreamArgs A{};
        A.g = g; A.c = c; A.a0 = x; A.a1 = q; A.o0 = y; A.part = part;
        return launch_cell_s<7>(A, st);
    }
    const int rows = cell_rows(g);
    const dim3 cg = cell_grid(g, rows);
    if (op == 0 && g.fc) NS_LAUNCH((k_apply<0, TopoMask>), cg, dim3(64, 4), 0, st, g, c, alpha, x, y, q, part, rows, stop);
    else if (op == 0) NS_LAUNCH((k_apply<0, TopoRect>), cg, dim3(64, 4), 0, st, g, c, alpha, x, y, q, part, rows, stop);
    else if (g.fc) NS_LAUNCH((k_apply<1, TopoMask>), cg, dim3(64, 4), 0, st, g, c, alpha, x, y, q, part, rows, stop);
    else NS_LAUNCH((k_apply<1, TopoRect>), cg, dim3(64, 4), 0, st, g, c, alpha, x, y, q, part, rows, stop);
    return (int)(cg.x * cg.y);
}

int launch_helm_rb_mask(const Geo& g, const Coef& c, double alpha, double omega, double* x, const double* b,
                        double* x2, const double* b2, int par, double* part, hipStream_t st) {
    const int rows = cell_rows(g);
    dim3 cg = cell_grid(g, rows);
    if (par < 2) cg.x = ((g.ny + 1) / 2 + 63) / 64;   // (one thread per cell of the colour)
    if (g.fc) NS_LAUNCH(k_helm_rb_mask<TopoMask>, cg, dim3(64, 4), 0, st, g, c, alpha, omega, x, b, x2, b2, par, part, rows);
    else NS_LAUNCH(k_helm_rb_mask<TopoRect>, cg, dim3(64, 4), 0, st, g, c, alpha, omega, x, b, x2, b2, par, part, rows);
    return (int)(cg.x * cg.y);
}
void launch_helm_rbt_mask(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                          const double* bu, const double* bv, double* uo, double* vo, hipStream_t st) {
    NS_LAUNCH(k_helm_rbt_mask, dim3((g.ny + 63) / 64, (g.nxl + RTM - 1) / RTM), dim3(64, 4), 0, st, g, c, alpha, omega,
              u, v, bu, bv, uo, vo);
}
// (r6) nsw (1..4) whole sweeps in one launch (k_helm_mt_mask), u, v -> uo, vo; part != null: the residuals of
// both fields after the last sweep, per workgroup (2 per workgroup); returns the workgroups (< 0: no such build)
template <int NSW, bool RES, bool BAND>
static int mt_launch(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                     const double* qbu, const double* qbv, const double* bu, const double* bv, double* uo, double* vo,
                     double* part, const int2* tiles, int ntiles, hipStream_t st) {
    constexpr int TI = MtTile<NSW>::TI, TJ = MtTile<NSW>::TJ, R = 2 * NSW + (RES ? 1 : 0);
    constexpr int EI = TI + 2 * R, EJ = TJ + 2 * R;
    constexpr int lds = (2 * EI * EJ + 4 * (EI + EJ)) * 8 + EI * EJ * 4;
    static_assert(EI <= 128 && EJ <= 128 && lds <= 80 * 1024, "table loaders / two workgroups per CU");
    lds_attr_once((const void*)k_helm_mt_mask<NSW, RES, BAND>, lds);
    const dim3 grid = BAND ? dim3(ntiles) : dim3((g.ny + TJ - 1) / TJ, (g.nxl + TI - 1) / TI);
    if (grid.x * grid.y == 0) return 0;
    NS_LAUNCH((k_helm_mt_mask<NSW, RES, BAND>), grid, dim3(MtTile<NSW>::NTH), lds, st, g, c, alpha, omega, u, v, qbu,
              qbv, bu, bv, uo, vo, part, tiles);
    return (int)(grid.x * grid.y);
}
int launch_helm_mt_mask(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                        const double* bu, const double* bv, double* uo, double* vo, int nsw, double* part,
                        hipStream_t st, const double* qbu, const double* qbv, const int* tiles, int ntiles) {
    if (!g.fc || g.nxl != g.nx) return -1;
    const int2* tl = reinterpret_cast<const int2*>(tiles);
    if (tiles) {   // the wall bands: 3 sweeps per launch, no residual
        if (nsw != 3 || part) return -1;
        return mt_launch<3, false, true>(g, c, alpha, omega, u, v, qbu, qbv, bu, bv, uo, vo, nullptr, tl, ntiles, st);
    }
    switch (nsw * 2 + (part ? 1 : 0)) {
#define NS_MT(K, RS) return mt_launch<K, RS, false>(g, c, alpha, omega, u, v, u, v, bu, bv, uo, vo, part, nullptr, 0, st)
        case 2: NS_MT(1, false);
        case 3: NS_MT(1, true);
        case 4: NS_MT(2, false);
        case 5: NS_MT(2, true);
        case 6: NS_MT(3, false);
        case 7: NS_MT(3, true);
        case 8: NS_MT(4, false);
        case 9: NS_MT(4, true);
#undef NS_MT
        default: return -1;
    }
}
void launch_diag_pc(int op, const Geo& g, const Coef& c, double alpha, const double* q, double* z, hipStream_t st,
                    const double* stop) {
    const dim3 cg = cell_grid(g);
    if (op == 0 && g.fc) NS_LAUNCH((k_diag_pc<0, TopoMask>), cg, dim3(64, 4), 0, st, g, c, alpha, q, z, stop);
    else if (op == 0) NS_LAUNCH((k_diag_pc<0, TopoRect>), cg, dim3(64, 4), 0, st, g, c, alpha, q, z, stop);
    else if (g.fc) NS_LAUNCH((k_diag_pc<1, TopoMask>), cg, dim3(64, 4), 0, st, g, c, alpha, q, z, stop);
    else NS_LAUNCH((k_diag_pc<1, TopoRect>), cg, dim3(64, 4), 0, st, g, c, alpha, q, z, stop);
}

int launch_bicg_vec(int mode, KrylovArgs a, hipStream_t st) {
    a.rows = cell_rows(a.g);
    const dim3 cg = cell_grid(a.g, a.rows);
    switch (mode) {
        case KV_INIT: NS_LAUNCH(k_bicg_vec<KV_INIT>, cg, dim3(64, 4), 0, st, a); break;
        case KV_P: NS_LAUNCH(k_bicg_vec<KV_P>, cg, dim3(64, 4), 0, st, a); break;
        case KV_V: NS_LAUNCH(k_bicg_vec<KV_V>, cg, dim3(64, 4), 0, st, a); break;
        case KV_T: NS_LAUNCH(k_bicg_vec<KV_T>, cg, dim3(64, 4), 0, st, a); break;
        default: NS_LAUNCH(k_bicg_vec<KV_X>, cg, dim3(64, 4), 0, st, a); break;
    }
    return (int)(cg.x * cg.y);
}

void launch_bicg_scal(int stage, const double* d, double n, double* sc, hipStream_t st) {
    NS_LAUNCH(k_bicg_scal, dim3(1), dim3(1), 0, st, stage, d, n, sc, 0.0, 0.0, stage == KSC_RESET ? -1 : 0);
}
void launch_bicg_start(double* sc, double thr, double b2, int maxit, hipStream_t st) {
    NS_LAUNCH(k_bicg_scal, dim3(1), dim3(1), 0, st, (int)KSC_RESET, (const double*)nullptr, 0.0, sc, thr, b2,
              std::max(maxit, 0));
}

bool correct_streams(const Geo& g) {
    // (a NEUMANN side's phi ghost reaches two cells inward: the grid kernel's grad_phi)
    return cell_streaming() && !g.fc && !(g.neu[0] || g.neu[1] || g.neu[2] || g.neu[3]);
}

int launch_correct_guess(const Geo& g, const Coef& c, double dt, const double* us, const double* vs, double* u,
                         double* v, const double* phi, double* part, const double* h1, const double* h2,
                         const double* h3, const double* gc, double* gout, hipStream_t st) {
    if (!correct_streams(g) || !h1 || (h3 && !h2)) return -1;
    CellStreamArgs A{};
    A.g = g; A.c = c; A.dt = dt; A.a0 = phi; A.a1 = us; A.a2 = vs; A.o0 = u; A.o1 = v; A.part = part;
    A.h1 = h1; A.h2 = h2; A.h3 = h3; A.gout = gout;
    A.gc0 = gc[0]; A.gc1 = gc[1]; A.gc2 = gc[2]; A.gc3 = gc[3];
    return launch_cell_s<6>(A, st);
}

int launch_correct(const Geo& g, const Coef& c, double dt, const double* us, const double* vs, double* u, double* v,
                   const double* phi, double* part, hipStream_t st) {
    if (correct_streams(g)) {
        CellStreamArgs A{};
        A.g = g; A.c = c; A.dt = dt; A.a0 = phi; A.a1 = us; A.a2 = vs; A.o0 = u; A.o1 = v; A.part = part;
        return launch_cell_s<5>(A, st);
    }
    if (mask_cell_streams(g)) {
        if (g_phase == 1) return 0;   // (as launch_div)
        const int ph = g_phase;
        g_phase = 0;
        CellStreamArgs A{};
        A.g = g; A.c = c; A.dt = dt; A.a0 = phi; A.a1 = us; A.a2 = vs; A.o0 = u; A.o1 = v; A.part = part; A.fc = g.fc;
        const int n1 = launch_cell_s<5>(A, st);
        const int n2 = (g.necell + 255) / 256;
        NS_LAUNCH(k_correct_cells, dim3(n2), dim3(256), 0, st, g, c, dt, us, vs, u, v, phi, part + 4 * n1);
        g_phase = ph;
        return n1 + n2;
    }
    const int rows = cell_rows(g);
    const dim3 cg = cell_grid(g, rows);
    if (g_phase == 1) return (int)(cg.x * cg.y);   // (cannot split: all with the edge phase)
    if (g.fc) NS_LAUNCH(k_correct<TopoMask>, cg, dim3(64, 4), 0, st, g, c, dt, us, vs, u, v, phi, part, rows);
    else NS_LAUNCH(k_correct<TopoRect>, cg, dim3(64, 4), 0, st, g, c, dt, us, vs, u, v, phi, part, rows);
    return (int)(cg.x * cg.y);
}

// Poisson tile: 32 x 128 (73 KB LDS, 2 workgroups / CU); Helmholtz u+v tile: 16 x 128.
constexpr int PTI = 32, PTJ = 128, JTI = 16, JTJ = 128;

static SweepArgs make_args(const Geo& g, const Coef& c, int TI, int TJ) {
    SweepArgs a{};
    a.g = g;
    a.c = c;
    a.tiles_j = (g.ny + TJ - 1) / TJ;
    a.ntiles = a.tiles_j * ((g.nxl + TI - 1) / TI);
    return a;
}

static int g_strip_rows = 0;  // 0 = adaptive
void set_strip_rows(int L) { g_strip_rows = L >= 4 ? (std::min(L, 64) & ~1) : 0; }

// waves of kernel `k` (256-thread workgroups) the whole chip holds at once
// CUs the compute stream may use (0: all): a multi-rank solver's compute stream leaves a few CUs
// to its comm stream (ns_solver.cpp, NSGPU_COMM_CUS), and "one resident round" is sized for the rest
static thread_local int g_compute_cus = 0;
void set_compute_cus(int n) { g_compute_cus = n; }

// per-device launch facts (function-static values set on the first call's device were
// reused by solvers on other devices): the current device's CU count, and the large dynamic-LDS
// attribute set once per kernel and device
int device_cus() {
    static std::mutex mu;
    static std::map<int, int> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find(dev);
    if (it != cache.end()) return it->second;
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    cache[dev] = c;
    return c;
}
void lds_attr_once(const void* kern, int bytes) {
    static std::mutex mu;
    static std::set<std::pair<int, const void*>> done;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lock(mu);
    if (done.insert({dev, kern}).second)
        (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

static long resident_waves(const void* k) {
    static std::mutex mu;
    static std::map<std::pair<int, const void*>, int> cache;   // blocks per CU, per device
    int nb = 0, dev = 0;
    (void)hipGetDevice(&dev);
    const int cus = device_cus();
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = cache.find({dev, k});
        if (it != cache.end()) {
            nb = it->second;
        } else {
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 256, 0);
            cache[{dev, k}] = nb;
            if (getenv("NSGPU_VERBOSE")) fprintf(stderr, "nsgpu: %p holds %d blocks/CU x %d CUs\n", k, nb, cus);
        }
    }
    const int n = g_compute_cus > 0 ? std::min(g_compute_cus, cus) : cus;
    return std::max(1L, (long)nb * 4 * n);
}

// rows per strip: the fewest rows (re-read halo rows cost (rows + halo) / rows of the
// traffic) such that every strip is resident in ONE round -- a second, partial round of
// the same length runs with the chip mostly idle.  lmin: below it the halo re-reads
// dominate (coarse multigrid levels are latency-bound and want short strips).
static int strip_rows(int nxl, long nsj, long cap, int lmin, int lmax) {
    if (g_strip_rows) return g_strip_rows;
    const long nsi = std::max(1L, cap / nsj);
    int L = (int)((nxl + nsi - 1) / nsi);
    L = (L + 1) & ~1;
    return std::min(std::max(L, lmin), lmax);
}

static StreamArgs stream_args(const Geo& g, const Coef& c, const double* in, double* out, const double* b,
                              const double* shift, double alpha, double omega, double* part, bool helm) {
    StreamArgs a{};
    a.in = in; a.out = out; a.b = b; a.shift = shift;
    a.cw = c.pw; a.ce = c.pe; a.bx = c.bx; a.cs = c.ps; a.cn = c.pn; a.by = c.by;
    (void)helm;
    a.alpha = alpha; a.omega = omega;
    a.nx = g.nx; a.ny = g.ny; a.i0 = g.i0; a.nxl = g.nxl; a.ld = g.ld;
    a.nsj = (g.ny + SW - 1) / SW;
    a.part = part;
    a.sr0 = g.sr0;
    a.sr1 = g.sr1;
    a.nt = 1;
    a.ntl = -1;   // per kernel (non-temporal in the prolongation pass only)
    return a;
}

// Exchange / compute overlap (multi-rank): the solver launches a pass twice, first the
// strips whose rows (and read cone of `depth` rows) lie inside the slab -- while the ghost
// rows are still in flight on the comm stream -- then, after the exchange, the edge strips.
void set_strip_phase(int phase) { g_phase = phase; }

// the strip subset of the current phase (k_sweep2 launchers); returns the workgroup count
// (0: nothing to launch)
// The strip rows of a two-sweep pass for the current overlap phase (set_strip_phase), reading
// `depth` rows beyond their own:
//   phase 0: the slab's rows in strips of L (strip_rows: one resident round);
//   phase 1: rows [d, nxl - d), whose read cone stays inside the slab (launched while the
//            ghost rows travel), in strips of L over those rows;
//   phase 2: the two edge bands [0, d) and [nxl - d, nxl) as two strips of d rows -- short
//            strips, so the part after the exchange is a row pipeline of d + 8 steps rather than
//            of L + 8;
// d = depth rounded up to even (the fused restriction pairs rows).  Partial slots: phase 1's
// strip rows, then phase 2's two.  Sets a.L and the launch's strip mapping; returns the
// pass's strip count (the same for both phases) and the launch's workgroups in *nblk.
// workgroups of a k_sweep2 / k_sweep3 launch over nf fields (strip_of's mapping)
static int strip_blocks(const StreamArgs& a, int nf) {
    if (WG2X2) return nf * ((a.nsj + 1) / 2) * ((a.nrun + 1) / 2);
    return (nf * a.nsj * a.nrun + 3) / 4;
}

static int plan_strips2(StreamArgs& a, long cap, int depth, int* nblk, int lmax = 64) {
    // strips of >= 20 rows: at 2048^2 (the first coarse level) 16 -> 20 rows is 41.9 -> 38.8 us per
    // FUSE_R pass (fewer halo rows per output row beats the extra waves); 24 / 28 measured slower
#ifndef LMIN2
#define LMIN2 20
#endif
    constexpr int lmin2 = LMIN2;
    const int d = (depth + 1) & ~1, R = a.nxl - 2 * d;
    a.pbase = 0;
    a.rb1 = 0;
    // WG2X2: the 2 x 2 workgroups pad nsj and the strip rows to even counts; size the round for that
    const long nsj_e = WG2X2 ? (a.nsj + 1) & ~1 : a.nsj;
    if (WG2X2) cap = std::max(2L, (cap / nsj_e) & ~1L) * nsj_e;
    if (g_phase == 0 || R < 2) {
        a.L = strip_rows(a.nxl, nsj_e, cap, lmin2, lmax);
        const int n = (a.nxl + a.L - 1) / a.L;
        a.nrun = g_phase == 1 ? 0 : n;   // (a slab too thin to split: all of it after the exchange)
        a.slo = n;
        a.rb0 = 0;
        a.rend = a.nxl;
        *nblk = strip_blocks(a, 1);
        return a.nsj * n;
    }
    a.L = strip_rows(R, nsj_e, cap, lmin2, lmax);
    const int n1 = (R + a.L - 1) / a.L;
    if (g_phase == 1) {
        a.nrun = a.slo = n1;
        a.rb0 = d;
        a.rend = a.nxl - d;
    } else {
        a.L = d;
        a.nrun = 2;
        a.slo = 1;
        a.rb0 = 0;
        a.rb1 = a.nxl - d;
        a.rend = a.nxl;
        a.pbase = n1;
    }
    *nblk = strip_blocks(a, 1);
    return a.nsj * (n1 + 2);
}

// count_only: return the strip (= partial) count a launch with residual would have, launch nothing
template <int OP, bool RB>
static int launch_stream(StreamArgs a, hipStream_t st, bool count_only = false) {
    if (count_only) a.part = reinterpret_cast<double*>(1);
    const long cap = resident_waves(a.part ? (const void*)k_sweep<OP, RB, true> : (const void*)k_sweep<OP, RB, false>);
    a.L = strip_rows(a.nxl, a.nsj, cap, 4);
    a.nsi = (a.nxl + a.L - 1) / a.L;
    const int nstr = a.nsj * a.nsi, nblk = (nstr + 3) / 4;
    if (count_only) return nstr;
    if (a.part) NS_LAUNCH((k_sweep<OP, RB, true>), dim3(nblk), dim3(256), 0, st, a);
    else NS_LAUNCH((k_sweep<OP, RB, false>), dim3(nblk), dim3(256), 0, st, a);
    return nstr;
}

int launch_pois_rbsor(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                      const double* rp, const double* shift, double* part, hipStream_t st) {
    return launch_stream<0, true>(stream_args(g, c, phi, out, rp, shift, 0.0, omega, part, false), st);
}

// two fused red-black sweeps: strips of 120 written columns reading rows ib-4 .. ie+3;
// with the output residual (part != null) 116 columns, rows ib-5 .. ie+4
template <int OP>
static int launch_stream2(StreamArgs a, const Geo& g, hipStream_t st, bool count_only = false) {
    if (count_only) a.part = reinterpret_cast<double*>(1);
    a.nsj = a.part ? (g.ny + SW2X - 1) / SW2X : (g.ny + SW2 - 1) / SW2;
    const long cap = resident_waves(a.part ? (const void*)k_sweep2<OP, true, FUSE_NONE>
                                           : (const void*)k_sweep2<OP, false, FUSE_NONE>);
    int nblk = 0;
    const int nstr = plan_strips2(a, cap, a.part ? 5 : 4, &nblk);
    if (count_only || !nblk) return nstr;
    if constexpr (OP == 1) {
        if (a.in2) {   // two fields: the multi-rank Helmholtz pair pass
            nblk = strip_blocks(a, 2);
            if (a.part) NS_LAUNCH((k_sweep2<OP, true, FUSE_UV>), dim3(nblk), dim3(256), 0, st, a);
            else NS_LAUNCH((k_sweep2<OP, false, FUSE_UV>), dim3(nblk), dim3(256), 0, st, a);
            return nstr;
        }
    }
    if (a.part) NS_LAUNCH((k_sweep2<OP, true, FUSE_NONE>), dim3(nblk), dim3(256), 0, st, a);
    else NS_LAUNCH((k_sweep2<OP, false, FUSE_NONE>), dim3(nblk), dim3(256), 0, st, a);
    return nstr;
}

int launch_pois_rbsor2_restrict(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                                const double* rp, const double* shift, const Geo& gc, double* bc, double* pc,
                                double* part, hipStream_t st, bool zin) {
    StreamArgs a = stream_args(g, c, phi, out, rp, shift, 0.0, omega, part, false);
    a.hx = c.hx; a.hy = c.hy; a.bc = bc; a.pc = pc; a.ldc = gc.ld;
    a.nsj = (g.ny + SW2X - 1) / SW2X;
    int nblk = 0;
    const void* k = zin ? (const void*)k_sweep2<0, false, FUSE_R, true> : (const void*)k_sweep2<0, false, FUSE_R>;
    const int nstr = plan_strips2(a, resident_waves(k), 5, &nblk);
    if (!nblk) return nstr;
    if (zin) NS_LAUNCH((k_sweep2<0, false, FUSE_R, true>), dim3(nblk), dim3(256), 0, st, a);
    else NS_LAUNCH((k_sweep2<0, false, FUSE_R>), dim3(nblk), dim3(256), 0, st, a);
    return nstr;
}

int launch_pois_rbsor2_restrict_guess(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                                      const double* rp, const double* shift, const Geo& gc, double* bc, double* pc,
                                      double* part, const double* h1, const double* h2, const double* h3,
                                      const double* gcoef, hipStream_t st) {
    if (g.nxl != g.nx || g_phase != 0 || !h1 || (h3 && !h2)) return -1;
    StreamArgs a = stream_args(g, c, phi, out, rp, shift, 0.0, omega, part, false);
    a.hx = c.hx; a.hy = c.hy; a.bc = bc; a.pc = pc; a.ldc = gc.ld;
    a.gh1 = h1; a.gh2 = h2; a.gh3 = h3;
    a.gc0 = gcoef[0]; a.gc1 = gcoef[1]; a.gc2 = gcoef[2]; a.gc3 = gcoef[3];
    a.nsj = (g.ny + SW2X - 1) / SW2X;
    int nblk = 0;
    const int nstr = plan_strips2(a, resident_waves((const void*)k_sweep2_gin), 5, &nblk);
    if (nblk) NS_LAUNCH(k_sweep2_gin, dim3(nblk), dim3(256), 0, st, a);
    return nstr;
}

int launch_pois_rbsor2_prolong(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                               const double* rp, const double* shift, const Geo& gc, const double* ec,
                               double* part, hipStream_t st) {
    StreamArgs a = stream_args(g, c, phi, out, rp, shift, 0.0, omega, part, false);
    a.ec = ec; a.ldc = gc.ld; a.ncx = gc.nx; a.ncy = gc.ny; a.ci0 = gc.i0; a.dsx = gc.dsx;
    // the iterate streamed non-temporally here: 113 -> 101 us at 4096^2 (b and the coarse
    // correction keep the Infinity Cache); neutral-to-worse in the other passes
#ifndef FP_NTL
#define FP_NTL 1
#endif
    if (a.ntl < 0) a.ntl = FP_NTL;
    a.nsj = (g.ny + SW2X - 1) / SW2X;
    int nblk = 0;
    // overlap depth 5, not the 4 of its fine-row cone: fine row 0 (even) reads coarse row -1,
    // whose exchange runs concurrently with the interior strips
    // (with the output residual the fine cone is 5 rows too; the coarse one stays at 3)
    if (FP_W4) {
        const void* k = part ? (const void*)k_sweep2_fp4<true> : (const void*)k_sweep2_fp4<false>;
        const int nstr = plan_strips2(a, resident_waves(k), 5, &nblk);
        if (nblk && part) NS_LAUNCH((k_sweep2_fp4<true>), dim3(nblk), dim3(256), 0, st, a);
        else if (nblk) NS_LAUNCH((k_sweep2_fp4<false>), dim3(nblk), dim3(256), 0, st, a);
        return nstr;
    }
    if (part) {
        const int nstr = plan_strips2(a, resident_waves((const void*)k_sweep2<0, true, FUSE_P>), 5, &nblk);
        if (nblk) NS_LAUNCH((k_sweep2<0, true, FUSE_P>), dim3(nblk), dim3(256), 0, st, a);
        return nstr;
    }
    const int nstr = plan_strips2(a, resident_waves((const void*)k_sweep2<0, false, FUSE_P>), 5, &nblk);
    if (nblk) NS_LAUNCH((k_sweep2<0, false, FUSE_P>), dim3(nblk), dim3(256), 0, st, a);
    return nstr;
}

// a V-cycle boundary of a whole level (k_sweep4): phi + P(ec) -> four RB sweeps -> out, the
// residual of `out` restricted into bc (pc := 0 unless null), r^2 partials; one rank only
int launch_pois_sweep4(const Geo& g, const Coef& c, double omega, const double* phi, double* out, const double* rp,
                       const double* shift, const Geo& gc, const double* ec, double* bc, double* pc, double* part,
                       hipStream_t st) {
    if (g.nxl != g.nx || g_phase != 0) return -1;
    StreamArgs a = stream_args(g, c, phi, out, rp, shift, 0.0, omega, part, false);
    a.hx = c.hx; a.hy = c.hy; a.bc = bc; a.pc = pc; a.ldc = gc.ld;
    a.ec = ec; a.ncx = gc.nx; a.ncy = gc.ny; a.ci0 = gc.i0; a.dsx = gc.dsx;
    a.nsj = (g.ny + SW4 - 1) / SW4;
    int nblk = 0;
    const int nstr = plan_strips2(a, resident_waves((const void*)k_sweep4), 9, &nblk, L4_MAX);
    if (nblk) NS_LAUNCH(k_sweep4, dim3(nblk), dim3(256), 0, st, a);
    return nstr;
}

// the LDS-tiled versions of the two launchers above (small levels); TT x TT tiles
template <int FUSE, bool RES = false, bool ZIN = false>
static int launch_tile2(const StreamArgs& a, const Geo& g, hipStream_t st) {
    const int tj32 = (g.ny + 31) / 32, n32 = tj32 * ((g.nxl + 31) / 32);
    if (n32 >= 512) {
        NS_LAUNCH((k_tile2<FUSE, 32, RES, ZIN>), dim3(n32), dim3(256), 0, st, a, tj32);
        return n32;
    }
    const int tj = (g.ny + 15) / 16, n = tj * ((g.nxl + 15) / 16);
    NS_LAUNCH((k_tile2<FUSE, 16, RES, ZIN>), dim3(n), dim3(256), 0, st, a, tj);
    return n;
}

int launch_pois_tile2_restrict(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                               const double* rp, const double* shift, const Geo& gc, double* bc, double* pc,
                               double* part, hipStream_t st, bool zin) {
    StreamArgs a = stream_args(g, c, phi, out, rp, shift, 0.0, omega, part, false);
    a.hx = c.hx; a.hy = c.hy; a.bc = bc; a.pc = pc; a.ldc = gc.ld;
    return zin ? launch_tile2<FUSE_R, false, true>(a, g, st) : launch_tile2<FUSE_R>(a, g, st);
}

int launch_pois_tile2_prolong(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                              const double* rp, const double* shift, const Geo& gc, const double* ec,
                              double* part, hipStream_t st) {
    StreamArgs a = stream_args(g, c, phi, out, rp, shift, 0.0, omega, part, false);
    a.ec = ec; a.ldc = gc.ld; a.ncx = gc.nx; a.ncy = gc.ny; a.ci0 = gc.i0; a.dsx = gc.dsx;
    return part ? launch_tile2<FUSE_P, true>(a, g, st) : launch_tile2<FUSE_P>(a, g, st);
}

int launch_pois_rbsor2(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                       const double* rp, const double* shift, double* part, hipStream_t st) {
    return launch_stream2<0>(stream_args(g, c, phi, out, rp, shift, 0.0, omega, part, false), g, st);
}

// one launch of the Helmholtz wall-band relaxation (k_helm_band: 3 RB-SOR sweeps of u and v on
// the cells within bw of a wall), band cells read from qu / qv (the rest from u / v), written to
// ou / ov; copy != 0: the band cells qu / qv -> ou / ov instead (k_band_copy).  Returns the tiles.
// copy 2: the 6-sweep one-launch tile (k_helm_band6, one rank: its cone is 12 rows); copy 3: the
// copy-back with that launch's tiles (k_band_copy<64>)
int launch_helm_band(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                     const double* qu, const double* qv, double* ou, double* ov, const double* ru, const double* rv,
                     int bw, int copy, hipStream_t st) {
    const int BT = copy >= 2 ? BAND6_BT : nsg::BT;
    if (copy >= 2 && (g.nxl != g.nx || g_phase)) return -1;
    BandArgs a{};
    a.q[0] = u; a.q[1] = v; a.qb[0] = qu; a.qb[1] = qv; a.out[0] = ou; a.out[1] = ov; a.b[0] = ru; a.b[1] = rv;
    a.cw = c.pw; a.ce = c.pe; a.bx = c.bx; a.cs = c.ps; a.cn = c.pn; a.by = c.by;
    a.alpha = alpha; a.omega = omega;
    a.nx = g.nx; a.ny = g.ny; a.i0 = g.i0; a.nxl = g.nxl; a.ld = g.ld;
    a.bw = bw;
    a.phase = copy ? 0 : g_phase;
    if (copy && g_phase == 1) return 0;   // (the copy-back runs whole, after the exchange)
    a.nti = (g.nxl + BT - 1) / BT;
    a.ntj = (g.ny + BT - 1) / BT;
    auto full = [&](int ti) {   // the tile row touches the W or E band
        const int lo = g.i0 + ti * BT, hi = std::min(g.i0 + (ti + 1) * BT, g.i0 + g.nxl);
        return lo < bw || hi > g.nx - bw;
    };
    a.fa = 0;
    while (a.fa < a.nti && full(a.fa)) a.fa++;
    a.fb = a.nti;
    while (a.fb > a.fa && full(a.fb - 1)) a.fb--;
    a.ncl = std::min((bw + BT - 1) / BT, a.ntj);
    a.ncr = std::max((g.ny - bw) / BT, a.ncl);
    const int n = (a.fa + a.nti - a.fb) * a.ntj + (a.fb - a.fa) * (a.ncl + a.ntj - a.ncr);
    if (n <= 0) return 0;
    if (copy == 2) {
        lds_attr_once((const void*)k_helm_band6, BAND6_LDS);
        NS_LAUNCH(k_helm_band6, dim3(n, 2), dim3(512), BAND6_LDS, st, a);
    } else if (copy == 3) {
        NS_LAUNCH(k_band_copy<BAND6_BT>, dim3(n, 2), dim3(256), 0, st, a);
    } else if (copy) {
        NS_LAUNCH(k_band_copy<nsg::BT>, dim3(n, 2), dim3(256), 0, st, a);
    } else {
        NS_LAUNCH(k_helm_band, dim3(n, 2), dim3(256), 0, st, a);
    }
    return n;
}

// three Helmholtz sweeps in one pass (k_sweep3; no residual): which = 1 u, 2 v, 3 both in one launch
int launch_helm_sweep3(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                       double* uo, double* vo, const double* ru, const double* rv, hipStream_t st, int which,
                       double* part) {
    StreamArgs a = stream_args(g, c, which == 2 ? v : u, which == 2 ? vo : uo, which == 2 ? rv : ru, nullptr, alpha,
                               omega, part, true);
    // the batch's last pass with its output residual (7-row cone: 7 ghost rows on slabs); rows in
    // flight: 3 for one field (114 vs 118 us at 4096^2 with 2), (r5) 2 for the two-field launch (its SD3 = 3
    // build spills 40 B per lane: 207 -> 191 us, bench 16,434 -> 16,725; profiles/r05/sd3/); NSGPU_SD3: A/B
    static const int sd3e = getenv("NSGPU_SD3") ? std::atoi(getenv("NSGPU_SD3")) : 0;
    const int sd3 = sd3e ? sd3e : (which == 3 ? 2 : 3);
    if (part) {
        a.nsj = (g.ny + SW3R - 1) / SW3R;
        int nblk = 0;
        const void* kr = which == 3 ? (sd3 == 3 ? (const void*)k_sweep3<FUSE_UV, true, 3> : (const void*)k_sweep3<FUSE_UV, true, 2>)
                                    : (sd3 == 3 ? (const void*)k_sweep3<FUSE_NONE, true, 3> : (const void*)k_sweep3<FUSE_NONE, true, 2>);
        // (two fields: half the resident round per field, strips up to L3_MAX rows)
        const int nstr = plan_strips2(a, resident_waves(kr) / (which == 3 ? 2 : 1), 7, &nblk, L3_MAX);
        if (which == 2) a.part = part + nstr;   // partials: u at [0, n), v at [n, 2n) (launch_helm_sweep2)
        if (!nblk) return nstr;
        if (which == 3) {
            a.in2 = v; a.out2 = vo; a.b2 = rv; a.part2 = part + nstr;
            nblk = strip_blocks(a, 2);
        }
        void* args[] = {&a};
        if (launch_raw(kr, dim3(nblk), dim3(256), args, 0, st) != hipSuccess) return -1;
        return nstr;
    }
    a.nsj = (g.ny + SW2X - 1) / SW2X;
    const void* k = which == 3 ? (const void*)k_sweep3<FUSE_UV> : (const void*)k_sweep3<FUSE_NONE>;
    int nblk = 0;
    const int nstr = plan_strips2(a, resident_waves(k) / (which == 3 ? 2 : 1), 6, &nblk, L3_MAX);
    if (!nblk) return nstr;
    if (which == 3) {
        a.in2 = v; a.out2 = vo; a.b2 = rv;
        nblk = strip_blocks(a, 2);
        NS_LAUNCH(k_sweep3<FUSE_UV>, dim3(nblk), dim3(256), 0, st, a);
    } else {
        NS_LAUNCH(k_sweep3<FUSE_NONE>, dim3(nblk), dim3(256), 0, st, a);
    }
    return nstr;
}

int launch_helm_sweep2(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                       double* uo, double* vo, const double* ru, const double* rv, double* part, hipStream_t st,
                       int which) {
    int n = 0;
    if (which == 3) {
        // both components in one launch (the multi-rank pair pass: one launch boundary, and one
        // edge-strip launch after the exchange, instead of two); partials: u at [0, n), v at [n, 2n)
        StreamArgs a = stream_args(g, c, u, uo, ru, nullptr, alpha, omega, part, true);
        n = launch_stream2<1>(a, g, st, true);   // strip count only
        a.in2 = v; a.out2 = vo; a.b2 = rv; a.part2 = part ? part + n : nullptr;
        return launch_stream2<1>(a, g, st);
    }
    if (which & 1) n = launch_stream2<1>(stream_args(g, c, u, uo, ru, nullptr, alpha, omega, part, true), g, st);
    if (which & 2) {
        StreamArgs a = stream_args(g, c, v, vo, rv, nullptr, alpha, omega, nullptr, true);
        if (!(which & 1)) n = launch_stream2<1>(a, g, st, true);   // strip count only
        a.part = part ? part + n : nullptr;
        n = launch_stream2<1>(a, g, st);
    }
    return n;
}


// -1 if the plane does not fit the kernel's 32-bit buffer offsets
template <class T>
static int launch_jacobi_s(const Geo& g, const Coef& c, double omega, const T* in, T* out, const T* rp,
                           const double* shift, double* part, hipStream_t st) {
    if ((size_t)(g.nxl + 2 * HALO) * g.ld * sizeof(T) >= (size_t)OOB) return -1;
    JacobiArgs<T> a{};
    a.in = in; a.out = out; a.b = rp; a.shift = shift;
    a.cw = c.pw; a.ce = c.pe; a.cs = c.ps; a.cn = c.pn;
    a.omega = omega;
    a.nx = g.nx; a.ny = g.ny; a.i0 = g.i0; a.nxl = g.nxl; a.ld = g.ld;
    constexpr int SWV = 62 * Lane16<T>::V;
    a.nsj = (g.ny + SWV - 1) / SWV;
    a.part = part;
    const bool nt = true;
    const void* k = part ? (nt ? (const void*)k_jacobi_s<T, true, true> : (const void*)k_jacobi_s<T, true, false>)
                         : (nt ? (const void*)k_jacobi_s<T, false, true> : (const void*)k_jacobi_s<T, false, false>);
    // strips of at most 24 rows (r4, tools/sweep_c5.py over NSGPU_STRIP_ROWS): past the Infinity Cache
    // one resident round of 64-row strips ran at 0.62 of the HBM peak (8192^2, 16384^2), several
    // rounds of 20-24-row strips at 0.66-0.67; at 4096^2 the one-round height is below 24 anyway
    a.L = strip_rows(a.nxl, a.nsj, resident_waves(k), 4, 24);
    a.nsi = (a.nxl + a.L - 1) / a.L;
    const int nstr = a.nsj * a.nsi, nblk = (nstr + 3) / 4;
    void* args[] = {&a};
    if (launch_raw(k, dim3(nblk), dim3(256), args, 0, st) != hipSuccess) return -1;
    return nstr;
}

int launch_pois_jacobi(const Geo& g, const Coef& c, double omega, const double* in, double* out, const double* rp,
                       const double* shift, double* part, hipStream_t st) {
    // the branch-free streaming sweep; a plane past 4 GiB: k_sweep<Jacobi>
    {
        const int n = launch_jacobi_s<double>(g, c, omega, in, out, rp, shift, part, st);
        if (n >= 0) return n;
    }
    return launch_stream<0, false>(stream_args(g, c, in, out, rp, shift, 0.0, omega, part, false), st);
}

int launch_pois_jacobi32(const Geo& g, const Coef& c, double omega, const float* in, float* out, const float* rp,
                         const double* shift, double* part, hipStream_t st) {
    return launch_jacobi_s<float>(g, c, omega, in, out, rp, shift, part, st);
}

void launch_to_f32(const Geo& g, const double* src, float* dst, hipStream_t st) {
    const long n = (long)g.nxl * g.ld;
    NS_LAUNCH(k_to_f32, dim3((unsigned)std::min<long>((n + 255) / 256, 8192)), dim3(256), 0, st, src, dst, n);
}
void launch_to_f64(const Geo& g, const float* src, double* dst, hipStream_t st) {
    const long n = (long)g.nxl * g.ld;
    NS_LAUNCH(k_to_f64, dim3((unsigned)std::min<long>((n + 255) / 256, 8192)), dim3(256), 0, st, src, dst, n);
}

int launch_helm_sweep(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                      double* uo, double* vo, const double* ru, const double* rv, double* part, hipStream_t st,
                      int which) {
    // u and v are independent systems with the same operator: two streaming passes
    int n = 0;
    if (which & 1) n = launch_stream<1, true>(stream_args(g, c, u, uo, ru, nullptr, alpha, omega, part, true), st);
    if (which & 2) {
        StreamArgs a = stream_args(g, c, v, vo, rv, nullptr, alpha, omega, nullptr, true);
        if (!(which & 1)) n = launch_stream<1, true>(a, st, true);   // strip count only
        a.part = part ? part + n : nullptr;
        n = launch_stream<1, true>(a, st);
    }
    return n;
}

int launch_pois_rbsor_tiled(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                      const double* rp, const double* shift, double* part, hipStream_t st) {
    SweepArgs a = make_args(g, c, PTI, PTJ);
    a.q[0] = phi; a.q[1] = nullptr;
    a.qo[0] = out; a.qo[1] = nullptr;
    a.b[0] = rp; a.b[1] = nullptr;
    a.shift = shift;
    a.omega = omega;
    a.alpha = 0.0;
    a.part = part;
    if (part) NS_LAUNCH((k_rb_sweep<PTI, PTJ, 0, 1, true>), dim3(a.ntiles), dim3(256), 0, st, a);
    else NS_LAUNCH((k_rb_sweep<PTI, PTJ, 0, 1, false>), dim3(a.ntiles), dim3(256), 0, st, a);
    return a.ntiles;
}

int launch_pois_jacobi_tiled(const Geo& g, const Coef& c, double omega, const double* in, double* out,
                             const double* rp, const double* shift, double* part, hipStream_t st) {
    SweepArgs a = make_args(g, c, JTI, JTJ);
    a.b[0] = rp;
    a.shift = shift;
    a.omega = omega;
    a.part = part;
    NS_LAUNCH((k_jacobi<JTI, JTJ>), dim3(a.ntiles), dim3(256), 0, st, a, in, out, 1);
    return a.ntiles;
}

int launch_pois_residual(const Geo& g, const Coef& c, const double* phi, const double* rp, const double* shift,
                         double* part, hipStream_t st) {
    SweepArgs a = make_args(g, c, JTI, JTJ);
    a.b[0] = rp;
    a.shift = shift;
    a.omega = 0.0;
    a.part = part;
    NS_LAUNCH((k_jacobi<JTI, JTJ>), dim3(a.ntiles), dim3(256), 0, st, a, phi, (double*)nullptr, 0);
    return a.ntiles;
}

int launch_restrict(const Geo& gf, const Coef& cf, const double* phi, const double* b, const double* shift,
                    const Geo& gc, const Coef& cc, double* bc, double* pc, double* part, hipStream_t st) {
    const int rows = cell_rows(gc);
    const dim3 cg = cell_grid(gc, rows);
    NS_LAUNCH(k_restrict, cg, dim3(64, 4), 0, st, gf, cf, phi, b, shift, gc, cc, bc, pc, part, rows);
    return (int)(cg.x * cg.y);
}

void launch_prolong(const Geo& gf, double* phi, const Geo& gc, const double* ec, hipStream_t st) {
    const int rows = cell_rows(gf);
    NS_LAUNCH(k_prolong, cell_grid(gf, rows), dim3(64, 4), 0, st, gf, phi, gc, ec, rows);
}

size_t coarse_vcycle_bytes(const Geo& g) {
    int dn;
    return sizeof(double) * (size_t)cv_image_size(g.nx, g.ny, &dn);
}

// Gauss-Jordan inverse with partial pivoting of the m x m row-major matrix a (in place)
static bool invert_dense(std::vector<double>& a, int m) {
    std::vector<double> inv((size_t)m * m, 0.0);
    for (int k = 0; k < m; k++) inv[(size_t)k * m + k] = 1.0;
    for (int c = 0; c < m; c++) {
        int p = c;
        for (int r = c + 1; r < m; r++)
            if (std::fabs(a[(size_t)r * m + c]) > std::fabs(a[(size_t)p * m + c])) p = r;
        if (a[(size_t)p * m + c] == 0.0) return false;
        if (p != c)
            for (int k = 0; k < m; k++) {
                std::swap(a[(size_t)p * m + k], a[(size_t)c * m + k]);
                std::swap(inv[(size_t)p * m + k], inv[(size_t)c * m + k]);
            }
        const double d = 1.0 / a[(size_t)c * m + c];
        for (int k = 0; k < m; k++) { a[(size_t)c * m + k] *= d; inv[(size_t)c * m + k] *= d; }
        for (int r = 0; r < m; r++) {
            if (r == c) continue;
            const double f = a[(size_t)r * m + c];
            if (f == 0.0) continue;
            for (int k = 0; k < m; k++) {
                a[(size_t)r * m + k] -= f * a[(size_t)c * m + k];
                inv[(size_t)r * m + k] -= f * inv[(size_t)c * m + k];
            }
        }
    }
    a.swap(inv);
    return true;
}

// the LDS image of k_coarse_vcycle for a whole level with spacings hx (nx), hy (ny): every
// level's spacings, ConstructLHS weights (a closed side: 2/h^2, face Dirichlet) and 1/diag,
// exactly as the kernel computed them before, and M for the direct last-level solve
int cv_image(const double* hx, const double* hy, int nx, int ny, int dlo, int dhi, std::vector<double>& img,
             int* dn) {
    const int n_img = cv_image_size(nx, ny, dn);
    LdsLv lv[LV_MAX];
    int nl = 0;
    lv_layout(nx, ny, lv, &nl);
    img.assign((size_t)n_img, 0.0);
    double* L = img.data();
    for (int k = 0; k < nl; k++) {
        const LdsLv& v = lv[k];
        for (int t = 0; t < v.nx; t++) L[v.hx + t] = k == 0 ? hx[t] : L[lv[k - 1].hx + 2 * t] + L[lv[k - 1].hx + 2 * t + 1];
        for (int t = 0; t < v.ny; t++) L[v.hy + t] = k == 0 ? hy[t] : L[lv[k - 1].hy + 2 * t] + L[lv[k - 1].hy + 2 * t + 1];
        for (int t = 0; t < v.nx; t++) {
            const double h = L[v.hx + t];
            L[v.cw + t] = t > 0 ? 2.0 / (h * (h + L[v.hx + t - 1])) : (dlo ? 2.0 / (h * h) : 0.0);
            L[v.ce + t] = t < v.nx - 1 ? 2.0 / (h * (h + L[v.hx + t + 1])) : (dhi ? 2.0 / (h * h) : 0.0);
        }
        for (int t = 0; t < v.ny; t++) {
            const double h = L[v.hy + t];
            L[v.cs + t] = t > 0 ? 2.0 / (h * (h + L[v.hy + t - 1])) : 0.0;
            L[v.cn + t] = t < v.ny - 1 ? 2.0 / (h * (h + L[v.hy + t + 1])) : 0.0;
        }
        for (int i = 0; i < v.nx; i++)
            for (int j = 0; j < v.ny; j++)
                L[v.idg + i * v.ny + j] = -1.0 / ((L[v.cw + i] + L[v.ce + i]) + (L[v.cs + j] + L[v.cn + j]));
    }
    if (*dn == 0) return n_img;
    // the last level's operator (lv_lap), bordered when it is singular (no closed side)
    const LdsLv& v = lv[nl - 1];
    const int n = *dn;
    const bool sing = !dlo && !dhi;
    const int m = sing ? n + 1 : n;
    std::vector<double> a((size_t)m * m, 0.0);
    for (int i = 0; i < v.nx; i++)
        for (int j = 0; j < v.ny; j++) {
            const int r = i * v.ny + j;
            const double cw = L[v.cw + i], ce = L[v.ce + i], cs = L[v.cs + j], cn = L[v.cn + j];
            a[(size_t)r * m + r] = -((cw + ce) + (cs + cn));
            if (i > 0) a[(size_t)r * m + r - v.ny] += cw;
            if (i < v.nx - 1) a[(size_t)r * m + r + v.ny] += ce;
            if (j > 0) a[(size_t)r * m + r - 1] += cs;
            if (j < v.ny - 1) a[(size_t)r * m + r + 1] += cn;
            if (sing) {
                a[(size_t)r * m + n] = 1.0;
                a[(size_t)n * m + r] = L[v.hx + i] * L[v.hy + j];
            }
        }
    if (!invert_dense(a, m)) return -1;
    double* M = L + (n_img - n * n);
    for (int r = 0; r < n; r++)
        for (int k = 0; k < n; k++) M[r * n + k] = a[(size_t)r * m + k];
    return n_img;
}

int launch_coarse_vcycle(const Geo& g, const double* img, int img_n, int dn, double* phi, const double* b, int cycles,
                         int pre, int post, int citers, double comega, double somega, int dlo, int dhi,
                         hipStream_t st, int zin) {
    const size_t bytes = coarse_vcycle_bytes(g);
    if (bytes != (size_t)img_n * sizeof(double)) return -1;
    if (bytes > 150 * 1024 || g.nxl != g.nx) return -1;
    lds_attr_once((const void*)k_coarse_vcycle<false>, 150 * 1024);
    lds_attr_once((const void*)k_coarse_vcycle<true>, 150 * 1024);
    // the 2 x 2-block smoother (every level but the last has even sides; a level of <= 4096 cells
    // fits the LDS, so its blocks fit the workgroup); NSGPU_CV_BLK=0: the cell-loop version (A/B)
    static const int blk_env = getenv("NSGPU_CV_BLK") ? std::atoi(getenv("NSGPU_CV_BLK")) : 1;
    const int blk = blk_env && (g.nx / 2) * (g.ny / 2) <= CV_THREADS ? 1 : 0;
    if (blk)
        NS_LAUNCH(k_coarse_vcycle<true>, dim3(1), dim3(CV_THREADS), bytes, st, g, img, img_n, dn, phi, b, cycles, pre,
                  post, citers, comega, somega, dlo, dhi, zin);
    else
        NS_LAUNCH(k_coarse_vcycle<false>, dim3(1), dim3(CV_THREADS), bytes, st, g, img, img_n, dn, phi, b, cycles, pre,
                  post, citers, comega, somega, dlo, dhi, zin);
    return 0;
}

// ---------------------------------------------- K4 coarsest level: exact separable solve (r4)
// The last multigrid level (<= 128^2 cells at 4096^2) is a box whose operator is separable:
// L = Lx (x) I + I (x) Ly, Lx / Ly the level's tridiagonal 1-D operators (pw / pe, ps / pn;
// symmetric after a diagonal scaling by sqrt(h)).  With their eigen-decompositions Lx = Vx Lx' Vx^-1
// (host, once: ns_solver.cpp direct_setup) the solve L X = B is
//     Y = E o (Vx^-1 B Vy^-T),  E_km = 1 / (lx_k + ly_m)  (0 on the null mode),   X = Vx Y Vy^T
// -- the same answer as the bordered system [A 1; w^T 0] the LDS V-cycle's last level solves
// (w.x = 0 with w the cell areas).  One launch per stage G = [E o] (P M Q): a workgroup owns a
// 16 x 16 block of G.  Every global load is issued up front, in one round (a chunked loop that
// waited for each chunk's loads took 26 us per launch): M whole and P's 16 rows go to LDS, the
// block's columns of Q to registers.  Eight waves then form T = P[I, :] M (16 x n2p, a column
// tile each) by fp64 MFMA (16x16x4, K over n1p, four independent accumulators per wave), T goes
// back through LDS, and the waves split T Q[:, J] over K, summed in a fixed order.  n1p, n2p = the sides rounded up to 16 (<= 128); P, Q, E are
// zero-padded there, M / G are guarded.  Replaces the 128^2 LDS-tiled passes and the
// one-workgroup coarse V-cycle (38 us per V-cycle at 4096^2, profiles/r03).
typedef double nsd4 __attribute__((ext_vector_type(4)));
constexpr int DIRECT_MAX = 128;                    // largest padded side
constexpr int DIRECT_LDS = 20480;                  // doubles (160 KiB)
constexpr int DIRECT_THREADS = 512;                // 8 waves: 2 per SIMD
__host__ __device__ inline int direct_r1(int n1p, int n2p) {   // region 1: M, then the 8 partial tiles
    return n1p * n2p > 2048 ? n1p * n2p : 2048;
}
__host__ __device__ inline int direct_r2(int n1p, int n2p) {   // region 2: P rows, then T, in doubles
    const int a = 16 * (n1p + 2), b = 16 * (n2p + 1);
    return a > b ? a : b;
}
__global__ __launch_bounds__(DIRECT_THREADS) void k_direct(const double* __restrict__ P, const double* __restrict__ M,
                                                           const double* __restrict__ Q, const double* __restrict__ E,
                                                           double* __restrict__ G, int n1, int n2, int n1p, int n2p,
                                                           int ldm, int ldg) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* Ms = sm;                        // n1p x n2p, row k's columns XOR-swizzled by 16 on odd k
    double* R2 = sm + direct_r1(n1p, n2p);  // P[I, :] (stride n1p + 2), later T (stride n2p + 1)
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int bi = blockIdx.x, bj = blockIdx.y;
    const int r16 = lane & 15, k4 = lane >> 4;
    const int sw = (n2p & 31) ? 0 : 16;     // (half-waves read rows k, k+1: their banks stay disjoint)
    const int ps = n1p + 2, ts = n2p + 1;
    // ---- one round of loads: Q's block columns (this wave's k-steps) to registers, P's rows and M
    // to LDS (16-B loads)
    constexpr int QV = DIRECT_MAX / 4 / 8;  // k-steps of 4 per wave in step 2
    const int nks = n2p / 4, colq = 16 * bj + r16;
    double qv[QV];
#pragma unroll
    for (int q = 0; q < QV; q++) {
        const int ks = w + 8 * q;
        qv[q] = ks < nks ? Q[(size_t)(4 * ks + k4) * n2p + colq] : 0.0;
    }
    {
        constexpr int NM = DIRECT_MAX * DIRECT_MAX / 2 / DIRECT_THREADS, NP = 16 * DIRECT_MAX / 2 / DIRECT_THREADS;
        double2 mv[NM], pv[NP];
        const int hm = n2p / 2, nm = n1p * hm, np = 8 * n1p;
#pragma unroll
        for (int q = 0; q < NM; q++) {
            const int e = threadIdx.x + DIRECT_THREADS * q, k = e / hm, c = 2 * (e - k * hm);
            double2 v = {0.0, 0.0};
            if (e < nm && k < n1) {
                const double* src = M + (size_t)k * ldm + c;
                if (c + 1 < n2) v = *reinterpret_cast<const double2*>(src);
                else if (c < n2) v.x = src[0];
            }
            mv[q] = v;
        }
#pragma unroll
        for (int q = 0; q < NP; q++) {
            const int e = threadIdx.x + DIRECT_THREADS * q;
            pv[q] = e < np ? reinterpret_cast<const double2*>(P + (size_t)16 * bi * n1p)[e] : double2{0.0, 0.0};
        }
#pragma unroll
        for (int q = 0; q < NM; q++) {
            const int e = threadIdx.x + DIRECT_THREADS * q, k = e / hm, c = 2 * (e - k * hm);
            if (e < nm) *reinterpret_cast<double2*>(Ms + k * n2p + (c ^ ((k & 1) ? sw : 0))) = mv[q];
        }
#pragma unroll
        for (int q = 0; q < NP; q++) {
            const int e = threadIdx.x + DIRECT_THREADS * q, r = (2 * e) / n1p, k = 2 * e - r * n1p;
            if (e < np) { R2[r * ps + k] = pv[q].x; R2[r * ps + k + 1] = pv[q].y; }
        }
    }
    __syncthreads();
    // ---- step 1: T = P[I, :] M, one column tile per wave (ct = w; n2p <= 128), four independent
    // accumulators (k-steps mod 4) so the MFMA chains overlap, summed in a fixed order
    const int ntile = n2p / 16;
    nsd4 t4 = {0.0, 0.0, 0.0, 0.0};
    if (w < ntile) {
        nsd4 acc[4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
        const int col = 16 * w + r16;
        for (int k0 = 0; k0 < n1p; k0 += 16) {
            double av[4], bv[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int k = k0 + 4 * j + k4;
                av[j] = R2[r16 * ps + k];
                bv[j] = Ms[k * n2p + (col ^ ((k & 1) ? sw : 0))];
            }
#pragma unroll
            for (int j = 0; j < 4; j++) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[j], bv[j], acc[j], 0, 0, 0);
        }
        t4 = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    }
    __syncthreads();   // (every wave is done with P's rows: T takes their place)
    if (w < ntile) {
#pragma unroll
        for (int r = 0; r < 4; r++) R2[(k4 + 4 * r) * ts + 16 * w + r16] = t4[r];   // (f64 C/D: row = k4 + 4 r)
    }
    __syncthreads();
    // ---- step 2: G[I, J] = T Q[:, J], the k-steps of K = n2p dealt over the 8 waves
    nsd4 g4 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < QV; q++) {
        const int ks = w + 8 * q;
        if (ks < nks) g4 = __builtin_amdgcn_mfma_f64_16x16x4f64(R2[r16 * ts + 4 * ks + k4], qv[q], g4, 0, 0, 0);
    }
    // (M's region is free: the eight partial tiles, summed in a fixed order)
#pragma unroll
    for (int r = 0; r < 4; r++) Ms[w * 256 + (k4 + 4 * r) * 16 + r16] = g4[r];
    __syncthreads();
    const int t = threadIdx.x;
    if (t < 256) {
        const int gi = 16 * bi + (t >> 4), gj = 16 * bj + (t & 15);
        double g = ((Ms[t] + Ms[256 + t]) + (Ms[512 + t] + Ms[768 + t])) +
                   ((Ms[1024 + t] + Ms[1280 + t]) + (Ms[1536 + t] + Ms[1792 + t]));
        if (E) g *= E[(size_t)gi * n2p + gj];
        if (gi < n1 && gj < n2) G[(size_t)gi * ldg + gj] = g;
    }
}

bool direct_fits(int n1, int n2) {
    const int n1p = (n1 + 15) / 16 * 16, n2p = (n2 + 15) / 16 * 16;
    return n1 >= 1 && n2 >= 1 && n1p <= DIRECT_MAX && n2p <= DIRECT_MAX &&
           direct_r1(n1p, n2p) + direct_r2(n1p, n2p) <= DIRECT_LDS;
}

int launch_direct(const double* P, const double* M, const double* Q, const double* E, double* G, int n1, int n2,
                  int ldm, int ldg, hipStream_t st) {
    const int n1p = (n1 + 15) / 16 * 16, n2p = (n2 + 15) / 16 * 16;
    if (!direct_fits(n1, n2) || ldm < n2 || ldg < n2) return -1;
    lds_attr_once((const void*)k_direct, DIRECT_LDS * 8);
    const size_t bytes = (size_t)(direct_r1(n1p, n2p) + direct_r2(n1p, n2p)) * sizeof(double);
    NS_LAUNCH(k_direct, dim3(n1p / 16, n2p / 16), dim3(DIRECT_THREADS), bytes, st, P, M, Q, E, G, n1, n2, n1p, n2p,
              ldm, ldg);
    return 0;
}

// ---------------------------------------------- outflow line solve (NEUMANN side, preconditioner)
// The 1-D problem of the Poisson preconditioner's outflow side: on the boundary
// row (a W or E outflow side: one slab row, j contiguous) solve T p = r - <r>, T the operator's
// y part (ConstructLHS's weights toward j -+ 1, walls closed), <r> the hy-weighted mean
// (T's compatibility condition), p_0 pinned to 0, then the plain mean removed.  One
// workgroup; parallel cyclic reduction in LDS (ny <= LINE_CAP).  p goes to the ghost row of
// `z1` and `z2` (the V-cycle iterate's two planes), where the hierarchy's Dirichlet-centre
// closure reads it as the side's data.
constexpr int LINE_CAP = 4096;
__global__ __launch_bounds__(1024) void k_line_solve(const double* __restrict__ r, const double* __restrict__ ps,
                                                     const double* __restrict__ pn, const double* __restrict__ hy,
                                                     int ny, double* __restrict__ p) {
    extern __shared__ __attribute__((aligned(16))) double S[];
    double *A = S, *B = S + ny, *C = S + 2 * ny, *D = S + 3 * ny;
    __shared__ double red[2][16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    // hy-weighted mean of r (fixed order: per-thread strided partials, then waves)
    double sr = 0.0, sh = 0.0;
    for (int j = t; j < ny; j += 1024) { sr += hy[j] * r[j]; sh += hy[j]; }
    for (int o = 32; o > 0; o >>= 1) { sr += __shfl_xor(sr, o, 64); sh += __shfl_xor(sh, o, 64); }
    if (lane == 0) { red[0][w] = sr; red[1][w] = sh; }
    __syncthreads();
    if (t == 0) {
        double a = 0.0, h = 0.0;
        for (int k = 0; k < 16; k++) { a += red[0][k]; h += red[1][k]; }
        red[0][0] = a / h;
    }
    __syncthreads();
    const double mean = red[0][0];
    for (int j = t; j < ny; j += 1024) {
        const double cs = ps[j], cn = pn[j];
        A[j] = j == 0 ? 0.0 : cs;
        C[j] = j == 0 ? 0.0 : cn;
        B[j] = j == 0 ? 1.0 : -(cs + cn);
        D[j] = j == 0 ? 0.0 : r[j] - mean;
    }
    __syncthreads();
    constexpr int PER = LINE_CAP / 1024;
    for (int st = 1; st < ny; st <<= 1) {
        double na[PER], nb[PER], nc[PER], nd[PER];
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const int j = t + q * 1024;
            if (j >= ny) continue;
            double a = A[j], b = B[j], c = C[j], d = D[j];
            if (j - st >= 0) {
                const double k1 = a / B[j - st];
                b -= C[j - st] * k1;
                d -= D[j - st] * k1;
                a = -A[j - st] * k1;
            } else {
                a = 0.0;
            }
            if (j + st < ny) {
                const double k2 = c / B[j + st];
                b -= A[j + st] * k2;
                d -= D[j + st] * k2;
                c = -C[j + st] * k2;
            } else {
                c = 0.0;
            }
            na[q] = a; nb[q] = b; nc[q] = c; nd[q] = d;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PER; q++) {
            const int j = t + q * 1024;
            if (j >= ny) continue;
            A[j] = na[q]; B[j] = nb[q]; C[j] = nc[q]; D[j] = nd[q];
        }
        __syncthreads();
    }
    // p = D / B, then its plain mean removed
    double sp = 0.0;
    for (int j = t; j < ny; j += 1024) { D[j] = D[j] / B[j]; sp += D[j]; }
    for (int o = 32; o > 0; o >>= 1) sp += __shfl_xor(sp, o, 64);
    __syncthreads();
    if (lane == 0) red[0][w] = sp;
    __syncthreads();
    if (t == 0) {
        double a = 0.0;
        for (int k = 0; k < 16; k++) a += red[0][k];
        red[1][0] = a / ny;
    }
    __syncthreads();
    const double pm = red[1][0];
    for (int j = t; j < ny; j += 1024) p[j] = D[j] - pm;
}

// the line solution p extended constantly along x: every row of the plane z (its halo rows
// included; columns ny .. ld zero) and, if zg, the one row zg (the other plane's ghost)
__global__ __launch_bounds__(256) void k_line_extend(const double* __restrict__ p, int ny, int ld, int rows,
                                                     double* __restrict__ z, double* __restrict__ zg) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= ld) return;
    const double v = j < ny ? p[j] : 0.0;
    for (int r = blockIdx.y; r < rows; r += gridDim.y) z[(ptrdiff_t)r * ld + j] = v;
    if (zg && blockIdx.y == 0) zg[j] = v;
}

int launch_line_solve(const double* r, const Coef& c, int ny, double* p, hipStream_t st) {
    if (ny > LINE_CAP) return -1;
    lds_attr_once((const void*)k_line_solve, 4 * LINE_CAP * (int)sizeof(double));
    NS_LAUNCH(k_line_solve, dim3(1), dim3(1024), (size_t)4 * ny * sizeof(double), st, r, c.ps, c.pn, c.hy, ny, p);
    return 0;
}

void launch_line_extend(const double* p, const Geo& g, double* z, int rows, double* zg, hipStream_t st) {
    NS_LAUNCH(k_line_extend, dim3((g.ld + 255) / 256, std::min(rows, 256)), dim3(256), 0, st, p, g.ny, g.ld, rows, z,
              zg);
}

void launch_reduce_sum(const double* p, int n, int nv, double* out, hipStream_t st) {
    NS_LAUNCH(k_reduce_sum, dim3(1), dim3(1024), 0, st, p, n, nv, out);
}
void launch_reduce_sum_segs(const double* p, int n, int nseg, double* out, hipStream_t st) {
    NS_LAUNCH(k_reduce_sum_segs, dim3(1), dim3(1024), 0, st, p, n, nseg, out);
}
void launch_reduce_min(const double* p, int n, int nv, double* out, hipStream_t st) {
    NS_LAUNCH(k_reduce_min, dim3(1), dim3(1024), 0, st, p, n, nv, out);
}
void launch_reduce_sum_min(const double* ps, int ns, int nvs, double* outs, const double* pm, int nm, int nvm,
                           double* outm, hipStream_t st) {
    NS_LAUNCH(k_reduce_sum_min, dim3(2), dim3(1024), 0, st, ps, ns, nvs, outs, pm, nm, nvm, outm);
}
void launch_reduce_sum_mean(const double* p, int n, double* sums, double ncells, double* out, hipStream_t st) {
    NS_LAUNCH(k_reduce_sum_mean, dim3(1), dim3(1024), 0, st, p, n, sums, ncells, out);
}
void launch_bus_reduce(const double* gathered, int P, int nv, int nsum, const int* dst, double* out, hipStream_t st) {
    BusDst d{};
    for (int t = 0; t < nv && t < 16; t++) d.d[t] = dst[t];
    NS_LAUNCH(k_bus_reduce, dim3(1), dim3(64), 0, st, gathered, P, nv, nsum, d, out);
}
void launch_finish_mean(const double* sums, double ncells, double* out, hipStream_t st) {
    NS_LAUNCH(k_finish_mean, dim3(1), dim3(1), 0, st, sums, ncells, out);
}
int launch_sums(const Geo& g, const double* f, double* part, hipStream_t st) {
    const int rows = cell_rows(g);
    const dim3 cg = cell_grid(g, rows);
    NS_LAUNCH(k_sums, cg, dim3(64, 4), 0, st, g, f, part, rows);
    return (int)(cg.x * cg.y);
}
void launch_axpby(const Geo& g, double a, const double* x, double b, const double* y, double* out, hipStream_t st,
                  double c, const double* z, double d, const double* w, double e, const double* v) {
    NS_LAUNCH(k_axpby, cell_grid(g), dim3(64, 4), 0, st, g, a, x, b, y, c, z, d, w, e, v, out);
}
int launch_area_sum(const Geo& g, const Coef& c, const double* b, double* part, hipStream_t st) {
    const int rows = cell_rows(g);
    const dim3 cg = cell_grid(g, rows);
    NS_LAUNCH(k_area_sum, cg, dim3(64, 4), 0, st, g, c, b, part, rows);
    return (int)(cg.x * cg.y);
}
void launch_area_fix(const Geo& g, const Coef& c, double* b, const double* sab, const double* shift, double area,
                     double inv_area, double n, double* kshift, hipStream_t st) {
    NS_LAUNCH(k_area_fix, cell_grid(g), dim3(64, 4), 0, st, g, c, b, sab, shift, area, inv_area, n, kshift);
}
void launch_fill_random(const Geo& g, double* phi, double* rp, uint64_t seed, hipStream_t st) {
    NS_LAUNCH(k_fill_random, cell_grid(g), dim3(64, 4), 0, st, g, phi, rp, seed);
}

}  // namespace nsg
