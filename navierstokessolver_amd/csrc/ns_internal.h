// ns_internal.h -- shared between the gfx950 kernels (ns_kernels.hip) and the
// C-ABI / orchestration layer (ns_solver.cpp).  Not installed.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <vector>

namespace nsg {

constexpr int HALO = 7;  // ghost rows per side: K1's MUSCL stencil (2), the 2-sweep pass's cone (4),
                         // the 2-sweep pass with fused restriction (5), the 3-sweep pass (6), the
                         // 3-sweep pass with its output residual (7: slabs end a Helmholtz batch
                         // on it like one rank does)

// Non-rectangular domains (polygons with holes / steps, Grid.cpp:131-185): one int32 code per
// cell of the bounding box, in a plane laid out like the fields (halo rows included):
//   FC_IN set = the cell is in the domain; bits 5k..5k+4 = the boundary edge on face k
//   (0 W, 1 E, 2 S, 3 N; Cell::edges, Grid.h:33) or FC_INT if the neighbour is in the domain.
constexpr int FC_IN = 1 << 20;
// (r5) the cell's neighbours up to 2 away along x and y (K1's MUSCL stencil) are all in the domain
constexpr int FC_DEEP = 1 << 21;
// (r6) FC_BAND: the cell lies within the wall-band width of a boundary face along its row or column (one rank;
// the masked Helmholtz solve's wall bands)
constexpr int FC_BAND = 1 << 22;
constexpr int FC_INT = 31;
constexpr int MAX_EDGES = 31;
__host__ __device__ inline int fc_edge(int code, int k) { return (code >> (5 * k)) & 31; }
// one polygon edge on the device: ghost stencils of ConstructGhostStencils (FluidSolver.cpp:84-103)
struct EdgeDev {
    int neu;            // NEUMANN outflow (velocity ghost q, phi ghost 2.5/-2/0.5)
    int enx, eny;       // outward normal
    double c0, c1;      // velocity ghost constants (u, v) of walls / inlets
};

// Geometry of one x-slab.  Fields are (nxl + 2*HALO) rows of ld doubles, j contiguous;
// pointers handed to kernels point at local row 0.  Global row = i0 + local row.
struct Geo {
    const int32_t* fc = nullptr;   // masked domains: topology codes at local row 0 (null: rectangle)
    const EdgeDev* et = nullptr;   // masked domains: edge table
    int nx, ny;       // global cells
    int i0, nxl;      // slab start (global) and local rows
    int ld;           // row stride in doubles (ny rounded up to 128: one streaming strip = 1 KiB per wave)
    // rectangle sides 0=W,1=E,2=S,3=N: velocity ghost q_g = neu ? q : -q + c[d]
    // (EvaluateGhostStencil_V, FluidSolver.cpp:166-173; constants :89-96)
    int neu[4];
    double c0[4], c1[4];
    int enx[4], eny[4];  // outward normal of the edge on that side
    // (r5) the rows whose values enter a launch's reductions (residual / norm / min-max partials), in
    // this geometry's local rows: a launch that also computes rows of the neighbours' slabs -- the deep
    // ghost rows of multi-rank steps (ns_solver.cpp deep_geo) -- sums only its own slab's rows
    int sr0 = 0, sr1 = 1 << 30;
    // Poisson multigrid levels of the outflow preconditioner: x sides (bit 0: i = -1, bit 1:
    // i = nx) closed by Dirichlet data on the face (weight 2/h^2 toward the ghost, which holds
    // the face value) instead of a wall; prolongation extends the correction there oddly
    // (0 on the face) rather than reflecting it
    int dsx = 0;
    // (r5) masked domains: the slab's domain cells that are not FC_DEEP (plane offsets li * ld + j, ascending) --
    // K1's LDS tiles take the FC_DEEP cells, a second launch these (launch_rhs)
    const int* ecell = nullptr;
    int necell = 0;
};

// 1-D coefficient tables (global index) built once from hx, hy (ConstructLHS, FluidSolver.cpp:113-131)
struct Coef {
    const double *hx, *hy;          // spacings
    const double *pw, *pe, *ps, *pn; // 2/(h (h+h_nb)) toward an existing neighbour, 0 at the boundary
    const double *bx, *by;          // Helmholtz Dirichlet boundary-face diagonal term 2/h^2 (0 inside)
    const double *rhx, *rhy;        // 1/h
    const double *rsx, *rsy;        // 2/(h_{i-1} + h_i) at index i (n+1 entries; 0 at both ends)
    // face interpolation weights of Div_V / GradP (FluidSolver.cpp:389-414, 429-452):
    // r = h_i / (h_nb + h_i) toward the lower (fw, fs) and upper (fe, fn) neighbour, 0 at a wall
    const double *fwx, *fex, *fsy, *fny;
    // (r5) hy uniform (every hy[j] equal): K1's column tables are then one wave-uniform value each
    // (k_rhs_s's UY variant keeps them in SGPRs; set by the solver for its finest level only)
    int yuni = 0;
};

struct Partials {
    double* p;      // per-block partials
    int n;          // number of blocks written
};

// ---- launchers (all asynchronous on `st`) ----
// K1: rhs_velocity (ConstructRHS_V); partials (sum ru^2, sum rv^2) per block
// depth: the rows beyond a strip it reads (2: MUSCL), which the exchange / compute overlap's phases split by
// (a deep-ghost launch passes its extension + 2: its extension rows wait for the exchange too)
// (r6) uo / vo / mm: the previous step's CorrectVelocities folded in (ns_solver's deferred K5, ns_step_async): u, v
// are u*, v*, phi is phi^n; the corrected u, v of every cell go to uo, vo and their min / max partials (4 per
// block, the same count as the return value) to mm.  Streaming kernel only (-1 otherwise)
int launch_rhs(const Geo& g, const Coef& c, double dt, double re, const double* u, const double* v,
               const double* phi, double* cu, double* cv, double* ru, double* rv, double* part, hipStream_t st,
               int depth = 2, double* uo = nullptr, double* vo = nullptr, double* mm = nullptr);
// K2: fused red-black SOR sweep of (I - a L_V) on u and v, (u,v) -> (uo,vo);
//     residual^2 partials of the input if part != null: u at part[0..n), v at part[n..2n), n returned
int launch_helm_sweep(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                      double* uo, double* vo, const double* ru, const double* rv, double* part, hipStream_t st,
                      int which = 3);
// K3: divergence / dt  + partial sums (sum, sum^2)
int launch_div(const Geo& g, const Coef& c, double dt, const double* u, const double* v, double* rp,
               double* part, hipStream_t st);
// K4: fused red-black SOR Poisson sweep phi -> out; residual^2 partials of the input iterate
int launch_pois_rbsor(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                      const double* rp, const double* shift, double* part, hipStream_t st);
// K4 Jacobi: out = in + w (b - shift - L in)/diag
int launch_pois_jacobi(const Geo& g, const Coef& c, double omega, const double* in, double* out,
                       const double* rp, const double* shift, double* part, hipStream_t st);
// K4 Jacobi on fp32 fields (rows of g.ld floats), fp64 arithmetic and residual partials
int launch_pois_jacobi32(const Geo& g, const Coef& c, double omega, const float* in, float* out, const float* rp,
                         const double* shift, double* part, hipStream_t st);
// the slab's own rows fp64 -> fp32 and back
void launch_to_f32(const Geo& g, const double* src, float* dst, hipStream_t st);
void launch_to_f64(const Geo& g, const float* src, double* dst, hipStream_t st);
// two red-black sweeps in one HBM pass (temporal blocking): same results as two calls above;
// residual partials (if part) are of the OUTPUT iterate, and then 5 ghost rows are read
// (4 without)
int launch_pois_rbsor2(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                       const double* rp, const double* shift, double* part, hipStream_t st);
// K2: three RB-SOR sweeps per pass (k_sweep3; no residual partials); which as above
// one launch of the Helmholtz wall-band relaxation (k_helm_band): 3 RB-SOR sweeps of u and v
// restricted to the cells within bw of a wall, every other cell held; the band cells are read from
// qu / qv and written to ou / ov, the others read from u / v; copy != 0: the band cells qu / qv ->
// ou / ov instead.  Needs 6 ghost rows of u, v, qu, qv and 5 of ru, rv; returns the tile count
int launch_helm_band(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                     const double* qu, const double* qv, double* ou, double* ov, const double* ru, const double* rv,
                     int bw, int copy, hipStream_t st);
// part != null: the pass also sums its output's residual (one field, one rank; < 0 otherwise)
int launch_helm_sweep3(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                       double* uo, double* vo, const double* ru, const double* rv, hipStream_t st, int which,
                       double* part = nullptr);
int launch_helm_sweep2(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                       double* uo, double* vo, const double* ru, const double* rv, double* part, hipStream_t st,
                       int which = 3);
// ns (3 or 4) Helmholtz sweeps of ONE component in one pass (q -> qo), a single slab only
// (-1 otherwise); residual partials of the output if part (part_second: written after as many
// slots, v's layout after u's); returns the partial count

// A/B reference: LDS-tiled fused sweeps (first version)
int launch_pois_rbsor_tiled(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                            const double* rp, const double* shift, double* part, hipStream_t st);
int launch_pois_jacobi_tiled(const Geo& g, const Coef& c, double omega, const double* in, double* out,
                             const double* rp, const double* shift, double* part, hipStream_t st);
// rows per streaming strip (tuning knob)
void set_strip_rows(int L);
// CUs the following launches' streams may use (0 = all): sizes "one resident round" of strips
void set_compute_cus(int n);
// the current device's CU count; hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per kernel and device
int device_cus();
void lds_attr_once(const void* kern, int bytes);
// the next kernel launch records a, b at its begin / end (hipExtLaunchKernel); pending() clears
// the request and says whether no launch took it
void time_next_launch(hipEvent_t a, hipEvent_t b);
bool time_next_launch_pending();
// a launcher outside ns_kernels.hip takes the pending request (and stamps its launch with a, b)
bool take_launch_timing(hipEvent_t& a, hipEvent_t& b);
// strip subset of the following two-sweep pass launches (k_sweep2): 0 all, 1 the strips
// whose read cone lies inside the slab, 2 the others (exchange / compute overlap)
void set_strip_phase(int phase);
// residual only
int launch_pois_residual(const Geo& g, const Coef& c, const double* phi, const double* rp,
                         const double* shift, double* part, hipStream_t st);
// K5: u = u* - dt grad phi ; min/max partials (4 per block)
int launch_correct(const Geo& g, const Coef& c, double dt, const double* us, const double* vs, double* u, double* v,
                   const double* phi, double* part, hipStream_t st);
// K5 takes the streaming strips here (a rectangle without a NEUMANN side)
bool correct_streams(const Geo& g);
// K5 + the next step's Poisson guess in the same pass (k_cell_s<6>): gout = gc[0] phi + gc[1] h1
// + gc[2] h2 + gc[3] h3 (h2 / h3 may be null) -- k_axpby's combination; -1 where K5 does not stream
int launch_correct_guess(const Geo& g, const Coef& c, double dt, const double* us, const double* vs, double* u,
                         double* v, const double* phi, double* part, const double* h1, const double* h2,
                         const double* h3, const double* gc, double* gout, hipStream_t st);
// reductions: sum `nv` interleaved values over n partials (p[k*nv + v]) -> out[v]
void launch_reduce_sum(const double* p, int n, int nv, double* out, hipStream_t st);
// nseg contiguous segments of n partials -> out[0..nseg) (k_reduce_sum's order per segment)
void launch_reduce_sum_segs(const double* p, int n, int nseg, double* out, hipStream_t st);
// min/max: partials are (umin, -umax, vmin, -vmax) per block -> out[4] = mins of each
// (r6) launch_reduce_sum (ps) and launch_reduce_min (pm) in one launch
void launch_reduce_sum_min(const double* ps, int ns, int nvs, double* outs, const double* pm, int nm, int nvm,
                           double* outm, hipStream_t st);
void launch_reduce_min(const double* p, int n, int nv, double* out, hipStream_t st);
// Poisson prep: from sums (S, S2) and N -> shift = S/N, out[1] = S2 - S^2/N (= ||b||^2)
// one rank: launch_reduce_sum (nv = 2) + launch_finish_mean in one launch
void launch_reduce_sum_mean(const double* p, int n, double* sums, double ncells, double* out, hipStream_t st);
void launch_finish_mean(const double* sums, double ncells, double* shift_and_bn2, hipStream_t st);
// multi-rank scalar bus: gathered = P rank slots of nv (<= 16) values; value t folded over the ranks in rank
// order (a sum for t < nsum, a min after) -> out[dst[t]]
void launch_bus_reduce(const double* gathered, int P, int nv, int nsum, const int* dst, double* out, hipStream_t st);
// (sum f, sum f^2) partials over own cells
int launch_sums(const Geo& g, const double* f, double* part, hipStream_t st);
// out = a x + b y (+ c z if z) (+ d w if w) (+ e v if v) over the slab's own cells
void launch_axpby(const Geo& g, double a, const double* x, double b, const double* y, double* out, hipStream_t st,
                  double c = 0.0, const double* z = nullptr, double d = 0.0, const double* w = nullptr,
                  double e = 0.0, const double* v = nullptr);
// stretched grids: partials of sum_c A_c b_c, then b_c -= m / A_c with m = (sab - shift * area) / n
// and kshift = the shift that leaves b - kshift mean-free (the Krylov solves)
int launch_area_sum(const Geo& g, const Coef& c, const double* b, double* part, hipStream_t st);
void launch_area_fix(const Geo& g, const Coef& c, double* b, const double* sab, const double* shift, double area,
                     double inv_area, double n, double* kshift, hipStream_t st);
// random fill of phi, rhs (sweep benchmark input)
void launch_fill_random(const Geo& g, double* phi, double* rp, uint64_t seed, hipStream_t st);


// the multigrid coarsening rule shared by the global hierarchy, the LDS V-cycle and the
// oracle (og_mg_solve): halve while both sizes are even, >= 4, and the level has > 16 cells
__host__ __device__ inline bool mg_can_coarsen(int nx, int ny) {
    return nx % 2 == 0 && ny % 2 == 0 && nx >= 4 && ny >= 4 && nx * ny > 16;
}

// multigrid transfers (K4 MG): fine residual -> coarse rhs (+ coarse phi := 0, partials of r^2 over
// fine cells); fine phi += bilinear(coarse correction)
int launch_restrict(const Geo& gf, const Coef& cf, const double* phi, const double* b, const double* shift,
                    const Geo& gc, const Coef& cc, double* bc, double* pc, double* part, hipStream_t st);
void launch_prolong(const Geo& gf, double* phi, const Geo& gc, const double* ec, hipStream_t st);

// the last pre-smoothing pass with the restriction fused in: two RB sweeps of phi -> out,
// then the residual of `out` restricted to the coarse rhs bc (+ coarse phi pc := 0 unless pc
// is null: the coarse level's first pass then takes its iterate as zero without reading it)
// and partials of r^2 over the fine cells (the MG convergence check); needs 5 ghost rows
// (none of phi with zin: the input iterate is identically zero and is not read)
int launch_pois_rbsor2_restrict(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                                const double* rp, const double* shift, const Geo& gc, double* bc, double* pc,
                                double* part, hipStream_t st, bool zin = false);

// the same with the input iterate formed on the fly (r4): gcoef[0] phi + gcoef[1] h1 + gcoef[2] h2 +
// gcoef[3] h3 (h2 / h3 may be null) -- the phi extrapolation, k_axpby's arithmetic; a whole level
// only (-1 otherwise)
int launch_pois_rbsor2_restrict_guess(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                                      const double* rp, const double* shift, const Geo& gc, double* bc, double* pc,
                                      double* part, const double* h1, const double* h2, const double* h3,
                                      const double* gcoef, hipStream_t st);

// the first post-smoothing pass with the prolongation fused in: phi + P(ec) enters two RB
// sweeps -> out (phi itself is not modified); needs 5 ghost rows of phi, 3 of ec.  part != null:
// partials of r^2 of `out` too (the V-cycle's convergence check after its last pass)
int launch_pois_rbsor2_prolong(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                               const double* rp, const double* shift, const Geo& gc, const double* ec,
                               double* part, hipStream_t st);

// a V-cycle boundary in one pass (k_sweep4, r4): FUSE_P of cycle c and FUSE_R of cycle c + 1 --
// phi + P(ec) enters four RB sweeps -> out, whose residual is restricted into bc (+ pc := 0 unless
// null) with r^2 partials; the same values as the two passes.  A whole level (one rank), -1 otherwise
int launch_pois_sweep4(const Geo& g, const Coef& c, double omega, const double* phi, double* out, const double* rp,
                       const double* shift, const Geo& gc, const double* ec, double* bc, double* pc, double* part,
                       hipStream_t st);
// the same two passes as LDS-tiled kernels for the latency-bound small levels (one load
// round per pass instead of a row pipeline); same results
int launch_pois_tile2_restrict(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                               const double* rp, const double* shift, const Geo& gc, double* bc, double* pc,
                               double* part, hipStream_t st, bool zin = false);
int launch_pois_tile2_prolong(const Geo& g, const Coef& c, double omega, const double* phi, double* out,
                              const double* rp, const double* shift, const Geo& gc, const double* ec,
                              double* part, hipStream_t st);

// coarse levels as one LDS-resident V-cycle (single rank): level g and its 2x coarsenings
size_t coarse_vcycle_bytes(const Geo& g);
// the host-built LDS image of the coarse V-cycle (every level's tables + the direct last-level
// solve's matrix; dn = its size, 0 = RB-SOR sweeps); its size in doubles or < 0
int cv_image(const double* hx, const double* hy, int nx, int ny, int dlo, int dhi, std::vector<double>& img, int* dn);
// zin: the level's phi is implicitly zero (not read)
int launch_coarse_vcycle(const Geo& g, const double* img, int img_n, int dn, double* phi, const double* b, int cycles,
                         int pre, int post, int citers, double comega, double somega, int dlo, int dhi,
                         hipStream_t st, int zin = 0);
// the coarsest level's exact separable solve (k_direct), one stage G = [E o] (P M Q): P n1p x n1p,
// Q n2p x n2p, E n1p x n2p (null: none), row-major and zero-padded to n1p / n2p = n1 / n2 rounded up
// to 16 (<= 128); M, G: n1 x n2 with row strides ldm, ldg.  < 0 if the sizes do not fit
// (direct_fits: padded sides <= 128, so that M and the workgroup's rows of P fit 160 KiB of LDS)
bool direct_fits(int n1, int n2);
int launch_direct(const double* P, const double* M, const double* Q, const double* E, double* G, int n1, int n2,
                  int ldm, int ldg, hipStream_t st);
// the outflow side's 1-D line solve of the Poisson preconditioner into the row p (ny <= 4096;
// -1 otherwise), and its constant extension along x over `rows` rows of the plane z (from its
// first halo row) and the single row zg (if not null)
int launch_line_solve(const double* r, const Coef& c, int ny, double* p, hipStream_t st);
void launch_line_extend(const double* p, const Geo& g, double* z, int rows, double* zg, hipStream_t st);

// NEUMANN outflow Poisson (BiCGStab on the true operator, right-preconditioned by one
// wall-closure V-cycle; ns_solver.cpp pois_solve_krylov).  Device scalar slots:
// (r5) the convergence test on the device: KS_STOP freezes every scalar stage and vector update (and the gated
// apply / diagonal launches) once r.r <= KS_THR, r.r = 0, a breakdown, divergence or KS_MAXIT iterations;
// KS_R2 keeps that r.r, KS_IT counts the completed iterations -- the host reads them once per batch of iterations
enum { KS_RHO = 0, KS_ALPHA, KS_OMEGA, KS_BETA, KS_MEAN, KS_SUMR0, KS_BRK, KS_STOP, KS_D = 8, KS_THR = 11, KS_IT,
       KS_MAXIT, KS_R2, KS_B2, KS_NUM = 16 };
// scalar stages (k_bicg_scal) and vector modes (k_bicg_vec)
enum { KSC_INIT = 0, KSC_RHO, KSC_ALPHA, KSC_MEAN, KSC_OMEGA, KSC_CHECK, KSC_RESET };
enum { KV_INIT = 0, KV_P, KV_V, KV_T, KV_X };
struct KrylovArgs {
    Geo g;
    double *x, *r, *r0, *p, *v, *s, *t, *ph, *sh;
    const double *b, *shift, *sc;
    double* part;
    int rows;
};
// y = A x with A the reference's Poisson matrix (op 0, NEUMANN outflow rows included) or its
// Helmholtz matrix I - alpha L_V (op 1), on a rectangle or a masked domain; partials
// (sum y, sum q*y) per block (q may be null); returns the partial count
// (r5) one red (par 0) or black (par 1) SOR half-sweep of the Helmholtz matrix I - alpha L_V on x in place (and on
// x2, rhs b2, in the same pass if not null), or (par 2) the block partials of ||b - A x||^2 and ||b2 - A x2||^2 (2
// per block; returns the block count); masked domains' Helmholtz solve (one rank)
int launch_helm_rb_mask(const Geo& g, const Coef& c, double alpha, double omega, double* x, const double* b,
                        double* x2, const double* b2, int par, double* part, hipStream_t st);
// (r5) one whole red-black sweep of the same operator on u and v (rhs bu, bv) out of place, u, v -> uo, vo (LDS tiles;
// the values of a red and a black launch of the above); one rank
// (r6) nsw (1..4) whole red-black SOR sweeps of the masked Helmholtz operator on u, v in one launch (LDS temporal
// blocking), u, v -> uo, vo; part: per-workgroup residuals of both fields after the last sweep (2 each; the
// workgroup count is returned); one rank; < 0 when not applicable
// tiles != null: the wall bands (FC_BAND cells only, 3 sweeps, one workgroup per (li0, j0) pair of `tiles`: the
// MT_TI x MT_TJ tiles holding a band cell), band cells read from qbu / qbv, only they written
constexpr int MT_TI = 32, MT_TJ = 64;
int launch_helm_mt_mask(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                        const double* bu, const double* bv, double* uo, double* vo, int nsw, double* part,
                        hipStream_t st, const double* qbu = nullptr, const double* qbv = nullptr,
                        const int* tiles = nullptr, int ntiles = 0);
void launch_helm_rbt_mask(const Geo& g, const Coef& c, double alpha, double omega, const double* u, const double* v,
                          const double* bu, const double* bv, double* uo, double* vo, hipStream_t st);
// (stop: a KS_STOP slot -- the grid kernels then do nothing once it is set; null: always run)
int launch_apply(int op, const Geo& g, const Coef& c, double alpha, const double* x, double* y, const double* q,
                 double* part, hipStream_t st, const double* stop = nullptr);
// z = q / diag(A) (Jacobi preconditioner of the masked-domain solves)
void launch_diag_pc(int op, const Geo& g, const Coef& c, double alpha, const double* q, double* z, hipStream_t st,
                    const double* stop = nullptr);
// one fused BiCGStab vector update (KV_*); 3 partials per block for KV_INIT / KV_T / KV_X
int launch_bicg_vec(int mode, KrylovArgs a, hipStream_t st);
// the scalar recurrences (KSC_*) from reduced sums d
void launch_bicg_scal(int stage, const double* d, double n, double* sc, hipStream_t st);
// (r5) a solve's start: KS_IT = 0, KS_STOP = 0, the test's threshold tol^2 b2, b2 and the iteration cap
void launch_bicg_start(double* sc, double thr, double b2, int maxit, hipStream_t st);

// max partials any launcher writes for this geometry
int max_partials(const Geo& g);

// ---- the direct Poisson solve of rectangles with uniform hy (ns_fps.hip, r4) ----
#ifndef FPS_ROWS
#define FPS_ROWS 16
#endif
constexpr int FPS_M = FPS_ROWS;    // rows per chunk of the tridiagonal recurrences
#ifndef FPS_GRP
#define FPS_GRP 4   // (r4 A/B at 4096^2: 8 -> 4 waves per workgroup, three workgroups per CU at 154 VGPRs: recurrences 149 -> 138 us)
#endif
constexpr int FPS_G = FPS_GRP;     // chunks per group (one workgroup of FPS_G waves)
constexpr int FPS_LOGN_MIN = 4;    // ny = 2^4 .. 2^13 (the row pair's FFT fits 128 KiB of LDS)
constexpr int FPS_LOGN_MAX = 13;
struct FpsArgs {
    int nx, i0, nxl, ny, ld;       // global rows, slab start, local rows, modes (= ny), row stride
    int nch, ngrp;                 // local chunks (nxl / FPS_M rounded up), groups (nch / FPS_G rounded up)
    int pin;                       // both x sides zero-flux: mode 0 is singular, its last row pinned
    const double *pw, *pe;         // x coefficients (global index; Coef::pw / pe)
    const double* mu;              // mode eigenvalues of Ly (ny)
    const double* rp0;             // nch x ld: 1 / pivot of the row before each chunk
    double* ca;                    // forward chunk aggregates (E, Pi: 2 x nch x ld)
    double *ga, *gc;               // forward: group aggregates (E, Pi: 2 x ngrp x ld), group carry-ins
    double *gb, *gx;               // backward: group aggregates (X, R), group carry-ins
    double* cb;                    // backward chunk aggregates (2 x nch x ld)
    const double* bt;              // two-pass recurrences: per chunk beta (d BX / d Y_in) and BR (2 x nch x ld, host)
    double* ya;                    // two-pass recurrences: every chunk's forward carry-in (nch x ld)
    const double* sh0 = nullptr;   // fused K3 (launch_fps_div): the mean, taken off mode 0 as sh0s * mean
    double sh0s = 0.0;             // (r6) mode 0's transform of the constant 1: ny (the DCT), sqrt(sum hy) (dense)
    // r5, multi-rank, the mean deferred to the forward allgather: k_fps_mid corrects mode 0's chunk aggregates
    // (E, BXl from b's raw coefficients) by the response to the constant ny * *m0s -- m0e / m0b: every local
    // chunk's forward end value / local back substitution of the constant 1 (host tables)
    const double *m0e = nullptr, *m0b = nullptr, *m0s = nullptr;
    // r5: a NEUMANN outflow E side (one rank, uniform hx, nx even): the last row eliminated into tridiagonal
    // form (piv_next), mode 0 solved in the projected sense with the shift k_fps_mid keeps in *s0
    int outE = 0;
    double* s0 = nullptr;
    // (r6) slabs: *s0 is given before t1b (the last rank's outflow row, all-reduced: launch_fps_oe_s0) -- every
    // kernel reads it there, none derives it from its own (not the outflow) last row
    int s0_given = 0;
    // r5: the pivots tabled (t1b / t2b without the fp64 division chain): for the modes k >= kfast (a multiple
    // of 128: whole waves) 1 / p of global rows < prow (ptab, prow x ld) and the converged value (pinf, ld);
    // ptab null: none
    const double *ptab = nullptr, *pinf = nullptr;
    int prow = 0, kfast = 1 << 30;
    // (r5, default: NSGPU_FPS_PTAB=2) no table: per 128-mode block the global row from which all its modes' pivots
    // sit at their fixed point (prowb, ld / 128 ints; 1 << 30: never) -- rows before it keep the division, rows
    // after it take pinf.  The table's reads (up to 1024 rows x ld) cost t1b more than the divisions they saved
    const int* prowb = nullptr;
    // (r5, one allgather per solve) k_fps_mid's first, rank-local pass: only the groups' backward aggregates (the
    // chunks' carries and BX are formed again after the allgather)
    int mid_local = 0;
    // (r5) slabs with deep ghost rows: k_fps_t2b also writes the transformed solution of the neighbours' edge rows
    // (local rows -1 and nxl, where a neighbour exists) -- the row below from the backward carry, the row above
    // from the forward carry and the slab's own first row -- so the inverse transform gives K5 phi's ghost rows
    int ghost = 0;
};
// the other ranks' part of a multi-rank scan (k_fps_scan / k_fps_scan_seg): gathered aggregates, P slots of
// `stride` doubles (E | Pi, or X | R, and forward with the deferred mean (sum b, sum b^2) at 2 ld); a1 / ge1:
// mode 0's rank / group aggregates of the constant 1 (the deferred mean's correction; null: none); shift <-
// (mean, ||b - mean||^2) (deferred mean)
struct FpsRank {
    const double* gath = nullptr;
    int P = 1, r = 0, stride = 0;
    const double *a1 = nullptr, *ge1 = nullptr;
    double ncells = 0.0;
    double* shift = nullptr;
    // (r5, one allgather per solve, backward) every rank's slot also holds its backward aggregate with a zero
    // forward carry-in (X0 at 2 ld + 8, R at 3 ld + 8): the carry-in from the ranks after this one folds X0_p +
    // B_p Yin_p (- ny mean X1_p for mode 0) with R_p, Yin_p every rank's forward carry-in from the same slots;
    // bq: B_p (P x ld, host table), x1: X1_p (P, mode 0's response to the constant 1)
    const double *bq = nullptr, *x1 = nullptr;
};
// log2(ny) if ny is a supported power of two, else -1
int fps_log2(int ny);
// DCT-II of nrows rows of (in - *shift) (shift may be null) -> out, or (inverse) DCT-III of in -> out;
// tw: ny complex e^{-2 pi i m / ny}, wk: ny complex e^{-i pi k / 2 ny} (interleaved doubles)
// oe_pair (forward only): the row pair whose second row is a NEUMANN outflow row (transformed as b_{n-1} -
// b_{n-2} / 2, FpsArgs::outE); -1: none
// (r5) ny = 16384 (fps_log2x): each row pair as two 8192-point transforms in one launch (tw8: the 8192-point
// twiddles); ny <= 8192: tw8 unused
// (r6) the inverse transform writing only the FC_IN cells of `fcm` (a masked domain's solution into phi, the rest
// of `out` untouched); -1 where unsupported (fps_idct_mask_ok)
bool fps_idct_mask_ok(int ny);
bool fps_fuse_ok(int ny, int outE);   // (r6) the divergence fused into the forward transform (launch_fps_div)
int launch_fps_idct_masked(const double* in, double* out, int nrows, int ny, int ld, const double* tw, const double* wk,
                           hipStream_t st, const int32_t* fcm);
int launch_fps_dct(bool inverse, const double* in, const double* shift, double* out, int nrows, int ny, int ld,
                   const double* tw, const double* wk, hipStream_t st, int oe_pair = -1, const double* tw8 = nullptr);
// (r5) log2(ny) also for ny = 16384 (the two-half transforms of launch_fps_dct), else as fps_log2
int fps_log2x(int ny);
// (r6) ny the mixed-radix transforms take (even, 16 .. 8192, prime factors 2, 3, 5, 7; not a power of two)
bool fps_gen_ok(int ny);
// (r6) the dense y transforms' matrices (column-major N x N) from the tridiagonal eigenvectors C (column k = the
// eigenvector of the k-th smallest eigenvalue) and sqrt(hy): F(k, j) = q_{N-1-k}[j] sqrt(hy_j), G(j, k) =
// q_{N-1-k}[j] / sqrt(hy_j) -- mode 0 (the zero eigenvalue) set exactly: F(0, j) = hy_j / sqrt(sum hy), G(j, 0) =
// 1 / sqrt(sum hy)
void launch_dense_mats(const double* C, const double* shy, double rsum, int N, double* F, double* G, hipStream_t st);
// K3 fused into the DCT (k_fps_dct_div): b = Div_V(u*, v*) / dt of the slab's rows -> their DCT-II
// coefficients in out (of b itself: FpsArgs::sh0 takes the mean off later), b stored too if not null,
// (sum b, sum b^2) per row pair p at part + 2 p.  phase 0: every row pair; 1: those whose rows need no
// ghost row of u*; 2: the others (the first and last pair).  Returns the partial count (the pairs), or
// -1 (ny unsupported)
int launch_fps_div(const Geo& g, const Coef& c, double dt, const double* u, const double* v, double* b, double* out,
                   double* part, int phase, const double* tw, const double* wk, hipStream_t st, int outE = 0);
void launch_fps_t1(const FpsArgs& a, const double* f, hipStream_t st);
void launch_fps_t2(const FpsArgs& a, double* f, hipStream_t st);
void launch_fps_t3(const FpsArgs& a, double* f, hipStream_t st);
// the two-pass form (ns_fps.hip): t1b (t1 + the local back substitution), mid (carries and final
// backward aggregates per chunk), t2b (the exact values)
void launch_fps_t1b(const FpsArgs& a, const double* f, hipStream_t st);
void launch_fps_mid(const FpsArgs& a, const double* f, hipStream_t st);
void launch_fps_t2b(const FpsArgs& a, double* f, hipStream_t st);
// (r6) slabs with an E outflow: out = 2 f'_{n-1} (mode 0 of the outflow row's eliminated coefficients) on the rank that
// holds that row (last != 0), 0 on the others -- all-reduced (sum) into mode 0's projected shift
void launch_fps_oe_s0(const double* f, int row, int ld, int last, double* out, hipStream_t st);
// group scan (forward: ga -> gc ascending; backward: gb -> gx descending) from the carry-in of the other
// ranks (R: the fold of their gathered aggregates; default: none, 0); rout (if not null) <- this rank's
// aggregate
void launch_fps_scan(const FpsArgs& a, bool backward, const FpsRank& R, double* rout, hipStream_t st);

// (r5) a masked domain's exact Poisson solve by the capacitance matrix of its interface with the bounding box
// (ns_fps.hip; ns_solver.cpp cap_setup / cap_solve): m faces (fi: the domain cell's plane offset, fj: the outside
// cell's, w: the face's operator weight), cinv = (C + 1 1^T / m)^-1 (m x m, row-major), y (m); the ncell cells on
// either side of a face (co: plane offset, cf: up to 4 signed face references +-(f + 1), + on the domain's side,
// 0: none)
// (r5) border = 1: the box has the E outflow (mode 0 of its solve and of the domain's in the projected sense): the
// system is bordered by the unknown constant lambda the domain's right-hand side takes (q + lambda 1_domain) and the
// row y0^T y = 0 -- cinv is (m + 1) x (m + 1), y[m] = lambda, e1 = L_box^+ 1_domain (a plane)
struct CapArgs {
    int m = 0, ncell = 0, border = 0;
    const double* e1 = nullptr;
    const int *fi = nullptr, *fj = nullptr, *co = nullptr;
    const int4* cf = nullptr;
    const double* w = nullptr;
    double *cinv = nullptr, *y = nullptr;
};
constexpr size_t CAP_LDS_MAX = 8192;   // k_cap_gemv: interface differences in LDS (64 KiB of doubles)
hipError_t launch_cap_gemv(const CapArgs& a, const double* z, hipStream_t st);                // y = cinv D^T z
void launch_cap_scatter(const CapArgs& a, double* q, int mode, hipStream_t st);         // q -= D_w y / q = 0 outside
void launch_cap_axpy(const Geo& g, const CapArgs& a, double* x, const double* z, int set, hipStream_t st);  // x += z (+ lambda e1)
void launch_cap_fill(const Geo& g, double* q, double val, hipStream_t st);   // set-up: q = val on the domain
void launch_cap_rhs(const Geo& g, const double* b, const double* shift, double* r, hipStream_t st);   // r = b - shift
void launch_cap_src(const CapArgs& a, double* q, int fprev, int f, hipStream_t st);     // set-up: column f's source
void launch_cap_col(const CapArgs& a, const double* z, int f, double* cmat, hipStream_t st);   // (f = m: the border)
void launch_gj_invert(double* A, int m, double* t, double* u, double* flag, int spd, hipStream_t st);

}  // namespace nsg
