/*
 * ns_oracle.h -- CPU restatement of shivams15/navierstokessolver's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or as the timed CPU baseline).  The product path (libnsgpu.so) never links
 * or calls it.
 *
 * Provenance / pinning (see DESIGN.md "Oracle"):
 *   - The reference (SRC/FluidSolver.cpp, SRC/Grid.cpp) needs PETSc, which
 *     is absent from this image; per the build rules it is treated as
 *     UNBUILDABLE here (no PETSc stand-in is written).
 *   - This file restates its algorithm function by function (citations are
 *     /root/reference/SRC file:line) and solves each linear system to a
 *     relative residual of 1e-13, i.e. it produces the converged discrete
 *     solution the reference's KSPs approximate at rtol 1e-8.
 *   - Pinned against the known-answer stdout trace of the 128^2 Re=100
 *     cavity recorded in SURVEY.md section 6 / 8(c) (steps 1,10,50,100,150,
 *     200); see tests/test_oracle.py.
 *
 * Layout: fields are indexed by the reference's compact cell id, assigned in
 * i-outer (x), j-inner (y) order (Grid.cpp:149-162).
 */
#ifndef NS_ORACLE_H
#define NS_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* bcTypes, Grid.h:6 */
enum { OG_INLET_UNI = 0, OG_INLET_PARABOLIC = 1, OG_WALL = 2, OG_PRESSURE = 3, OG_NEUMANN = 4 };

typedef struct og_grid og_grid;
typedef struct og_solver og_solver;

const char* og_last_error(void);

/* OpenMP threads for the per-cell loops (default 1: the checker runs serially; bench.py's
 * cpu_baseline times 1 thread and the host's cores). */
void og_set_threads(int n);
int  og_get_threads(void);

/* Grid from a clockwise axis-parallel polygon (Grid.cpp:28-185).
 * xspec/yspec: nsx (nsy) rows of {start, end, ncells, ratio}; ratio -1 = uniform.
 * btype/binfo: one entry per polygon edge, in vertex order (FluidSolver.cpp:639-655). */
og_grid* og_grid_polygon(int nv, const double* vx, const double* vy,
                         int nsx, const double* xspec, int nsy, const double* yspec,
                         const int* btype, const double* binfo);
void og_grid_free(og_grid* g);
int  og_grid_N(const og_grid* g);
int  og_grid_nx(const og_grid* g);
int  og_grid_ny(const og_grid* g);
/* copies: hx (nx), hy (ny), id (nx*ny), tag (nx*ny*4), cell centres (N each) */
void og_grid_info(const og_grid* g, double* hx, double* hy, int* id, int* tag,
                  double* xc, double* yc);

/* ---- per-kernel restatements (all arrays indexed by compact id, length N) ---- */

/* grad(phi) at every cell, GradP FluidSolver.cpp:420-456 */
void og_grad_phi(const og_grid* g, const double* phi, double* gx, double* gy);

/* ConstructRHS_V FluidSolver.cpp:327-363 (+ DiffusiveFlux, ConvectiveFlux,
 * SlopeLimiter, ApplyBoundaryConditions).  gx, gy = divPhi (grad phi^{n-1}).
 * cu, cv: in = convective derivative of step n-1, out = of step n. */
void og_rhs_velocity(const og_grid* g, double dt, double re,
                     const double* u, const double* v, const double* gx, const double* gy,
                     double* cu, double* cv, double* rhs_u, double* rhs_v);

/* ConstructRHS_phi + Div_V FluidSolver.cpp:365-418 (no mean removal) */
void og_divergence(const og_grid* g, double dt, const double* us, const double* vs,
                   double* rhs_phi);

/* CorrectVelocities FluidSolver.cpp:512-534: u = us - dt*gx(phi) ... */
void og_correct(const og_grid* g, double dt, const double* us, const double* vs,
                const double* phi, double* u, double* v, double* gx, double* gy);

/* operators assembled by ConstructLHS FluidSolver.cpp:105-145, applied matrix-free */
void og_apply_poisson(const og_grid* g, const double* phi, double* out);           /* L phi */
void og_apply_helmholtz(const og_grid* g, double alpha, const double* q, double* out); /* (I - a L_V) q */

/* ExportData pressure FluidSolver.cpp:577-581: P = phi - alpha * L phi */
void og_pressure(const og_grid* g, double alpha, const double* phi, double* P);

/* Sweeps the GPU path uses (restated here for kernel parity + CPU baseline).
 * Rectangular grids whose boundary faces are all Dirichlet (walls/inlets). */
/* one weighted-Jacobi sweep on L phi = b - shift: out = in + w (b - shift - L in)/diag.
 * returns sum over cells of (b - shift - L in)^2  (residual of the INPUT iterate) */
double og_poisson_jacobi_sweep(const og_grid* g, const double* in, double* out,
                               const double* b, double shift, double omega);
/* one red-black SOR sweep in place (red = (i+j) even first). returns the
 * residual^2 of the input iterate. */
double og_poisson_rbsor_sweep(const og_grid* g, double* phi, const double* b,
                              double shift, double omega);
/* red-black SOR sweep for (I - a L_V) q = rhs, in place, u and v batched.
 * returns residual^2 (u + v) of the input iterate. */
double og_helmholtz_rbsor_sweep(const og_grid* g, double alpha, double* u, double* v,
                                const double* ru, const double* rv, double omega);

/* ---- converged linear solves (oracle KSP replacement, rel. residual tol) ---- */
int og_solve_helmholtz(const og_grid* g, double alpha, const double* rhs, double* x,
                       double rtol, int maxit);
/* removes the null-space (plain mean) from rhs in place first (FluidSolver.cpp:550) */
int og_solve_poisson(const og_grid* g, double* rhs, double* x, double rtol, int maxit);

/* ---- geometric multigrid (the GPU path's Poisson solver, restated for parity and as
 *      the same-algorithm CPU baseline).  Rectangles with Dirichlet-type faces. ---- */
/* fine residual (b - shift - L phi) -> coarse rhs, area-weighted average of each 2x2 block */
void og_mg_restrict(int nx, int ny, const double* hx, const double* hy, const double* phi, const double* b,
                    double shift, double* bc);
/* phi (nx x ny) += bilinear prolongation of the coarse correction ec (nx/2 x ny/2) */
void og_mg_prolong(int nx, int ny, const double* ec, double* phi);
/* the multigrid's exact coarsest-level solve: the first coarse level of <= cells cells (sides
 * <= 128) ends the hierarchy and is solved by its separable eigen-decomposition (the GPU's
 * NSGPU_DIRECT_CELLS; default 128^2, 0 = the round-3 hierarchy down to <= 16 cells) */
void og_mg_set_direct(long cells);
/* V-cycle solve of L x = rhs - mean(rhs) (rhs is mean-removed in place): RB Gauss-Seidel
 * smoothing (pre/post sweeps), coarsening while both sizes are even, >= 4 and > 16 cells,
 * coarsest level by red-black SOR (2n+10 iterations at the optimal omega); stops when the residual after pre-smoothing is
 * <= rtol * ||rhs||.  Returns V-cycles. */
int og_mg_solve(const og_grid* g, double* rhs, double* x, double rtol, int pre, int post, int maxcycles);
/* the same with the smoother over-relaxed by omega (the GPU path's default is 1.1) */
int og_mg_solve_w(const og_grid* g, double* rhs, double* x, double rtol, int pre, int post, int maxcycles,
                  double omega);

/* ---- the GPU's direct Poisson solve (ns_fps.hip, r4), restated: a rectangle with zero-flux faces,
 *      uniform hy (r6: any hx -- Thomas' coefficients are per row), ny = 2^p in [16, 16384] (og_fps_ok);
 *      DCT-II along y, one Thomas solve per mode along x (mode 0's last unknown pinned to 0), DCT-III.
 *      rhs is mean-removed in place (and, hx stretched, area-projected: b_c -= (sum A b / N) / A_c);
 *      returns 1 (one "iteration") or -1 ---- */
int og_fps_ok(const og_grid* g);
int og_fps_solve(const og_grid* g, double* rhs, double* x);

/* ---- full time stepper (FluidSolver::Solve, FluidSolver.cpp:536-567) ---- */
og_solver* og_solver_new(og_grid* g, double dt, double re, double rtol);
void og_solver_free(og_solver* s);
/* algorithm: 0 = Krylov solves (the reference's kind, default); 1 = the GPU path's
 * algorithm (red-black SOR Helmholtz with omega_v, multigrid Poisson V(2,2) with the
 * red-black smoother over-relaxed by omega_mg); 2 = the same with the direct Poisson solve
 * where og_fps_ok (the GPU's default there, r4), multigrid elsewhere */
void og_solver_set_algorithm(og_solver* s, int gpu_algorithm, double omega_v, double omega_mg);
/* k_helm_band restated: `sweeps` RB-SOR sweeps of u and v on the cells within w of a wall */
int og_helm_band(const og_grid* g, double a, double* u, double* v, const double* ru, const double* rv, double omega,
                 int w, int sweeps);
/* the GPU algorithm's Helmholtz wall-band relaxation: `sweeps` RB-SOR sweeps within `width` of a wall */
void og_solver_set_band(og_solver* s, int width, int sweeps);
/* one time step; mm = {umin, umax, vmin, vmax}; its = {it_u, it_v, it_phi} */
int  og_solver_step(og_solver* s, double* mm, int* its);
/* get / set state: u, v, phi, cu0, cv0, gx, gy (divPhi) -- any pointer may be NULL */
void og_solver_get(const og_solver* s, double* u, double* v, double* phi,
                   double* cu, double* cv, double* gx, double* gy);
void og_solver_set(og_solver* s, const double* u, const double* v, const double* phi,
                   const double* cu, const double* cv, const double* gx, const double* gy);

#ifdef __cplusplus
}
#endif
#endif
