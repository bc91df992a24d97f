/*
 * nsgpu.h -- C-ABI of libnsgpu.so, the MI355X (gfx950) implementation of the
 * shivams15/navierstokessolver hot path: FluidSolver::Solve's
 * advect / diffuse / project time step and its pressure-Poisson solve.
 *
 * Plain C types only (no torch / HIP types), so the reference-side host code
 * (navierstokessolver_amd/host/FluidSolver.cpp, ctypes in Python, ...) can bind
 * it directly.  Each entry point names the reference interface it replaces
 * (/root/reference/SRC/<file>:<line>).
 *
 * Conventions
 *   - every call returns 0 on success and a negative NS_E* code on failure;
 *     ns_last_error() holds the message (thread-local).  Nothing throws or aborts.
 *   - the caller owns all host buffers; the library copies them.
 *   - one host thread drives one ns_solver (handles are not thread-safe).
 *   - ns_get_fields / ns_set_fields exchange fields in the reference's compact
 *     cell-id order (the PETSc Vec of FluidSolver.h:6-18; ids i outer / x, j inner / y,
 *     cells outside the polygon skipped: Grid.cpp:149-162).  With nranks > 1 each rank
 *     exchanges its own x-slab: the compact ids ns_local_cells() names, i.e. the
 *     domain's cells in global rows ns_slab_range().  ns_get_array / ns_set_array copy
 *     the slab's nx_local x ny bounding-box plane instead (the same thing for a
 *     rectangle; 0 outside a polygon).
 *   - all state lives in HBM; ns_step() synchronises with the host once per
 *     residual check and once at the end of the step (its ns_stats), mirroring
 *     the reference's per-step printf (FluidSolver.cpp:554-560).
 */
#ifndef NSGPU_H
#define NSGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NSGPU_ABI_VERSION 9   /* 2: ns_grid_desc.face_edge (non-rectangular domains);
                                 3: ns_get/set_fields in compact-id order on polygons, ns_local_cells;
                                 4: NS_POISSON_MG is 0, so a zero-initialised ns_params selects the
                                    multigrid (RB-SOR moved to 3; the value 2 is rejected);
                                 5: ns_stats.x_link_bytes appended;
                                 6: ns_stats.t_cycle_kernel_ms / n_cycle_kernels and
                                    t_guess_kernel_ms / n_guess_kernels appended (the finest
                                    level's V-cycle-boundary and guess-forming passes);
                                 7: ns_stats.t_rhs_kernel_ms / n_rhs_kernels (K1) and the direct
                                    Poisson solve's kernel times t_fps_dct_ms / t_fps_tri_ms /
                                    t_fps_idct_ms / n_fps_solves appended;
                                 8: ns_stats.phi_checked appended (res_phi is -1 on a direct solve
                                    whose residual was not computed);
                                 9: ns_stats.t_k5_kernel_ms / n_k5_kernels (K5), t_band_kernel_ms /
                                    n_band_kernels (the Helmholtz wall bands) and k5_deferred appended */

typedef struct ns_solver ns_solver;  /* opaque: device memory, stream, RCCL comm */

/* status codes */
#define NS_OK        0
#define NS_EINVAL   -1  /* bad argument / unsupported configuration */
#define NS_EHIP     -2  /* HIP runtime failure */
#define NS_ERCCL    -3  /* RCCL failure */
#define NS_ENOMEM   -4
#define NS_EDIVERGE -5  /* non-finite values / solver did not converge */

/* boundary-condition types: bcTypes, Grid.h:6 */
#define NS_BC_INLET_UNI       0
#define NS_BC_INLET_PARABOLIC 1  /* rejected: empty ghost constant in the reference (FluidSolver.cpp:86-87,171) */
#define NS_BC_WALL            2
#define NS_BC_PRESSURE        3  /* rejected: no ghost stencil in the reference (FluidSolver.cpp:150,168) */
#define NS_BC_NEUMANN         4  /* outflow: velocity ghost q, phi ghost 2.5 phi_0 - 2 phi_1 + 0.5 phi_2
                                    (FluidSolver.cpp:98-101); needs NS_POISSON_MG, whose hierarchy then
                                    preconditions a BiCGStab solve of the true Poisson matrix */

/* Poisson solvers */
#define NS_POISSON_MG     0  /* the default (0): on a rectangle without outflow sides, uniform spacings and
                                ny = 2^p (16 .. 8192) the direct solve -- DCT along y, tridiagonal
                                recurrences along x, inverse DCT: one "iteration", residual ~1e-13,
                                checked periodically and refined by V-cycles if above rtol; elsewhere
                                (NSGPU_FPS=0 everywhere) geometric multigrid V-cycles, RB Gauss-Seidel
                                smoother */
#define NS_POISSON_JACOBI 1  /* weighted Jacobi sweeps (ping-pong) to rtol: O(n^2) sweeps per solve */
#define NS_POISSON_RBSOR  3  /* fused red-black SOR sweeps to rtol: O(n) sweeps per solve */

/* One boundary edge of the polygon (Edge, Grid.h:20-26). */
typedef struct ns_edge {
    int32_t nx, ny;   /* outward normal, one of (+-1,0),(0,+-1) */
    int32_t type;     /* NS_BC_* */
    double  info;     /* bcInfo: wall tangential speed / inlet speed */
} ns_edge;

/* Grid geometry (replaces the Grid object FluidSolver reads, Grid.h:42-69).
 * Rectangle: cell_id == face_edge == NULL and the four sides W,E,S,N each covered by
 * exactly one edge (found by its normal) -- the streaming / multigrid fast path.
 * Any other polygon (steps, holes, split sides; Grid.cpp:131-185): cell_id and
 * face_edge describe it cell by cell over the nx*ny bounding box; the time step then
 * runs the masked kernels, a Jacobi-preconditioned BiCGStab Helmholtz solve and a BiCGStab
 * Poisson solve preconditioned by one V-cycle of the bounding box's multigrid. */
typedef struct ns_grid_desc {
    int32_t nx, ny;           /* cells in x and y (Grid::hx.size(), hy.size()) */
    const double* hx;         /* nx spacings (Grid::hx) */
    const double* hy;         /* ny spacings (Grid::hy) */
    int32_t n_edges;
    const ns_edge* edges;     /* Grid::edges, in vertex order */
    const int32_t* cell_id;   /* nx*ny ids or -1 (outside); NULL = full rectangle */
    const int32_t* face_edge; /* nx*ny*4: boundary edge on the W,E,S,N face or -1 (Cell::edges, Grid.h:33);
                                 required with cell_id */
} ns_grid_desc;

/* Optional host-side transport for the x-slab exchanges (tests, or clusters without
 * RCCL): the library stages ghost rows through pinned host memory and calls these.
 * exchange: send_lo goes to rank-1, send_hi to rank+1; recv_lo is filled from rank-1,
 *           recv_hi from rank+1 (NULL where there is no neighbour); count doubles each.
 * allreduce: in place over n doubles, op 0 = sum, 1 = min.  Both return 0 on success. */
typedef struct ns_host_transport {
    void* user;
    int (*exchange)(void* user, const double* send_lo, const double* send_hi, double* recv_lo, double* recv_hi,
                    int64_t count);
    int (*allreduce)(void* user, double* buf, int32_t n, int32_t op);
} ns_host_transport;

typedef struct ns_params {
    double  dt;               /* FluidSolver::dt */
    double  re;               /* FluidSolver::re */
    int32_t poisson;          /* NS_POISSON_* */
    double  rtol;             /* relative residual tolerance of each solve (reference: 1e-8, FluidSolver.cpp:68,80) */
    int32_t max_iters;        /* sweep cap per solve (0 = 200000) */
    double  omega;            /* Poisson SOR/Jacobi weight (0 = automatic) */
    double  omega_v;          /* Helmholtz SOR weight (0 = 1.0) */
    int32_t check_every;      /* sweeps between residual checks (0 = automatic) */
    int32_t device;           /* HIP device ordinal (-1 = current / LOCAL_RANK) */
    int32_t timing;           /* 1 = time every Poisson sweep kernel with HIP events */
    /* x-slab decomposition over ranks (one process per GPU) */
    int32_t rank, nranks;
    const void* nccl_id;      /* 128-byte ncclUniqueId from rank 0 (NULL if nranks == 1) */
    /* multigrid (NS_POISSON_MG): smoothing sweeps per level before / after the coarse
     * correction, and sweeps of the coarsest solve (0 = defaults 2 / 2 / automatic) */
    int32_t mg_pre, mg_post, mg_coarse_iters;
    const ns_host_transport* host_transport;  /* NULL = RCCL (nranks > 1) */
    double mg_omega;          /* over-relaxation of the red-black smoother (0 = default 1.1:
                               * 4.1 vs 4.6 V-cycles per step at 4096^2, tools/mg_params_sweep.py) */
} ns_params;

/* Per-step result (the reference prints iter, umin, umax, vmin, vmax: FluidSolver.cpp:559-560). */
typedef struct ns_stats {
    double  umin, umax, vmin, vmax;
    int32_t it_u, it_v, it_phi;      /* sweeps of the Helmholtz solves; Poisson sweeps (RB-SOR / Jacobi) or V-cycles (MG) */
    double  res_u, res_v, res_phi;   /* final relative residuals (of the input of the last sweep); res_phi = -1
                                      * when this step's Poisson residual was not computed (phi_checked 0) */
    double  t_poisson_kernel_ms;     /* sum of Poisson sweep-kernel durations (timing == 1; multigrid: the
                                      * finest level's sweeps and prolongation passes) */
    int32_t n_poisson_kernels;       /* number of Poisson sweep kernels timed */
    int32_t n_checks;                /* residual checks (host syncs) in the step */
    double  t_restrict_kernel_ms;    /* multigrid: sum of the finest level's restriction-pass durations (timing == 1) */
    int32_t n_restrict_kernels;      /* number of those passes timed */
    double  t_helm_kernel_ms;        /* single rank: sum of the timed Helmholtz pass durations (one velocity
                                        component each, K2: the two-sweep passes and the 3-sweep passes
                                        with the residual stage -- 24 B/cell either; timing == 1) */
    int32_t n_helm_kernels;          /* number of those passes timed */
    int32_t n_exchanges;             /* ghost-row exchange groups of the step (multi-rank / loopback) */
    int32_t n_allreduces;            /* all-reduces of the step (multi-rank / loopback) */
    double  x_link_bytes;            /* bytes this rank sends over its busiest peer link in the step
                                      * (one side's ghost rows of every exchange + its slab of every
                                      * agglomeration gather; multi-rank / loopback) */
    double  t_cycle_kernel_ms;       /* multigrid, one rank: sum of the finest level's V-cycle-boundary
                                      * pass durations (k_sweep4: cycle c's prolongation + 2 sweeps and
                                      * cycle c+1's 2 sweeps + restriction in one pass; timing == 1) */
    int32_t n_cycle_kernels;         /* number of those passes timed */
    double  t_guess_kernel_ms;       /* multigrid, one rank: sum of the durations of the solves' first
                                      * finest restriction passes that form the phi extrapolation on the
                                      * fly (k_sweep2_gin; timing == 1) */
    int32_t n_guess_kernels;         /* number of those passes timed */
    double  t_rhs_kernel_ms;         /* sum of K1's durations (ConstructRHS_V, k_rhs_s; timing == 1; multi-rank:
                                      * the split launch between marker events) */
    int32_t n_rhs_kernels;           /* number of K1 launches timed */
    double  t_fps_dct_ms;            /* direct Poisson solve (timing == 1): the rows' DCT (k_fps_dct) */
    double  t_fps_tri_ms;            /*   the tridiagonal recurrences along x (k_fps_t1, scan, t2, scan, t3;
                                      *   one interval, allgathers included on slabs) */
    double  t_fps_idct_ms;           /*   the inverse DCT (k_fps_idct) */
    int32_t n_fps_solves;            /* number of direct solves timed */
    int32_t phi_checked;             /* 1: res_phi is this step's Poisson residual, computed and tested against
                                      * rtol (every multigrid / Krylov / sweep solve; the direct solve on its
                                      * first solve, every 16th after it, and on every solve once a checked
                                      * residual came within 1/100 of rtol); 0: a direct solve not checked on
                                      * this step (res_phi = -1) -- a fixed arithmetic sequence whose residual
                                      * the last check measured */
    double  t_k5_kernel_ms;          /* (ABI 9) K5's duration (CorrectVelocities, k_cell_s<5>; timing == 1).  K5 is the
                                      * step's last launch: ns_step reports its own step's, ns_step_async the
                                      * previous step's (read at this step's first host sync, like the monitor) */
    int32_t n_k5_kernels;            /* number of K5 launches timed (0 or 1) */
    double  t_band_kernel_ms;        /* (ABI 9) the Helmholtz wall-band launches (k_helm_band; timing == 1) */
    int32_t n_band_kernels;          /* number of band launches timed */
    int32_t k5_deferred;             /* (ABI 9) 1: this step's K1 applied the previous ns_step_async step's
                                      * CorrectVelocities on the fly (k_rhs_sc: K5 folded into K1, 88 B/cell;
                                      * the async step ends after its Poisson solve) */
} ns_stats;

/* device arrays addressable by ns_get_array / ns_set_array */
#define NS_ARR_U     0  /* u (u* between K2 and K5) */
#define NS_ARR_V     1
#define NS_ARR_PHI   2
#define NS_ARR_CU    3  /* convective derivative of the previous step (convectiveDer_u0) */
#define NS_ARR_CV    4
#define NS_ARR_RU    5  /* RHS_u */
#define NS_ARR_RV    6
#define NS_ARR_RPHI  7  /* RHS_phi (div u* / dt, before mean removal) */
#define NS_ARR_TMP   8  /* Poisson sweep ping-pong partner */
#define NS_ARR_TMPU  9  /* Helmholtz sweep ping-pong partners */
#define NS_ARR_TMPV 10
#define NS_NUM_ARR  11

/* kernels addressable by ns_kernel */
#define NS_K_RHS        1  /* K1 rhs_velocity            (ConstructRHS_V, FluidSolver.cpp:327-363) */
#define NS_K_HELMHOLTZ  2  /* K2 helmholtz sweep x iters  (KSPSolve(uSolver) x2, :547-548) */
#define NS_K_DIV        3  /* K3 divergence + sums        (ConstructRHS_phi, :365-378) */
#define NS_K_POISSON    4  /* K4 Poisson sweep x iters    (KSPSolve(phiSolver), :551) */
#define NS_K_CORRECT    5  /* K5 correct + min/max        (CorrectVelocities, :512-534) */
#define NS_K_HELM_SOLVE 6  /* converged Helmholtz solve   (:547-548) */
#define NS_K_POIS_SOLVE 7  /* converged Poisson solve incl. null-space removal (:550-551) */
#define NS_K_RESIDUAL   8  /* Poisson residual ||rhs - mean - L phi||^2 -> out[0] (no update) */
#define NS_K_POISSON32  9  /* K4 Jacobi x iters on fp32 copies of phi, rhs_phi (fp64 arithmetic and residual,
                              SURVEY.md 8(d) C5); phi <- the fp32 result widened */
#define NS_K_HELM_BAND 10  /* the Helmholtz solve's wall-band relaxation of u, v (k_helm_band: 6 RB-SOR sweeps,
                              two launches of 3, on the cells within max(32, min(nx, ny) / 32) of a wall,
                              the rest held); no output */

/* ---- lifecycle: FluidSolver(char*, Grid*) = SolverInitialize + SolverSetup (FluidSolver.cpp:8-58) ---- */
int  ns_create(const ns_grid_desc* grid, const ns_params* params, ns_solver** out);
void ns_destroy(ns_solver* s);

/* ---- one full time step: the body of FluidSolver::Solve's loop (FluidSolver.cpp:546-560) ---- */
int  ns_step(ns_solver* s, ns_stats* out);
/* the same step without its closing host sync: out's umin..vmax are the PREVIOUS
 * ns_step_async's min/max (NaN on the first), so a caller printing them per step prints the
 * reference's monitor sequence one step late; ns_monitor waits for the latest step's.
 * The host can enqueue the next step while this one's last kernels run. */
int  ns_step_async(ns_solver* s, ns_stats* out);
int  ns_monitor(ns_solver* s, double* mm /* [4]: umin, umax, vmin, vmax */);

/* per-kernel HIP-event timing (ns_params.timing) switched on / off between steps */
int  ns_set_timing(ns_solver* s, int on);

/* ---- state access (host buffers, local slab) ----
 * ns_get_fields / ns_set_fields: compact-id order (prevField->u, v, phi and
 * convectiveDer_u0 / _v0, FluidSolver.h:6-18 / FluidSolver.cpp:40-43), `count` doubles each
 * as ns_local_cells reports; element k is the cell with compact id first_id + k.
 * ns_get_array / ns_set_array: the slab's nx_local x ny bounding-box plane of any NS_ARR_*. */
int  ns_get_fields(ns_solver* s, double* u, double* v, double* phi);
int  ns_set_fields(ns_solver* s, const double* u, const double* v, const double* phi,
                   const double* cu0, const double* cv0);
int  ns_local_cells(ns_solver* s, int64_t* first_id, int64_t* count);
int  ns_get_array(ns_solver* s, int which, double* host);
int  ns_set_array(ns_solver* s, int which, const double* host);

/* ---- individual kernels (tests and bench) ----
 * out (may be NULL) receives kernel-specific scalars:
 *   NS_K_HELMHOLTZ / NS_K_POISSON: out[0] = residual^2 of the last sweep's input
 *   NS_K_DIV:     out[0] = sum rhs, out[1] = sum rhs^2
 *   NS_K_CORRECT: out[0..3] = umin, umax, vmin, vmax
 *   NS_K_*_SOLVE: out[0] = sweeps used, out[1] = final relative residual
 *   NS_K_RESIDUAL: out[0] = residual^2 */
int  ns_kernel(ns_solver* s, int which, int iters, double* out);

/* Multigrid transfers alone (tests): op 0 = restriction of the current residual
 * rhs_phi - mean - L phi into `coarse` (nx/2 x ny/2, host, the slab's coarse rows);
 * op 1 = prolongation: phi += bilinear(`coarse`).  Needs NS_POISSON_MG with >= 2 levels. */
int  ns_mg_transfer(ns_solver* s, int op, double* coarse);

/* Fill phi and rhs_phi with reproducible uniform [-1,1) values generated on the
 * device (splitmix64 of (seed, global cell)), rhs mean-removed: the sweep benchmark input. */
int  ns_fill_random(ns_solver* s, uint64_t seed);

/* Time `iters` Poisson sweep kernels (after `warmup`) with HIP events on the
 * solver's stream: out[0] = average kernel ms, out[1] = total ms. */
int  ns_time_poisson(ns_solver* s, int warmup, int iters, double* out);

/* The same for the fp32-field Jacobi sweep (12 B/cell; configs[4]: "fp32 fields + fp64
 * Poisson residual"): phi and rhs_phi are copied to fp32 planes first (allocated on first
 * use, 3 x 4 B/cell); out[0..2] as above, out[3] = residual^2 of the last sweep's input. */
int  ns_time_poisson_fp32(ns_solver* s, int warmup, int iters, double* out);

/* ---- host-side helpers (no GPU needed) ---- */
/* the x-slab [i0, i1) of `rank` out of `nranks` for nx cells */
int  ns_slab_range(int32_t nx, int32_t nranks, int32_t rank, int32_t* i0, int32_t* i1);
/* size in bytes of an ncclUniqueId, and produce one (rank 0 only; needs RCCL, no GPU) */
int  ns_nccl_id_size(void);
int  ns_nccl_get_id(void* out128);
/* device bytes one solver allocates for this grid */
int64_t ns_device_bytes(int32_t nx_local, int32_t ny);
/* version / last error */
int  ns_abi_version(void);
const char* ns_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* NSGPU_H */
