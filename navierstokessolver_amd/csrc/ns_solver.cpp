// ns_solver.cpp -- C-ABI (include/nsgpu.h) and time-step orchestration of libnsgpu.so.
//
// One ns_solver = one x-slab on one MI355X: all fields resident in HBM, one HIP
// stream, and (nranks > 1) one RCCL communicator whose neighbour send/recv pairs
// move contiguous ghost rows over xGMI.  The step mirrors FluidSolver::Solve's
// loop body (/root/reference/SRC/FluidSolver.cpp:546-560):
//   K1 rhs -> K2 Helmholtz sweeps (u, v) -> K3 div -> null-space mean -> K4
//   Poisson sweeps -> K5 correct + min/max.
// The reference's Krylov solves (GMRES+ILU, BCGSL+BJacobi, rtol 1e-8,
// FluidSolver.cpp:61-82) are replaced by red-black SOR sweeps run to the same
// relative-residual tolerance, checked every few sweeps from a fused residual.
#include <rccl/rccl.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <dlfcn.h>
#include <limits>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/nsgpu.h"
#include "ns_internal.h"

namespace {

thread_local std::string g_err;

void set_err(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

#define HIPCHK(x)                                                                        \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            set_err("%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            return NS_EHIP;                                                              \
        }                                                                                \
    } while (0)

#define NCCLCHK(x)                                                                          \
    do {                                                                                    \
        ncclResult_t r_ = (x);                                                              \
        if (r_ != ncclSuccess) {                                                            \
            set_err("%s failed: %s (%s:%d)", #x, ncclGetErrorString(r_), __FILE__, __LINE__); \
            return NS_ERCCL;                                                                \
        }                                                                                   \
    } while (0)

#define CHK(x)                 \
    do {                       \
        int rc_ = (x);         \
        if (rc_ != 0) return rc_; \
    } while (0)

// device scalar slots
enum {
    S_DIVSUM = 0,   // 2: sum rhs, sum rhs^2
    S_SHIFT = 2,    // 2: mean, ||rhs - mean||^2
    S_HBN = 4,      // 2: ||ru||^2, ||rv||^2
    S_RES = 6,      // 2: residual^2 (u, v) or (phi, -)
    S_MM = 8,       // 4: umin, -umax, vmin, -vmax
    S_AUX = 12,     // 4
    S_KSHIFT = 16,  // 1: the Krylov solves' shift after consistent_rhs (see there)
    // multi-rank scalar bus (r5, bus()): this rank's partial values, gathered from every rank and folded
    // into the global slots above -- K1's ||RHS||^2 (-> S_HBN), the Helmholtz residuals (-> S_RES, S_AUX)
    // and the previous K5's min / max (-> S_MM); contiguous, in this order
    S_HBNL = 18,    // 2
    S_RESL = 20,    // 2
    S_AUXL = 22,    // 2
    S_MML = 24,     // 4
    S_KRY = 28,     // 7: (r5) a BiCGStab batch's verdict for the host (KS_STOP, KS_BRK, KS_IT, KS_R2, r.r, alpha, omega)
    S_OE = 35,      // 1: (r6) slabs with an E outflow: mode 0's projected shift 2 f'_{n-1}, all-reduced
    S_NUM = 36
};
constexpr int BUS_NV = 10, BUS_NSUM = 6;

}  // namespace

// one multigrid level (level 0 = the solver's own PHI / TMP / RPHI arrays)
struct MgLevel {
    nsg::Geo g{};
    nsg::Coef c{};
    double *phi = nullptr, *tmp = nullptr, *b = nullptr;  // current iterate, ping-pong partner, rhs
    double* mem = nullptr;                               // planes (levels >= 1)
    double* coef = nullptr;                              // coefficient tables (levels >= 1)
    std::vector<double> hx, hy;                          // host spacings
    int minrows = 0;                                     // fewest rows any rank holds of this level
    // coarse-level agglomeration (nranks > 1): a replicated level lives WHOLE on every rank
    // (g.i0 = 0, g.nxl = g.nx) and is smoothed with no exchange.  The first replicated level
    // is reached from the last distributed one through this rank's slab of it (gs) and
    // gathered (every rank's rows si0[q] .. si0[q] + sn[q]) after the restriction.
    bool repl = false;
    // multi-rank: the rhs ghost rows are owed -- they travel with the level's next overlapped
    // FUSE_R exchange instead of in an exchange round of their own (flush_b otherwise)
    bool b_pend = false;
    // the level's iterate is identically zero but not stored (the restriction from the level
    // above skipped its phi := 0 writes): its first pass -- the fused restriction pass or the LDS
    // coarse V-cycle -- takes it as zero without reading it or its ghost rows; any other consumer
    // materialises the zeros first (zero_phi)
    bool zero = false;
    // multi-rank: the iterate's 5 ghost rows were sent right after this level's fused restriction
    // pass (riding on the next exchange group down the V-cycle): the prolongation pass needs no
    // exchange of its own for them -- phi is not written in between
    bool phi_ghost = false;
    nsg::Geo gs{};
    std::vector<int> si0, sn;
};

struct ns_solver {
    nsg::Geo g{};
    nsg::Coef c{};
    int device = 0;
    hipStream_t st = nullptr;
    double dt = 0, re = 0, rtol = 1e-8, omega = 0, omega_v = 1.0;
    int poisson = NS_POISSON_MG, max_iters = 200000, check_every = 0, timing = 0;
    double* base = nullptr;      // all fields
    size_t plane = 0;            // doubles per field plane
    double* arr[NS_NUM_ARR] = {};  // pointer to local row 0 of each field
    double* coef = nullptr;      // device coefficient tables
    double* part = nullptr;      // per-block partials
    double* scal = nullptr;      // device scalars
    double* hs = nullptr;        // pinned host mirror of scal
    int rank = 0, nranks = 1;
    ncclComm_t comm = nullptr;
    double ncells = 0;           // global cell count
    std::vector<hipEvent_t> ev;  // timing events (pairs)
    std::vector<char> evtag;     // per pair: 0 = sweep / prolongation pass, 1 = restriction pass
    std::vector<hipEvent_t> hev; // Helmholtz pass timing events (pairs; timing == 1, single rank)
    int hn = 0;                  // Helmholtz pairs recorded this step
    std::vector<int> hcomp;      // components per recorded Helmholtz launch (2: the one-rank two-field pass)
    int helm_batch0 = 4, pois_batch0 = 8;
    int helm_next = 4;           // first Helmholtz batch of the next step (adaptive unless check_every)
    int helm_adapt = 1;
    bool triple = true;          // 3-sweep passes allowed on this decomposition (slabs >= 2*HALO rows)
    bool sweep3 = true;          // single rank: odd Helmholtz batches start with a 3-sweep pass (k_sweep3)
    bool helm_band = true;       // Helmholtz: wall-band relaxation before the global passes (k_helm_band)
    // (r6) one rank, 6 band sweeps as ONE k_helm_band6 launch + copy-back (NSGPU_BAND6=1): half the band bytes, but
    // the launches are latency-bound, not HBM-bound -- 100 + 13 us against 2 x 48.5 (profiles/r06/ab/): off
    bool band6 = false;
    int band_w = 128, band_sweeps = 6;   // its width (cells from a wall: min(nx, ny) / 32) and RB-SOR sweeps (a multiple of 3)
    bool sweep3_res = true;      // one rank: a Helmholtz batch may end on a 3-sweep pass with its residual
    int helm_uv = 1;             // NSGPU_HELM_UV=0: one rank's 3-sweep batch as two one-field launches (A/B)
    int helm_probe = 0;          // steps since the Helmholtz first-pass residual was last sampled
    int tiled = 0;               // NSGPU_SWEEP=tiled: A/B against the first (LDS-tiled) sweep kernels
    int fuse_restrict = 1;       // NSGPU_FUSED_RESTRICT=0: separate k_restrict pass (A/B)
    int fuse_prolong = 1;        // NSGPU_FUSED_PROLONG=0: separate k_prolong pass (A/B)
    int tile_small = 1;          // NSGPU_TILE_SMALL=0: no LDS-tiled fused passes on small levels (A/B)
    int ext_timing = 1;          // NSGPU_EXT_TIMING=0: marker events around timed launches (t_begin)
    int phi_extrap = 3;          // Poisson initial guess: NSGPU_PHI_EXTRAP=0 phi^{n-1}, 1 linear, 2 quadratic,
                                 // 3 (default) cubic while the last solve took > 1 V-cycle, else quadratic
    int mg_predict = 1;          // NSGPU_MG_PREDICT=0: a residual check (host sync) after every V-cycle
    double mg_rate2 = 0.0;       // last measured per-cycle contraction of ||r||^2
    int mg_hist[4] = {-1, -1, -1, -1};   // V-cycles the last four solves converged at (first check)
    double* phim = nullptr;      // phi^{n-2} (the extrapolation's second point; rotates with PHI / TMP)
    double* phim2 = nullptr;     // phi^{n-3} (quadratic / cubic extrapolation)
    double* phim3 = nullptr;     // phi^{n-4} (cubic extrapolation)
    double* phim4 = nullptr;     // phi^{n-5} (quartic, NSGPU_PHI_EXTRAP=4: A/B only)
    double* phim_mem = nullptr;  // the extra planes' allocation
    float* f32_mem = nullptr;    // fp32-field sweep planes (configs[4]), allocated on first use
    float* f32[3] = {};          // phi, its ping-pong partner, rhs_phi (rows of g.ld floats)
    int phim_valid = 0;          // history planes holding data (0 after a reset / an injected phi)
    int verbose = 0;             // NSGPU_VERBOSE=1: solver residual histories on stderr
    long pair_min_cells = 2048L * 2048L;   // NSGPU_PAIR_MIN_CELLS: smallest level smoothed in 2-sweep passes
    // multi-rank: ghost-row exchanges of the two-sweep passes run on a comm stream while the
    // pass's interior strips run (NSGPU_OVERLAP=0: exchange, then the whole pass)
    int overlap = 1;
    int helm_b_pend = 0;          // RHS_u / RHS_v ghost rows owed to the first Helmholtz pair pass
    // ghost-row requests riding on the NEXT exchange group (halo_reqs / gather_level), e.g. a
    // multigrid level's post-restriction iterate (MgLevel::phi_ghost)
    struct Piggy { const nsg::Geo* g; double* f; int w; };
    Piggy piggy[4];
    int npiggy = 0;
    hipStream_t cst = nullptr;
    // multi-rank: CUs reserved for the comm stream (its RCCL kernels run beside the compute
    // stream's strips instead of queueing behind them; NSGPU_COMM_CUS, 0 = no masks)
    int comm_cus = 0, compute_cus = 0;
    hipEvent_t xev[2] = {nullptr, nullptr};
    hipEvent_t fev = nullptr;     // fetch_begin / fetch_end: the scalars' copy to the host is done
    // ns_step_async: the step's min/max travel to mm_host behind the step's last kernel (mev);
    // read by the next ns_step_async (after that step's first host sync) or by ns_monitor
    double* mm_host = nullptr;
    hipEvent_t mev = nullptr;
    int mm_pending = 0;
    int extrap_pending = 0;       // ns_step: the phi extrapolation waits to hide a host sync
    std::vector<MgLevel> lv;     // multigrid hierarchy (NS_POISSON_MG)
    int mg_pre = 2, mg_post = 2, mg_coarse_iters = 0;
    double mg_omega_c = 1.0, mg_omega_s = 1.1;
    bool mg_coarse_lds = false;
    // r4: the coarsest level solved exactly by its separable eigen-decomposition (k_direct, two
    // launches): the first whole coarse level of <= direct_cells cells (NSGPU_DIRECT_CELLS, default
    // 128^2; 0 = the LDS V-cycle below it as in round 3).  dmat: P1 = Vx^-1, Q1 = Vy^-T, E, P2 = Vx,
    // Q2 = Vy^T (direct_setup), padded to multiples of 16
    // r4: a V-cycle boundary on the finest level in one pass (k_sweep4): cycle c's prolongation pass
    // is deferred when c's output is not checked (p_pending) and runs fused with cycle c+1's
    // restriction pass.  NSGPU_FUSE4=0: the two passes (A/B, the equivalence test's reference)
    int fuse4 = 1;
    bool p_pending = false;
    // r4: the phi extrapolation formed inside the solve's first restriction pass (k_sweep2_gin) instead
    // of by k_axpby: extrapolate_phi only rotates the planes and leaves the guess's sources here;
    // K3 then runs speculatively behind the Helmholtz check.  Measured (r4, 4096^2 driver form): the
    // pass takes 241 us (184 VGPRs, 2 waves / SIMD, five streams) against FUSE_R 87 + k_axpby 104 us,
    // 9,924-9,961 vs 9,957-10,143 MLUPS -- so opt-in (NSGPU_GIN=1); default k_axpby (round 3)
    int gin = 0;
    bool gin_pending = false;
    const double* gin_src[4] = {nullptr, nullptr, nullptr, nullptr};
    double gin_c[4] = {0, 0, 0, 0};
    bool mg_direct = false;
    long direct_cells = 128L * 128L;
    double* dmat = nullptr;
    const double *dP1 = nullptr, *dQ1 = nullptr, *dE = nullptr, *dP2 = nullptr, *dQ2 = nullptr;
    // NEUMANN outflow (pois_solve_krylov): BiCGStab planes r, r0, p, v, s, t, ph, sh, scratch
    // (null without an outflow side) and the recurrence scalars
    double* kv[9] = {};
    double* kv_mem = nullptr;
    double* lrow = nullptr;      // outflow preconditioner: its line solution (one row, in kv_mem)
    double* cvimg = nullptr;     // the LDS coarse V-cycle's image (nsg::cv_image), cv_n doubles
    int cv_n = 0, cv_dn = 0;
    double* ksc = nullptr;
    bool pc_active = false;      // inside mg_precond: level 0 has no mean shift
    bool pc_timing = false;      // ... and its level-0 passes are timed (the outflow Poisson solve)
    bool krylov_mg = false;      // the Poisson BiCGStab is preconditioned by a V-cycle (else Jacobi)
    // the outflow preconditioner: a rectangle whose only NEUMANN side is W (0) or
    // E (1): the V-cycle's hierarchy closes that side with a Dirichlet-centre ghost whose data,
    // on the finest level, is the side's 1-D line solve (launch_line_solve); -1 = walls
    int out_side = -1;
    bool consist = false;        // stretched grid, no outflow: consistent_rhs() before every Poisson solve
    bool fps_xuni = true;        // (r6) the direct solve's hx is uniform (false: x-stretched, unfused, no pivot fixed points)
    // (r6) the dense y transforms (hy stretched, or an ny no FFT plan takes): Ly's eigenvectors through rocSOLVER's
    // tridiagonal eigensolver at create, the transforms as rocBLAS GEMMs (F: forward, G: inverse, N x N each)
    bool fps_dense = false;
    rocblas_handle rb = nullptr;
    double *dense_mem = nullptr, *dF = nullptr, *dG = nullptr;
    double area = 0.0;           // sum of the domain's cell areas
    double inv_area = 0.0;       // sum of their reciprocals
    int32_t* fc_mem = nullptr;   // masked domain: topology plane (g.fc) and edge table (g.et)
    int32_t* mband_tiles = nullptr;   // (r6) masked, one rank: the (li0, j0) of the mt tiles holding a wall-band cell
    int mband_n = 0;
    int32_t* ecell_mem = nullptr;   // (r5) masked domain: the slab's domain cells that are not FC_DEEP (g.ecell)
    nsg::EdgeDev* et_mem = nullptr;
    ns_host_transport ht{};      // host transport (ht.exchange != NULL) instead of RCCL
    double* stage = nullptr;     // pinned staging for the host transport
    size_t stage_n = 0;
    // masked domain: this slab's bounding-box cells -> compact cell id - cid0 (-1 outside), so
    // ns_get_fields / ns_set_fields speak the reference's compact Vec order (Grid.cpp:149-162)
    std::vector<int32_t> cid;
    int64_t cid0 = 0, ncid = 0;  // first compact id of the slab and its in-domain cell count
    std::vector<double> hbuf;    // host bounding-box staging for that gather / scatter
    // NSGPU_RCCL_LOOPBACK=1 (test / measurement hook): a 1-rank RCCL communicator whose every
    // peer is this process.  One rank: every exchange point of the step runs its RCCL group with
    // peer == self (both ghost sides from this slab's own edge rows) and every reduction an
    // ncclAllReduce -- the multi-rank call sites on one GPU; ghost rows beyond the walls carry
    // zero weight, so the step is the plain single-rank step.  nranks > 1 with neither an
    // ncclUniqueId nor a host transport: a VIRTUAL slab -- rank `rank`'s slab, hierarchy,
    // launches and RCCL groups (exchanges, the agglomeration gather) with self as every peer,
    // reductions over this slab only: the per-rank time of a multi-GPU step without the other
    // GPUs (tools/slab_projection.py).
    int loopback = 0;
    // virtual slab only (NSGPU_VIRTUAL_ITERS="h:c,h:c,..."): the slab's own residuals are not the
    // global solve's, so each step replays the global run's Helmholtz sweeps h and V-cycles c
    // (cycled over the list), with one residual check (host sync) per solve like a predicted one
    std::vector<std::pair<int, int>> replay;
    size_t replay_k = 0;
    int rp_h = 0, rp_c = -1;        // this step's replayed counts (0 / -1: converge normally)
    int n_xchg = 0, n_allred = 0;   // exchange groups / all-reduces issued in the current step
    double x_link = 0.0;            // bytes over this rank's busiest peer link in the current step
    // speculative CorrectVelocities: inside a time step, the multigrid's residual check that
    // the cycle history predicts to pass enqueues K5 (into the ping-pong partners, with its
    // min/max) BEFORE the host waits for the residual, so the GPU works through the host round
    // trip; k5_spec = 1 after a passing check (the step then only swaps), 0 otherwise (K5 runs
    // again after the last cycle: u* is untouched, K5 writes TMPU / TMPV)
    int in_step = 0, k5_spec = 0, n_spec = 0, n_spec_hit = 0;
    int speculate = 1;           // NSGPU_SPECULATE=0: no speculative K5 / K3 (the equivalence test's reference)
    // r4: K5 may form the next step's Poisson guess (k_cell_s<6>, NSGPU_K5_GUESS=1; default: k_axpby
    // at the next step as in round 3); guess_ready: TMP holds it (branch guess_branch of extrap_plan) -- any entry
    // point that may write TMP or the phi planes clears it.  K3 then runs speculatively behind the
    // Helmholtz residual check (k3_spec: rhs_phi is this step's), which the extrapolation used to fill
    // Measured (r4, 4096^2 driver form): k_cell_s<6> 242 us against K5 128 + k_axpby 104 us -- no gain
    // (9,819-9,822 vs 9,821-9,863 MLUPS), so it is opt-in (NSGPU_K5_GUESS=1)
    int k5_guess = 0, guess_ready = 0, guess_branch = 0, k3_spec = 0;
    int cur_cycles = -1;         // V-cycles of the Poisson solve in progress (at its K5)
    int last_cycles = -1;        // V-cycles of the last multigrid solve (-1: none / Krylov)
    // r4: the direct Poisson solve (ns_fps.hip) of a rectangle with zero-flux phi sides and uniform hy
    // (ny a power of two): DCT along y, tridiagonal recurrences along x, inverse DCT -- no iteration,
    // so no initial guess (no phi history planes).  Its output residual (a separate pass: 76 us at
    // 4096^2) is checked on the first solve of a run and every fps_check-th after it (NSGPU_FPS_CHECK,
    // default 16; 1 = every solve; a standalone ns_kernel solve always); the check's host sync hides
    // behind a speculative K5, and a residual above rtol continues with multigrid V-cycles from this
    // phi.  The solve is a fixed arithmetic sequence: its residual does not drift between checks
    // (1e-13 .. 1e-12 of ||b|| at 4096^2).  NSGPU_FPS=0: multigrid
    bool fps = false;
    bool fps_pc = false;         // masked domain: the bounding box's direct solve preconditions BiCGStab (NSGPU_FPS_PC=0: V-cycle)
    // (r5) and, with at most NSGPU_CAP_MAX (4096) interface faces, the exact solve by the capacitance matrix
    // (cap_setup / cap_solve; NSGPU_CAP=0: BiCGStab preconditioned by the box's solve, A/B)
    nsg::CapArgs cap{};
    void* cap_mem = nullptr;
    nsg::FpsArgs fa{};
    double* fps_mem = nullptr;
    const double *fps_tw = nullptr, *fps_wk = nullptr;
    const double* fps_tw8 = nullptr;   // (r5) ny = 16384: the 8192-point halves' twiddles
    int fps_check = 16;
    int fps_passes = 2;          // full passes of the tridiagonal recurrences (NSGPU_FPS_PASSES=3: t1 / t2 / t3)
    long fps_solves = 0;
    // multi-rank: this rank's aggregate of a recurrence (2 x ld), every rank's (nranks x 2 x ld, one
    // allgather per direction and solve) and the carry-in folded from them (ld)
    double *fps_ragg = nullptr, *fps_gath = nullptr;
    size_t fps_n = 0;            // (r5) the allgather's slot: 2 x ld aggregates + (sum b, sum b^2) + padding
    // (r5) ONE allgather per solve (NSGPU_FPS_ONEGATHER=0: two, A/B): the slot also carries the rank's backward
    // aggregate with a zero forward carry-in (2 more ld), which is affine in that carry-in (FpsRank::bq); og_b /
    // og_x1: the host tables B_p (every rank, per mode) and X1_p
    bool fps_og = false, fps_og_mean = false;
    const double *og_b = nullptr, *og_x1 = nullptr;
    // r5, multi-rank rectangles on the direct solve: the fused K3's sums are not all-reduced -- they ride
    // on the recurrences' forward allgather (at 2 ld of each rank's slot), and the mean comes off mode 0
    // afterwards, as the linear response of its aggregates to the constant ny * mean (host tables m0: every
    // local chunk's E / BXl and group's aggregate of the constant 1, every rank's; fps_setup).
    // NSGPU_FPS_DEFER=0: the all-reduce before the solve (A/B).  mean_pend: this step's sums wait there
    bool fps_defer = false, mean_pend = false;
    const double *m0e = nullptr, *m0b = nullptr, *m0g = nullptr, *m0a = nullptr;
    double fps_res = -1.0;       // the last checked solve's relative residual
    int kpred[3] = {1, 1, 1};    // (r5) the last BiCGStab solve's iterations: Poisson, Helmholtz u, v (bicgstab's batch)
    // (r5) a masked domain's Helmholtz solve on one rank by red-black SOR (NSGPU_MASK_HELM=krylov: BiCGStab); the
    // sweeps the last step needed (the next step's first batch)
    bool mask_rb = true, mask_rbt = true;
    bool mask_mt = true;   // (r6) masked Helmholtz: up to 4 sweeps per launch + the residual in the last (NSGPU_MASK_MT=0: rbt)
    int mask_band = 6;     // (r6) masked Helmholtz: wall-band sweeps before the global ones (NSGPU_MASK_BAND; 0 off, multiple of 6)
    int mask_helm_next = 4, mask_helm_ok = 0;
    // r5, multi-rank rectangles: the Helmholtz check's collective is an allgather of every rank's
    // S_HBNL .. S_MML (bus()): K1's norms and the previous step's K5 min / max ride on it, so neither
    // takes a collective of its own (NSGPU_BUS=0: the per-reduction all-reduces, A/B); bus_mem holds
    // the P gathered slots of BUS_NV values
    bool bus = false;
    double* bus_mem = nullptr;
    // r5, multi-rank rectangles on the direct solve: DEEP ghost rows.  K1 computes its rows and deep_e =
    // 8 + 6 R rows of each neighbour's slab (R: the wall bands' 3-sweep launches), its exchange carrying u,
    // v, phi that deep; the band launches then compute 6 rows fewer each and need no exchange, and the
    // residual 3-sweep pass finds its 7-row cone valid and computes one neighbour row more, which K3 reads --
    // one exchange group (K1's) where r4 had 1 + R + 1 + 1 (deep_geo; NSGPU_DEEP=0: the r4 exchanges, A/B).  hp: the finest planes' ghost rows per side
    // (HALO, or deep_e + HALO + 2); cu_ext / u_ext: ghost rows of cu, cv / of u, v (the Helmholtz
    // iterates) known valid now
    int hp = nsg::HALO;
    bool deep = false;
    int deep_e = 0, cu_ext = 0, u_ext = 0;
    int phi_ext = 0;             // (r5) phi's ghost row valid from the direct solve (deep slabs, k_fps_t2b's ghost rows)
    bool fps_strict = false;     // a check failed or came within 1/100 of rtol: check every solve
    bool hbn_pend = false;       // slabs: K1's ||RHS||^2 partial sums await the Helmholtz check's all-reduce
    // K3 fused into the direct solve's DCT (r4, launch_fps_div; NSGPU_FPS_FUSE=0: K3 + the DCT): inside
    // steps the divergence goes straight into the transformed plane, rhs_phi is stored only for a checked
    // solve; fps_pre: the plane holds this step's coefficients (pois_solve_fps skips its DCT)
    bool fps_fuse = true, fps_pre = false, fps_pre_b = false;
    // timed steps: K1 (kev[0..1]) and the direct solve's transforms / recurrences (kev[2..7]); (r6) the wall-band
    // launches (kev[8..11], two launches) and K5 (kev[12..13], read at the next host sync: k5_pend)
    hipEvent_t kev[14] = {};
    int band_timed = 0, k5_pend = 0;
    // (r6) the deferred correction: an ns_step_async step ends after its Poisson solve (U, V = u*, v*, PHI = phi^n)
    // and the next step's K1 applies CorrectVelocities on the fly (k_rhs_sc: K5 folded into K1 -- one HBM pass
    // of 40 B/cell less); any other entry point that reads or writes the fields runs K5 first (materialize)
    bool k5_defer_ok = false;    // one rank, rectangle, no NEUMANN side, the direct solve, hy uniform, streaming K1
    int corr_pend = 0, defer_now = 0, corr_k1 = 0;   // corr_k1: this step's K1 applied a deferred correction
};

namespace {

int ensure_stage(ns_solver* s, size_t n) {
    if (s->stage_n >= n) return 0;
    if (s->stage) HIPCHK(hipHostFree(s->stage));
    s->stage = nullptr;
    HIPCHK(hipHostMalloc(&s->stage, n * sizeof(double), hipHostMallocDefault));
    s->stage_n = n;
    return 0;
}

// one ghost-row request: `w` rows (contiguous: w * ld doubles) of field f on level geometry g
struct HaloReq {
    const nsg::Geo* g;
    double* f;
    int w;
};

// the RCCL / host-transport call sites are live: several ranks, or the one-rank loopback
inline bool comm_on(const ns_solver* s) { return s->nranks > 1 || s->loopback; }

// the RCCL send / recv pairs of ghost-row requests (inside the caller's ncclGroupStart / End)
int halo_rccl(ns_solver* s, const HaloReq* reqs, int nreq, hipStream_t xs) {
    const bool lo = s->rank > 0 || s->nranks == 1, hi = s->rank < s->nranks - 1 || s->nranks == 1;
    const int p_lo = s->loopback ? 0 : s->rank - 1, p_hi = s->loopback ? 0 : s->rank + 1;
    const bool self = s->nranks == 1;
    for (int k = 0; k < nreq; k++) {
        const HaloReq& q = reqs[k];
        const size_t cnt = (size_t)q.w * q.g->ld;
        const int ld = q.g->ld, nxl = q.g->nxl;
        double* f = q.f;
        const double *flo = self ? f - (ptrdiff_t)q.w * ld : f, *fhi = f + (ptrdiff_t)(self ? nxl : nxl - q.w) * ld;
        s->x_link += 8.0 * (double)cnt;   // (each side is its own link)
        if (lo) {
            NCCLCHK(ncclSend(flo, cnt, ncclDouble, p_lo, s->comm, xs));
            NCCLCHK(ncclRecv(f - (ptrdiff_t)q.w * ld, cnt, ncclDouble, p_lo, s->comm, xs));
        }
        if (hi) {
            NCCLCHK(ncclSend(fhi, cnt, ncclDouble, p_hi, s->comm, xs));
            NCCLCHK(ncclRecv(f + (ptrdiff_t)nxl * ld, cnt, ncclDouble, p_hi, s->comm, xs));
        }
    }
    return 0;
}

// ghost rows to / from the x-neighbours; every request of the list goes in ONE RCCL group
// (one latency for all of them)
int halo_reqs(ns_solver* s, const HaloReq* reqs_in, int nreq_in, hipStream_t xs = nullptr) {
    if (!xs) xs = s->st;
    if (!comm_on(s)) return 0;
    s->n_xchg++;
    // the requests riding along (ns_solver::piggy) join this group; a list that does not fit is
    // an error, never a silently dropped request (its level would read stale ghost rows)
    constexpr int MAXREQ = 8 + 4;
    if (nreq_in < 0 || nreq_in + s->npiggy > MAXREQ) {
        set_err("halo exchange: %d requests + %d riding along exceed %d", nreq_in, s->npiggy, MAXREQ);
        return NS_EINVAL;
    }
    HaloReq reqs[MAXREQ];
    int nreq = 0;
    for (int k = 0; k < nreq_in; k++) reqs[nreq++] = reqs_in[k];
    for (int k = 0; k < s->npiggy; k++) reqs[nreq++] = HaloReq{s->piggy[k].g, s->piggy[k].f, s->piggy[k].w};
    s->npiggy = 0;
    const bool lo = s->rank > 0 || s->nranks == 1, hi = s->rank < s->nranks - 1 || s->nranks == 1;
    // (loopback: the 1-rank communicator's only rank, 0, is every peer; a one-rank loopback sends
    // its physical ghost rows round trip unchanged -- they may hold boundary data, e.g. the
    // outflow preconditioner's)
    const bool self = s->nranks == 1;
    if (s->ht.exchange) {
        for (int k = 0; k < nreq; k++) {
            const HaloReq& q = reqs[k];
            const size_t cnt = (size_t)q.w * q.g->ld;
            const int ld = q.g->ld, nxl = q.g->nxl;
            double* f = q.f;
            CHK(ensure_stage(s, 4 * cnt));
            double *slo = s->stage, *shi = slo + cnt, *rlo = shi + cnt, *rhi = rlo + cnt;
            const double *flo = self ? f - (ptrdiff_t)q.w * ld : f, *fhi = f + (ptrdiff_t)(self ? nxl : nxl - q.w) * ld;
            s->x_link += 8.0 * (double)cnt;   // (as halo_rccl: each side is its own link)
            if (lo) HIPCHK(hipMemcpyAsync(slo, flo, cnt * 8, hipMemcpyDeviceToHost, xs));
            if (hi) HIPCHK(hipMemcpyAsync(shi, fhi, cnt * 8, hipMemcpyDeviceToHost, xs));
            HIPCHK(hipStreamSynchronize(xs));
            if (s->ht.exchange(s->ht.user, lo ? slo : nullptr, hi ? shi : nullptr, lo ? rlo : nullptr,
                               hi ? rhi : nullptr, (int64_t)cnt) != 0) {
                set_err("host transport exchange failed");
                return NS_ERCCL;
            }
            if (lo) HIPCHK(hipMemcpyAsync(f - (ptrdiff_t)q.w * ld, rlo, cnt * 8, hipMemcpyHostToDevice, xs));
            if (hi) HIPCHK(hipMemcpyAsync(f + (ptrdiff_t)nxl * ld, rhi, cnt * 8, hipMemcpyHostToDevice, xs));
            HIPCHK(hipStreamSynchronize(xs));
        }
        return 0;
    }
    NCCLCHK(ncclGroupStart());
    CHK(halo_rccl(s, reqs, nreq, xs));
    NCCLCHK(ncclGroupEnd());
    return 0;
}

// A two-sweep pass whose ghost rows must be exchanged first: the pass's interior strips (their
// read cone inside the slab) are launched on the compute stream, the exchange runs on the comm
// stream meanwhile, and the edge strips follow once it is done (nsg::set_strip_phase).  Every
// RCCL call stays totally ordered across streams: the exchange waits for everything before the
// pass, and everything after it waits for the exchange.  `launch` launches the pass (k_sweep2
// launchers only) and returns its partial count or < 0.
int halo_reqs(ns_solver* s, const HaloReq* reqs, int nreq, hipStream_t xs);
template <class F>
int overlapped(ns_solver* s, const HaloReq* reqs, int nreq, F&& launch) {
    if (!comm_on(s) || !s->overlap || !s->cst) {
        CHK(halo_reqs(s, reqs, nreq, s->st));
        return launch();
    }
    HIPCHK(hipEventRecord(s->xev[0], s->st));
    nsg::set_strip_phase(1);
    int n = launch();
    nsg::set_strip_phase(0);
    if (n < 0) return n;
    HIPCHK(hipStreamWaitEvent(s->cst, s->xev[0], 0));
    CHK(halo_reqs(s, reqs, nreq, s->cst));
    HIPCHK(hipEventRecord(s->xev[1], s->cst));
    HIPCHK(hipStreamWaitEvent(s->st, s->xev[1], 0));
    nsg::set_strip_phase(2);
    n = launch();
    nsg::set_strip_phase(0);
    return n;
}

int halo_reqs(ns_solver* s, std::initializer_list<HaloReq> reqs) {
    return halo_reqs(s, reqs.begin(), (int)reqs.size());
}

int halo_g(ns_solver* s, const nsg::Geo& g, std::initializer_list<double*> fields, int w) {
    if (!comm_on(s)) return 0;
    HaloReq r[4];
    int n = 0;
    for (double* f : fields)
        if (n < 4) r[n++] = HaloReq{&g, f, w};
    return halo_reqs(s, r, n);
}

int halo(ns_solver* s, std::initializer_list<double*> fields, int w) { return halo_g(s, s->g, fields, w); }

// (r5) the geometry of a launch that also computes e rows of each neighbour's slab (none beyond the domain);
// *elo = the rows added below (pointers into the planes move down by as many rows: shp); reductions keep to
// the slab's own rows (Geo::sr0 / sr1)
nsg::Geo deep_geo(const ns_solver* s, int e, int* elo) {
    nsg::Geo g = s->g;
    const int lo = std::min(e, g.i0), hi = std::min(e, g.nx - g.i0 - g.nxl);
    g.i0 -= lo;
    g.nxl += lo + hi;
    g.sr0 = lo;
    g.sr1 = lo + s->g.nxl;
    *elo = lo;
    return g;
}
inline double* shp(double* p, int elo, int ld) { return p - (ptrdiff_t)elo * ld; }

int allreduce(ns_solver* s, double* d, int n, ncclRedOp_t op) {
    if (!comm_on(s)) return 0;
    s->n_allred++;
    if (s->ht.allreduce) {
        CHK(ensure_stage(s, std::max(n, 64)));
        HIPCHK(hipMemcpyAsync(s->stage, d, n * 8, hipMemcpyDeviceToHost, s->st));
        HIPCHK(hipStreamSynchronize(s->st));
        if (s->ht.allreduce(s->ht.user, s->stage, n, op == ncclMin ? 1 : 0) != 0) {
            set_err("host transport allreduce failed");
            return NS_ERCCL;
        }
        HIPCHK(hipMemcpyAsync(d, s->stage, n * 8, hipMemcpyHostToDevice, s->st));
        return 0;
    }
    NCCLCHK(ncclAllReduce(d, d, n, ncclDouble, op, s->comm, s->st));
    return 0;
}

// the multi-rank scalar bus (r5): one allgather of every rank's S_HBNL .. S_MML, folded in rank order
// into S_HBN (K1's ||RHS||^2), S_RES / S_AUX (the Helmholtz residuals) and S_MM (K5's min / max):
// sums for the first BUS_NSUM values, mins after
int allgather(ns_solver* s, const double* mine, double* all, size_t n);
int bus(ns_solver* s) {
    static const int dst[BUS_NV] = {S_HBN, S_HBN + 1, S_RES, S_RES + 1, S_AUX, S_AUX + 1,
                                    S_MM, S_MM + 1, S_MM + 2, S_MM + 3};
    static_assert(S_RESL == S_HBNL + 2 && S_AUXL == S_RESL + 2 && S_MML == S_AUXL + 2 && S_MML + 4 == S_HBNL + BUS_NV,
                  "the bus payload is S_HBNL .. S_MML, contiguous");
    CHK(allgather(s, s->scal + S_HBNL, s->bus_mem, BUS_NV));
    nsg::launch_bus_reduce(s->bus_mem, s->nranks, BUS_NV, BUS_NSUM, dst, s->scal, s->st);
    return 0;
}
// the bus carries this step's reductions (inside a step of a multi-rank rectangle)
inline bool bus_on(const ns_solver* s) { return s->bus && s->in_step; }

// copy all device scalars to the host and wait: the only host syncs of a step
int fetch(ns_solver* s) {
    HIPCHK(hipMemcpyAsync(s->hs, s->scal, S_NUM * sizeof(double), hipMemcpyDeviceToHost, s->st));
    HIPCHK(hipStreamSynchronize(s->st));
    return 0;
}

// the same in two halves: work enqueued between them (independent of the scalars) keeps the
// GPU busy while the host waits for the copy and decides what to launch next
int fetch_begin(ns_solver* s) {
    HIPCHK(hipMemcpyAsync(s->hs, s->scal, S_NUM * sizeof(double), hipMemcpyDeviceToHost, s->st));
    HIPCHK(hipEventRecord(s->fev, s->st));
    return 0;
}
int fetch_end(ns_solver* s) {
    HIPCHK(hipEventSynchronize(s->fev));
    return 0;
}
int extrapolate_phi(ns_solver* s);

// A timed kernel call.  One rank: the call is a single launch, timed by the dispatch's own
// begin / end stamps (hipExtLaunchKernel's events: the interval rocprofv3's kernel trace
// reports).  Multi-rank calls (exchanges, split launches) and NSGPU_EXT_TIMING=0: marker
// events around the call, which also count the launch's dispatch latency.
int t_begin(ns_solver* s, hipEvent_t a, hipEvent_t b) {
    if (s->nranks == 1 && s->ext_timing) {
        nsg::time_next_launch(a, b);
        return 0;
    }
    HIPCHK(hipEventRecord(a, s->st));
    return 0;
}
int t_end(ns_solver* s, hipEvent_t a, hipEvent_t b) {
    if (s->nranks == 1 && s->ext_timing) {
        if (nsg::time_next_launch_pending()) {   // the call launched no kernel: an empty interval
            HIPCHK(hipEventRecord(a, s->st));
            HIPCHK(hipEventRecord(b, s->st));
        }
        return 0;
    }
    HIPCHK(hipEventRecord(b, s->st));
    return 0;
}
int ensure_kev(ns_solver* s) {
    for (auto& e : s->kev)
        if (!e) HIPCHK(hipEventCreate(&e));
    return 0;
}
float kev_ms(ns_solver* s, int k) {
    float ms = 0.f;
    return hipEventElapsedTime(&ms, s->kev[k], s->kev[k + 1]) == hipSuccess ? ms : 0.f;
}
int ensure_events(ns_solver* s, size_t n) {
    while (s->ev.size() < n) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        s->ev.push_back(e);
    }
    if (s->evtag.size() < n / 2 + 1) s->evtag.resize(n / 2 + 1, 0);
    return 0;
}

// Helmholtz sweeps of the fields in `which` (1 = u, 2 = v, 3 = both): U,V -> TMPU,TMPV, then
// swap so NS_ARR_U/V stay "current".  Partials: u at part[0, nb), v at part[nb, 2 nb).
int helm_sweep(ns_solver* s, double alpha, double* part, int which = 3) {
    const int nb = nsg::launch_helm_sweep(s->g, s->c, alpha, s->omega_v, s->arr[NS_ARR_U], s->arr[NS_ARR_V],
                                          s->arr[NS_ARR_TMPU], s->arr[NS_ARR_TMPV], s->arr[NS_ARR_RU],
                                          s->arr[NS_ARR_RV], part, s->st, which);
    if (which & 1) std::swap(s->arr[NS_ARR_U], s->arr[NS_ARR_TMPU]);
    if (which & 2) std::swap(s->arr[NS_ARR_V], s->arr[NS_ARR_TMPV]);
    return nb;
}

// three Helmholtz sweeps in one pass (k_sweep3; with `part`: + the output residual, one rank), then
// swap; a residual pass of one component is HIP-event timed like the pairs (24 B/cell either way:
// the bench's Helmholtz-pass roofline)
int helm_sweep3(ns_solver* s, double alpha, int which, double* part = nullptr) {
    const bool t = s->timing && which != 3 && part;
    if (t) {
        if (s->hev.size() < 2 * (size_t)(s->hn + 1)) {
            const size_t old = s->hev.size();
            s->hev.resize(2 * (size_t)(s->hn + 8));
            for (size_t k = old; k < s->hev.size(); k++)
                if (hipEventCreate(&s->hev[k]) != hipSuccess) { set_err("hipEventCreate failed"); return -1; }
        }
        if (t_begin(s, s->hev[2 * s->hn], s->hev[2 * s->hn + 1]) != 0) return -1;
    }
    const int nb = nsg::launch_helm_sweep3(s->g, s->c, alpha, s->omega_v, s->arr[NS_ARR_U], s->arr[NS_ARR_V],
                                           s->arr[NS_ARR_TMPU], s->arr[NS_ARR_TMPV], s->arr[NS_ARR_RU],
                                           s->arr[NS_ARR_RV], s->st, which, part);
    if (nb < 0) return nb;
    if (t) {
        if (t_end(s, s->hev[2 * s->hn], s->hev[2 * s->hn + 1]) != 0) return -1;
        if (s->hcomp.size() <= (size_t)s->hn) s->hcomp.resize(s->hn + 8, 1);
        s->hcomp[s->hn++] = 1;
    }
    if (which & 1) std::swap(s->arr[NS_ARR_U], s->arr[NS_ARR_TMPU]);
    if (which & 2) std::swap(s->arr[NS_ARR_V], s->arr[NS_ARR_TMPV]);
    return nb;
}

// two Helmholtz sweeps in one pass (temporal blocking), then swap
int helm_sweep2(ns_solver* s, double alpha, double* part, int which = 3) {
    // timing: one-component passes only (the bench's 24 B/cell roofline figure)
    const bool t = s->timing && which != 3;
    if (t) {
        if (s->hev.size() < 2 * (size_t)(s->hn + 1)) {
            const size_t old = s->hev.size();
            s->hev.resize(2 * (size_t)(s->hn + 8));
            for (size_t k = old; k < s->hev.size(); k++)
                if (hipEventCreate(&s->hev[k]) != hipSuccess) { set_err("hipEventCreate failed"); return -1; }
        }
        if (t_begin(s, s->hev[2 * s->hn], s->hev[2 * s->hn + 1]) != 0) return -1;
    }
    const int nb = nsg::launch_helm_sweep2(s->g, s->c, alpha, s->omega_v, s->arr[NS_ARR_U], s->arr[NS_ARR_V],
                                           s->arr[NS_ARR_TMPU], s->arr[NS_ARR_TMPV], s->arr[NS_ARR_RU],
                                           s->arr[NS_ARR_RV], part, s->st, which);
    if (t) {
        if (t_end(s, s->hev[2 * s->hn], s->hev[2 * s->hn + 1]) != 0) return -1;
        if (s->hcomp.size() <= (size_t)s->hn) s->hcomp.resize(s->hn + 8, 1);
        s->hcomp[s->hn++] = 1;
    }
    if (which & 1) std::swap(s->arr[NS_ARR_U], s->arr[NS_ARR_TMPU]);
    if (which & 2) std::swap(s->arr[NS_ARR_V], s->arr[NS_ARR_TMPV]);
    return nb;
}

// `n` Helmholtz sweeps: pairs in one pass each (ghost width 4, 5 with a residual), a single
// sweep for an odd remainder.  Residual partials of the LAST launch go to `part_last`, of the
// first launch to `part_first` (either may be null): a pair reports the residual of its
// output, a single sweep that of its input.  Returns the last launch's partial count;
// *first_at / *last_at = the sweep count the reported residuals belong to.
// Single rank: all of u's passes, then all of v's (helm_split): each field's rhs is then the
// only re-read stream of its passes and can stay in the Infinity Cache (the outputs are
// non-temporal stores).  Multi-rank: u and v pass by pass, their ghost rows in one exchange.
int helm_sweeps(ns_solver* s, double alpha, int n, double* part_first, double* part_last, int* nb_first,
                int* first_at, int* last_at) {
    int nb = 0;
    // one rank: u's passes, then v's -- or, with helm_uv, a batch of a single 3-sweep residual pass
    // per component as ONE two-field launch (each field's strips twice as long: one resident round)
    const bool split = s->nranks == 1 && !(s->helm_uv && n == 3 && s->sweep3 && s->triple && s->sweep3_res &&
                                          !part_first && !s->tiled);
    for (int which : {split ? 1 : 3, split ? 2 : 0}) {
        if (!which) break;
        int k = 0, launch = 0;
        while (k < n) {
            // sweeps per pass: pairs (single sweeps with NSGPU_SWEEP=tiled), and the batch ends on
            // a pair, whose residual is its output's: 3-sweep passes while >= 5 remain (7 = 3+2+2,
            // 8 = 3+3+2, 11 = 3+3+3+2: a third fewer HBM passes); an odd remainder of >= 3 otherwise
            // starts with a single sweep.  Every pass equals its single sweeps bit for bit, so one
            // rank and slabs agree.  A probing first pass stays a pair (2+3+2)
            int w = std::min(s->tiled ? 1 : 2, n - k);
            if (!s->tiled && !(launch == 0 && part_first)) {
                // (a batch may also end on a 3-sweep pass with the residual stage, 7-row cone:
                // 5 = 3+2, 3 = 3, 6 = 3+3 -- slabs too, with 7 ghost rows)
                const bool end3 = s->sweep3_res;
                if (s->sweep3 && s->triple && (n - k >= 5 || (end3 && (n - k == 3 || n - k == 6)))) w = 3;
                else if (((n - k) & 1) && n - k >= 3) w = 1;
            }
            const bool last = k + w >= n;
            double* part = last ? part_last : (launch == 0 ? part_first : nullptr);
            // iterate ghost rows each pass reads: its cone (3-sweep 6, 2-sweep 4, + 1 with the
            // residual stage; single sweep 2 -- k_sweep reads one, K1 needs two anyway)
            const int hw = w == 3 ? (part ? 7 : 6) : (w == 2 ? (part ? 5 : 4) : 2);
            if (which == 3 && w >= 2 && !s->tiled) {
                // multi-rank pair / triple pass: u and v ghost rows in one exchange, overlapped
                // (the rhs ghost rows -- 6: the residual 3-sweep pass's first stage -- ride along on
                // the solve's first pass)
                const HaloReq r[4] = {{&s->g, s->arr[NS_ARR_U], hw}, {&s->g, s->arr[NS_ARR_V], hw},
                                      {&s->g, s->arr[NS_ARR_RU], 6}, {&s->g, s->arr[NS_ARR_RV], 6}};
                const int nr = s->helm_b_pend ? 4 : 2;
                s->helm_b_pend = 0;
                // (one rank: the two-field residual pass is HIP-event timed as two component passes)
                const bool t2 = s->nranks == 1 && s->timing && part && w == 3;
                if (t2) {
                    if (s->hev.size() < 2 * (size_t)(s->hn + 1)) {
                        const size_t old = s->hev.size();
                        s->hev.resize(2 * (size_t)(s->hn + 8));
                        for (size_t q = old; q < s->hev.size(); q++)
                            if (hipEventCreate(&s->hev[q]) != hipSuccess) { set_err("hipEventCreate failed"); return -1; }
                    }
                    CHK(t_begin(s, s->hev[2 * s->hn], s->hev[2 * s->hn + 1]));
                }
                // (r5, deep ghost rows: the wall bands left u, v valid deep enough -- no exchange; the residual
                // 3-sweep pass then also computes one row of each neighbour's slab, so that K3 finds u*, v*'s ghost
                // row valid and needs no exchange either -- its residual summed over the slab's own rows)
                const bool valid = s->deep && s->u_ext >= hw;
                const int ex = valid && w == 3 && part && s->u_ext >= hw + 1 ? 1 : 0;
                nb = valid ? -1 : 0;
                auto pass = [&]() {
                    if (w == 3 && ex) {
                        int lo = 0;
                        const int ld = s->g.ld;
                        const nsg::Geo gk = deep_geo(s, ex, &lo);
                        return nsg::launch_helm_sweep3(gk, s->c, alpha, s->omega_v, shp(s->arr[NS_ARR_U], lo, ld),
                                                       shp(s->arr[NS_ARR_V], lo, ld), shp(s->arr[NS_ARR_TMPU], lo, ld),
                                                       shp(s->arr[NS_ARR_TMPV], lo, ld), shp(s->arr[NS_ARR_RU], lo, ld),
                                                       shp(s->arr[NS_ARR_RV], lo, ld), s->st, 3, part);
                    }
                    if (w == 3)
                        return nsg::launch_helm_sweep3(s->g, s->c, alpha, s->omega_v, s->arr[NS_ARR_U], s->arr[NS_ARR_V],
                                                       s->arr[NS_ARR_TMPU], s->arr[NS_ARR_TMPV], s->arr[NS_ARR_RU],
                                                       s->arr[NS_ARR_RV], s->st, 3, part);
                    return nsg::launch_helm_sweep2(s->g, s->c, alpha, s->omega_v, s->arr[NS_ARR_U], s->arr[NS_ARR_V],
                                                   s->arr[NS_ARR_TMPU], s->arr[NS_ARR_TMPV], s->arr[NS_ARR_RU],
                                                   s->arr[NS_ARR_RV], part, s->st, 3);
                };
                nb = valid ? pass() : overlapped(s, r, nr, pass);
                s->u_ext = ex;
                if (nb < 0) return nb;
                if (t2) {
                    CHK(t_end(s, s->hev[2 * s->hn], s->hev[2 * s->hn + 1]));
                    if (s->hcomp.size() <= (size_t)s->hn) s->hcomp.resize(s->hn + 8, 1);
                    s->hcomp[s->hn++] = 2;
                }
                std::swap(s->arr[NS_ARR_U], s->arr[NS_ARR_TMPU]);
                std::swap(s->arr[NS_ARR_V], s->arr[NS_ARR_TMPV]);
            } else {
                if (s->helm_b_pend) {
                    s->helm_b_pend = 0;
                    CHK(halo(s, {s->arr[NS_ARR_RU], s->arr[NS_ARR_RV]}, 6));
                }
                if (which == 3) CHK(halo(s, {s->arr[NS_ARR_U], s->arr[NS_ARR_V]}, hw));
                else if (w <= 2) CHK(halo(s, {s->arr[which == 1 ? NS_ARR_U : NS_ARR_V]}, hw));
                nb = w == 3 ? helm_sweep3(s, alpha, which, part)
                            : (w >= 2 ? helm_sweep2(s, alpha, part, which) : helm_sweep(s, alpha, part, which));
                if (nb < 0) return NS_EHIP;
            }
            const int at = w >= 2 ? k + w : k;   // a multi-sweep pass reports its output's residual
            if (launch == 0) {
                if (nb_first) *nb_first = nb;
                if (first_at) *first_at = at;
            }
            if (last) *last_at = at;
            k += w;
            launch++;
        }
    }
    return nb;
}

// one Poisson sweep PHI -> TMP (RB-SOR or Jacobi), then swap
int pois_sweep(ns_solver* s, double* part) {
    int nb;
    if (s->tiled) {
        if (s->poisson == NS_POISSON_JACOBI)
            nb = nsg::launch_pois_jacobi_tiled(s->g, s->c, s->omega, s->arr[NS_ARR_PHI], s->arr[NS_ARR_TMP],
                                               s->arr[NS_ARR_RPHI], s->scal + S_SHIFT, part ? part : s->part, s->st);
        else
            nb = nsg::launch_pois_rbsor_tiled(s->g, s->c, s->omega, s->arr[NS_ARR_PHI], s->arr[NS_ARR_TMP],
                                              s->arr[NS_ARR_RPHI], s->scal + S_SHIFT, part, s->st);
    } else if (s->poisson == NS_POISSON_JACOBI)
        nb = nsg::launch_pois_jacobi(s->g, s->c, s->omega, s->arr[NS_ARR_PHI], s->arr[NS_ARR_TMP],
                                     s->arr[NS_ARR_RPHI], s->scal + S_SHIFT, part ? part : s->part, s->st);
    else
        nb = nsg::launch_pois_rbsor(s->g, s->c, s->omega, s->arr[NS_ARR_PHI], s->arr[NS_ARR_TMP],
                                    s->arr[NS_ARR_RPHI], s->scal + S_SHIFT, part, s->st);
    std::swap(s->arr[NS_ARR_PHI], s->arr[NS_ARR_TMP]);
    return nb;
}

// fp32-field planes (phi, partner, rhs), zeroed once: the ghost rows and the row padding stay finite
int ensure_f32(ns_solver* s) {
    if (s->f32_mem) return 0;
    if (hipMalloc(&s->f32_mem, 3 * s->plane * sizeof(float)) != hipSuccess) {
        set_err("hipMalloc of the fp32 planes failed");
        return NS_ENOMEM;
    }
    HIPCHK(hipMemsetAsync(s->f32_mem, 0, 3 * s->plane * sizeof(float), s->st));
    for (int k = 0; k < 3; k++) s->f32[k] = s->f32_mem + k * s->plane + (size_t)s->hp * s->g.ld;
    return 0;
}

// the fp32 planes seen as rows of g.ld / 2 doubles (the ghost-row exchange moves doubles)
nsg::Geo f32_view(const ns_solver* s) {
    nsg::Geo v = s->g;
    v.ld = s->g.ld / 2;
    return v;
}

// one fp32-field Jacobi sweep f32[0] -> f32[1] (residual partials of the input), then swap
int pois_sweep32(ns_solver* s, double* part, int* nb) {
    const nsg::Geo v = f32_view(s);
    CHK(halo_g(s, v, {reinterpret_cast<double*>(s->f32[0])}, 1));
    *nb = nsg::launch_pois_jacobi32(s->g, s->c, s->omega, s->f32[0], s->f32[1], s->f32[2], s->scal + S_SHIFT,
                                    part ? part : s->part, s->st);
    if (*nb < 0) { set_err("fp32 Jacobi sweep: launch failed or plane past 4 GiB"); return NS_EINVAL; }
    std::swap(s->f32[0], s->f32[1]);
    return 0;
}

// phi, rhs_phi -> the fp32 planes
int to_f32(ns_solver* s) {
    CHK(ensure_f32(s));
    nsg::launch_to_f32(s->g, s->arr[NS_ARR_PHI], s->f32[0], s->st);
    nsg::launch_to_f32(s->g, s->arr[NS_ARR_RPHI], s->f32[2], s->st);
    HIPCHK(hipGetLastError());
    return 0;
}

int next_batch(int prev_batch, double prev_r2, int prev_at, double r2, int at, double tol2, int cap) {
    // geometric model of the residual contraction between two checks
    if (prev_r2 > 0 && r2 > 0 && r2 < prev_r2 && at > prev_at) {
        const double rate = std::log(r2 / prev_r2) / (double)(at - prev_at);  // < 0
        const double need = std::log(tol2 / r2) / rate;
        int b = (int)std::ceil(need) + 1;
        b = std::max(b, 2);
        b = std::min(b, std::max(64, 4 * prev_batch));
        return std::min(b, cap);
    }
    return std::min(std::max(prev_batch, 2) * 2, cap);
}

struct KrylovSolve {
    int op;
    double alpha;
    bool mg;
    double* x;
    const double* b;
    const double* shift;
    double b2;
    const char* name;
    ns_stats* stt = nullptr;   // the Poisson solve's: its preconditioner's level-0 passes are timed
};

int bicgstab(ns_solver* s, const KrylovSolve& ks, int* its, double* res);
int correct_launch(ns_solver* s, double* part2);
int divergence(ns_solver* s);
bool fps_checks_next(const ns_solver* s);
bool gin_ok(const ns_solver* s);

// the wall bands' relaxation before the global Helmholtz passes (k_helm_band: band_sweeps RB-SOR
// sweeps, 6 by default in launches of 3, of u and v on the cells within band_w = max(32, min(nx,
// ny) / 32) of a wall, the rest held; the residual of the guess u^n lives there).  Slabs: the
// iterates' ghost rows (6: the kernel's cone) and the right-hand sides' (5) before each launch;
// the first global pass exchanges the relaxed iterates' rows again.
int helm_band(ns_solver* s, double alpha) {
    // launches of 3 sweeps: even ones read the band from the iterates and write it to the
    // scratch planes, odd ones back (no tile writes what another reads); an odd count ends with
    // a copy-back.  Slabs: each launch after a 6-row exchange of the planes it reads the band from
    double *U = s->arr[NS_ARR_U], *V = s->arr[NS_ARR_V], *TU = s->arr[NS_ARR_TMPU], *TV = s->arr[NS_ARR_TMPV];
    const int rounds = std::max(1, s->band_sweeps / 3);
    if (s->deep && s->u_ext >= s->deep_e && s->in_step) {
        // (r5) deep ghost rows: round k computes deep_e - 6 (k + 1) rows of each neighbour's slab from the
        // rows K1's exchange brought (u, v) and K1 computed (rhs) -- no exchange; the last round leaves
        // deep_e - 6 R = 8 valid rows for the residual 3-sweep pass (its 7-row cone + the row it computes for K3)
        const int ld = s->g.ld;
        double *RU = s->arr[NS_ARR_RU], *RV = s->arr[NS_ARR_RV];
        int e = s->deep_e;
        for (int k = 0; k < rounds; k++) {
            const bool odd = k & 1;
            e -= 6;
            int lo = 0;
            const nsg::Geo gk = deep_geo(s, e, &lo);
            nsg::launch_helm_band(gk, s->c, alpha, s->omega_v, shp(U, lo, ld), shp(V, lo, ld), shp(odd ? TU : U, lo, ld),
                                  shp(odd ? TV : V, lo, ld), shp(odd ? U : TU, lo, ld), shp(odd ? V : TV, lo, ld),
                                  shp(RU, lo, ld), shp(RV, lo, ld), s->band_w, 0, s->st);
        }
        if (rounds & 1) {
            int lo = 0;
            const nsg::Geo gk = deep_geo(s, e, &lo);
            nsg::launch_helm_band(gk, s->c, alpha, s->omega_v, shp(U, lo, ld), shp(V, lo, ld), shp(TU, lo, ld),
                                  shp(TV, lo, ld), shp(U, lo, ld), shp(V, lo, ld), shp(RU, lo, ld), shp(RV, lo, ld),
                                  s->band_w, 1, s->st);
        }
        s->u_ext = e;
        s->helm_b_pend = 0;
        return 0;
    }
    const bool tb = s->timing && s->in_step && s->nranks == 1;   // (r6: the bench's band line)
    if (tb) CHK(ensure_kev(s));
    if (s->band6 && s->nranks == 1 && rounds == 2) {
        // (r6) one rank, 6 sweeps: ONE launch of 64 x 64 tiles with their 12-cell cone (k_helm_band6) into the
        // scratch planes, then the band cells' copy-back -- 80 B per band cell instead of 2 x 48 (one timed
        // interval: the bench's band line is the pair)
        if (tb) CHK(t_begin(s, s->kev[8], s->kev[9]));
        const int n = nsg::launch_helm_band(s->g, s->c, alpha, s->omega_v, U, V, U, V, TU, TV, s->arr[NS_ARR_RU],
                                            s->arr[NS_ARR_RV], s->band_w, 2, s->st);
        if (n >= 0) {
            nsg::launch_helm_band(s->g, s->c, alpha, s->omega_v, U, V, TU, TV, U, V, s->arr[NS_ARR_RU],
                                  s->arr[NS_ARR_RV], s->band_w, 3, s->st);
            if (tb) {
                CHK(t_end(s, s->kev[8], s->kev[9]));
                s->band_timed = 1;
            }
            return 0;
        }
        if (tb) CHK(t_end(s, s->kev[8], s->kev[9]));   // (unsupported here: the launches of 3 below)
    }
    for (int k = 0; k < rounds; k++) {
        const bool odd = k & 1;
        auto launch = [&]() {
            return nsg::launch_helm_band(s->g, s->c, alpha, s->omega_v, U, V, odd ? TU : U, odd ? TV : V,
                                         odd ? U : TU, odd ? V : TV, s->arr[NS_ARR_RU], s->arr[NS_ARR_RV],
                                         s->band_w, 0, s->st);
        };
        if (tb && k < 2) {
            CHK(t_begin(s, s->kev[8 + 2 * k], s->kev[9 + 2 * k]));
            launch();
            CHK(t_end(s, s->kev[8 + 2 * k], s->kev[9 + 2 * k]));
            s->band_timed = k + 1;
        } else if (s->nranks > 1) {
            // the exchange overlapped with the tiles that read no neighbour's rows
            const HaloReq r[4] = {{&s->g, odd ? TU : U, 6}, {&s->g, odd ? TV : V, 6},
                                  {&s->g, s->arr[NS_ARR_RU], 6}, {&s->g, s->arr[NS_ARR_RV], 6}};
            const int nr = s->helm_b_pend ? 4 : 2;
            s->helm_b_pend = 0;
            const int n = overlapped(s, r, nr, launch);
            if (n < 0) return n;
        } else {
            launch();
        }
    }
    if (rounds & 1)
        nsg::launch_helm_band(s->g, s->c, alpha, s->omega_v, U, V, TU, TV, U, V, s->arr[NS_ARR_RU],
                              s->arr[NS_ARR_RV], s->band_w, 1, s->st);
    return 0;
}

// ---------------- Helmholtz (I - a L_V) u* = RHS_u, v* likewise (KSPSolve(uSolver), FluidSolver.cpp:547-548)
// Initial guess u^n (in place), its wall bands relaxed first: converged solution is the same;
// fewer sweeps than the reference's zero guess.
int helm_solve(ns_solver* s, int* its, double* resu, double* resv) {
    const double alpha = s->dt / (2 * s->re);
    if (s->g.fc && s->nranks == 1 && s->mask_rb) {
        // (r5) masked domain, one rank: red-black SOR on I - alpha L_V (strongly diagonally dominant: alpha / h^2 ~ 0.06
        // at 1024^2), u and v sweep by sweep, the residual of both checked after a batch -- the first batch what
        // the previous step needed (NSGPU_MASK_HELM=krylov: the BiCGStab of rounds 1-4)
        // (||RHS_u||^2, ||RHS_v||^2 come with the first batch's residuals: no host read before it)
        const double tol2 = s->rtol * s->rtol;
        double bu = 0.0, bv = 0.0;
        int sweeps = 0, batch = std::max(1, s->mask_helm_next);
        double r2u = 0.0, r2v = 0.0;
        if (s->mask_mt && s->mask_band > 0 && s->mband_n > 0) {
            // (r6) the wall bands first (the residual of the guess u^n lives there, as on the rectangle): launches
            // of 3 sweeps on the FC_BAND cells, U -> TU, then (U, TU) -> U (an even count: the band ends in U)
            const double *RU = s->arr[NS_ARR_RU], *RV = s->arr[NS_ARR_RV];
            const int nl = s->mask_band / 3;
            for (int l = 0; l < nl; l++) {
                double *U = s->arr[NS_ARR_U], *V = s->arr[NS_ARR_V], *TU = s->arr[NS_ARR_TMPU], *TV = s->arr[NS_ARR_TMPV];
                const bool odd = l & 1;
                const int rc = nsg::launch_helm_mt_mask(s->g, s->c, alpha, s->omega_v, U, V, RU, RV, odd ? U : TU,
                                                        odd ? V : TV, 3, nullptr, s->st, odd ? TU : U, odd ? TV : V,
                                                        s->mband_tiles, s->mband_n);
                if (rc < 0) { set_err("masked wall-band launch failed"); return NS_EINVAL; }
            }
        }
        for (;;) {
            const int n = std::min(batch, s->max_iters - sweeps);
            // (u and v in the same launches: the topology decoded once -- 4 -> 2 launches per sweep)
            double *U = s->arr[NS_ARR_U], *V = s->arr[NS_ARR_V];
            const double *RU = s->arr[NS_ARR_RU], *RV = s->arr[NS_ARR_RV];
            // (r5) whole sweeps in LDS tiles, U, V -> TU, TV -> U, V (an odd batch: its first sweep as the two
            // in-place half-sweeps); NSGPU_MASK_RBT=0: half-sweeps only (A/B)
            double *TU = s->arr[NS_ARR_TMPU], *TV = s->arr[NS_ARR_TMPV];
            if (s->mask_mt) {
                // (r6) up to 4 sweeps per launch (k_helm_mt_mask: LDS temporal blocking), U, V <-> TU, TV, the
                // batch's last launch with the residuals of both fields -- no pass of its own
                const int nl = (n + 3) / 4;
                int left = n, nb = -1;
                bool in_t = false;
                for (int l = 0; l < nl; l++) {
                    const int k = (left + (nl - l) - 1) / (nl - l);
                    nb = nsg::launch_helm_mt_mask(s->g, s->c, alpha, s->omega_v, in_t ? TU : U, in_t ? TV : V, RU, RV,
                                                  in_t ? U : TU, in_t ? V : TV, k, left == k ? s->part : nullptr, s->st);
                    if (nb < 0) { set_err("masked Helmholtz tile launch failed"); return NS_EINVAL; }
                    in_t = !in_t;
                    left -= k;
                }
                if (in_t) {
                    std::swap(s->arr[NS_ARR_U], s->arr[NS_ARR_TMPU]);
                    std::swap(s->arr[NS_ARR_V], s->arr[NS_ARR_TMPV]);
                }
                sweeps += n;
                nsg::launch_reduce_sum(s->part, nb, 2, s->scal + S_RES, s->st);
                CHK(fetch(s));
                bu = s->hs[S_HBN];
                bv = s->hs[S_HBN + 1];
                r2u = s->hs[S_RES];
                r2v = s->hs[S_RES + 1];
                if (!std::isfinite(r2u) || !std::isfinite(r2v)) { set_err("Helmholtz residual is not finite"); return NS_EDIVERGE; }
                if ((r2u <= tol2 * bu && r2v <= tol2 * bv) || sweeps >= s->max_iters) break;
                batch = 2;
                continue;
            }
            for (int k = 0; k < n; k++) {
                if (s->mask_rbt && (n - k) % 2 == 0) {
                    nsg::launch_helm_rbt_mask(s->g, s->c, alpha, s->omega_v, U, V, RU, RV, TU, TV, s->st);
                    nsg::launch_helm_rbt_mask(s->g, s->c, alpha, s->omega_v, TU, TV, RU, RV, U, V, s->st);
                    k++;
                    continue;
                }
                for (int par : {0, 1})
                    nsg::launch_helm_rb_mask(s->g, s->c, alpha, s->omega_v, U, RU, V, RV, par, nullptr, s->st);
            }
            sweeps += n;
            const int nb = nsg::launch_helm_rb_mask(s->g, s->c, alpha, s->omega_v, U, RU, V, RV, 2, s->part, s->st);
            nsg::launch_reduce_sum(s->part, nb, 2, s->scal + S_RES, s->st);
            CHK(fetch(s));
            bu = s->hs[S_HBN];
            bv = s->hs[S_HBN + 1];
            r2u = s->hs[S_RES];
            r2v = s->hs[S_RES + 1];
            if (!std::isfinite(r2u) || !std::isfinite(r2v)) { set_err("Helmholtz residual is not finite"); return NS_EDIVERGE; }
            if ((r2u <= tol2 * bu && r2v <= tol2 * bv) || sweeps >= s->max_iters) break;
            batch = 2;
        }
        *resu = bu > 0 ? std::sqrt(r2u / bu) : std::sqrt(r2u);
        *resv = bv > 0 ? std::sqrt(r2v / bv) : std::sqrt(r2v);
        *its = sweeps;
        // (the next step's first batch: what this one needed; after 4 steps in a row whose first batch sufficed,
        // one sweep fewer -- the flow settles and the solves need fewer sweeps than at the start)
        const bool first_ok = sweeps <= std::max(1, s->mask_helm_next);
        if (first_ok && ++s->mask_helm_ok >= 4) {
            s->mask_helm_next = std::max(2, sweeps - 1);
            s->mask_helm_ok = 0;
        } else {
            s->mask_helm_next = sweeps;
            if (!first_ok) s->mask_helm_ok = 0;
        }
        return 0;
    }
    if (s->g.fc) {
        // masked domain: u then v, each a Jacobi-preconditioned BiCGStab on I - alpha L_V
        CHK(fetch(s));   // ||RHS_u||^2, ||RHS_v||^2
        int iu = 0, iv = 0;
        const KrylovSolve ku{1, alpha, false, s->arr[NS_ARR_U], s->arr[NS_ARR_RU], nullptr, s->hs[S_HBN], "helmholtz u"};
        CHK(bicgstab(s, ku, &iu, resu));
        const KrylovSolve kw{1, alpha, false, s->arr[NS_ARR_V], s->arr[NS_ARR_RV], nullptr, s->hs[S_HBN + 1], "helmholtz v"};
        CHK(bicgstab(s, kw, &iv, resv));
        *its = std::max(iu, iv);
        return 0;
    }
    const double tol2 = s->rtol * s->rtol;
    if (s->helm_band && !s->tiled) CHK(helm_band(s, alpha));
    // first batch: what the previous step needed (consecutive steps converge alike), so a
    // step normally costs one residual check
    int sweeps = 0, batch = s->rp_h > 0 ? s->rp_h : s->helm_next, prev_at = -1;
    const int n0 = batch;
    double prev_r2 = -1;
    double first_r2 = -1, last_r2 = -1;   // max over u, v of r^2 / ||b||^2
    int first_at = 0, last_at = 0;
    double* p0 = s->part + 2 * (size_t)nsg::max_partials(s->g) / 2;  // second half: first-launch residuals
    for (;;) {
        const int n = std::min(batch, s->max_iters - sweeps);
        // the first pass's residual (a fifth pipeline stage: +20 % on that pass) feeds the next
        // step's batch prediction; consecutive steps converge alike, so it is sampled on every
        // 8th step only (and whenever the predicted batch fell short: see below)
        // (not on a batch of <= 3 sweeps: one pass, or 1 + 2 on slabs -- a probing pair would leave
        // a lone last sweep, whose residual is its input's)
        const bool first = sweeps == 0 && n > 3 && (s->helm_probe == 0 || !s->helm_adapt);
        int nb0 = 0, at0 = 0, at = 0;
        const int nb = helm_sweeps(s, alpha, n, first ? p0 : nullptr, s->part, &nb0, &at0, &at);
        at += sweeps;
        sweeps += n;
        const bool ub = bus_on(s);
        nsg::launch_reduce_sum_segs(s->part, nb, 2, s->scal + (ub ? S_RESL : S_RES), s->st);          // u, v
        if (first) nsg::launch_reduce_sum_segs(p0, nb0, 2, s->scal + (ub ? S_AUXL : S_AUX), s->st);
        static_assert(S_RES == S_HBN + 2, "the deferred RHS norms and the residuals in one all-reduce");
        if (ub) {
            // (r5) one allgather: K1's norms, these residuals and the previous step's K5 min / max
            CHK(bus(s));
        } else {
            if (s->hbn_pend) CHK(allreduce(s, s->scal + S_HBN, 4, ncclSum));
            else CHK(allreduce(s, s->scal + S_RES, 2, ncclSum));
            if (first) CHK(allreduce(s, s->scal + S_AUX, 2, ncclSum));
        }
        s->hbn_pend = false;
        CHK(fetch_begin(s));
        if (s->extrap_pending && !s->guess_ready && !(s->gin && gin_ok(s) && s->phim_valid > 0)) {
            // the Poisson initial guess does not depend on u*: it runs on the GPU while the
            // host waits for this check
            s->extrap_pending = 0;
            CHK(extrapolate_phi(s));
        } else if (s->speculate && s->in_step) {
            // (r4: K5 formed the guess) K3 instead: the divergence of this batch's u*, v* --
            // the step's rhs_phi if the check passes, formed again after the next batch if not
            CHK(divergence(s));
            s->k3_spec = 1;
        }
        CHK(fetch_end(s));
        const double r2u = s->hs[S_RES], r2v = s->hs[S_RES + 1];
        const double bu = s->hs[S_HBN], bv = s->hs[S_HBN + 1];
        const bool ok = s->rp_h > 0 || ((r2u <= tol2 * bu || r2u == 0.0) && (r2v <= tol2 * bv || r2v == 0.0));
        *resu = bu > 0 ? std::sqrt(r2u / bu) : std::sqrt(r2u);
        *resv = bv > 0 ? std::sqrt(r2v / bv) : std::sqrt(r2v);
        if (!std::isfinite(r2u) || !std::isfinite(r2v)) { set_err("Helmholtz residual is not finite"); *its = sweeps; return NS_EDIVERGE; }
        if (s->verbose) {
            if (first)
                fprintf(stderr, "nsgpu helmholtz: after %d sweeps rel. residual u %.3e v %.3e\n", at0,
                        std::sqrt(s->hs[S_AUX] / std::max(bu, 1e-300)), std::sqrt(s->hs[S_AUX + 1] / std::max(bv, 1e-300)));
            fprintf(stderr, "nsgpu helmholtz: after %d sweeps rel. residual u %.3e v %.3e\n", at, *resu, *resv);
        }
        const double r2 = std::max(r2u / std::max(bu, 1e-300), r2v / std::max(bv, 1e-300));
        if (first) {
            first_r2 = std::max(s->hs[S_AUX] / std::max(bu, 1e-300), s->hs[S_AUX + 1] / std::max(bv, 1e-300));
            first_at = at0;
        }
        last_r2 = r2;
        last_at = at;
        if (ok || sweeps >= s->max_iters) break;
        if (first) {  // residual after the first launch -> contraction rate
            prev_r2 = std::max(s->hs[S_AUX] / std::max(bu, 1e-300), s->hs[S_AUX + 1] / std::max(bv, 1e-300));
            prev_at = at0;
        }
        const int nbatch = next_batch(batch, prev_r2, prev_at, r2, at, tol2, s->max_iters) - (sweeps - at);
        prev_r2 = r2;
        prev_at = at;
        // even batches (whole 2-sweep passes), or any with the 3-sweep pass (3 + 2 + ... ; a
        // multi-rank odd batch ends with a single sweep: the same count, bit-identical values)
        batch = std::max(s->sweep3 ? nbatch : nbatch + (nbatch & 1), 2);
    }
    *its = sweeps;
    // next step's first batch: the sweeps this step's measured contraction says suffice
    // (from the first launch's residual), else the sweeps it took
    int need = sweeps;
    if (s->helm_adapt && first_r2 > 0 && last_r2 > 0 && last_r2 < first_r2 && last_at > first_at) {
        const double rate = std::log(last_r2 / first_r2) / (double)(last_at - first_at);
        const double more = std::log(tol2 / first_r2) / rate;
        if (std::isfinite(more)) need = std::min(sweeps, first_at + std::max(0, (int)std::ceil(more)));
    }
    s->helm_next = s->helm_adapt ? std::max(2, s->sweep3 ? need : need + (need & 1)) : s->helm_batch0;
    // probe again in 8 steps, or on the next step if this one needed more than one batch
    s->helm_probe = (sweeps > n0) ? 0 : (s->helm_probe + 1) % 8;
    return 0;
}

// ---------------- Poisson L phi = rhs - mean  (MatNullSpaceRemove + KSPSolve(phiSolver), FluidSolver.cpp:550-551)
// Warm start from phi^{n-1} (KSPSetInitialGuessNonzero, :54).  Expects S_SHIFT set.
int pois_solve(ns_solver* s, int* its, double* res, ns_stats* stt) {
    const double tol2 = s->rtol * s->rtol;
    int sweeps = 0, batch = s->pois_batch0, prev_at = -1;
    double prev_r2 = -1;
    double tms = 0.0;
    int tn = 0, nchk = 0;
    for (;;) {
        const int n = std::min(batch, s->max_iters - sweeps);
        if (s->timing) CHK(ensure_events(s, 2 * (size_t)n));
        int nb = 0;
        for (int k = 0; k < n; k++) {
            double* part = k == n - 1 ? s->part : nullptr;
            CHK(halo(s, {s->arr[NS_ARR_PHI]}, 2));
            if (s->timing) CHK(t_begin(s, s->ev[2 * k], s->ev[2 * k + 1]));
            nb = pois_sweep(s, part);
            if (s->timing) CHK(t_end(s, s->ev[2 * k], s->ev[2 * k + 1]));
        }
        sweeps += n;
        nsg::launch_reduce_sum(s->part, nb, 1, s->scal + S_RES, s->st);
        CHK(allreduce(s, s->scal + S_RES, 1, ncclSum));
        CHK(fetch(s));
        nchk++;
        if (s->timing) {
            for (int k = 0; k < n; k++) {
                float ms = 0.f;
                HIPCHK(hipEventElapsedTime(&ms, s->ev[2 * k], s->ev[2 * k + 1]));
                tms += ms;
            }
            tn += n;
        }
        const double r2 = s->hs[S_RES], b2 = s->hs[S_SHIFT + 1];
        *res = b2 > 0 ? std::sqrt(r2 / b2) : std::sqrt(r2);
        if (!std::isfinite(r2)) { set_err("Poisson residual is not finite"); *its = sweeps; return NS_EDIVERGE; }
        if (r2 <= tol2 * b2 || r2 == 0.0 || sweeps >= s->max_iters) break;
        const double rr = r2 / b2;
        const int nbatch = next_batch(batch, prev_r2, prev_at, rr, sweeps - 1, tol2, s->max_iters);
        prev_r2 = rr;
        prev_at = sweeps - 1;
        batch = nbatch;
    }
    *its = sweeps;
    if (stt) {
        stt->t_poisson_kernel_ms += tms;
        stt->n_poisson_kernels += tn;
        stt->n_checks += nchk;
    }
    return 0;
}

// ---------------- multigrid Poisson solve (V-cycles; smoother = the streaming RB sweep)
// the finest level's rhs shift (the null-space mean); none while preconditioning
const double* shift0(const ns_solver* s) { return s->pc_active ? nullptr : s->scal + S_SHIFT; }

MgLevel& level(ns_solver* s, int l) {
    MgLevel& L = s->lv[l];
    if (l == 0) { L.phi = s->arr[NS_ARR_PHI]; L.tmp = s->arr[NS_ARR_TMP]; L.b = s->arr[NS_ARR_RPHI]; }
    return L;
}

// ghost rows of level l (nothing to exchange on a replicated level)
int halo_l(ns_solver* s, int l, std::initializer_list<double*> fields, int w) {
    if (s->lv[l].repl) return 0;
    return halo_g(s, s->lv[l].g, fields, w);
}

// the rhs ghost rows of level l, if still owed (MgLevel::b_pend)
int flush_b(ns_solver* s, int l) {
    MgLevel& L = level(s, l);
    if (!L.b_pend) return 0;
    L.b_pend = false;
    return halo_l(s, l, {L.b}, 4);
}

// levels whose smoothing runs as two-sweep passes: the HBM-bound ones (>= 2048^2 local
// cells); the coarser ones are latency-bound and the fused pass's deeper row pipeline only
// costs there (tools/sweep_levels2.py: 512^2 9.5 us/sweep fused vs 8.1 single).  A
// distributed level always pairs (one exchange per two sweeps) when every rank's slab can
// feed the 5-row ghost exchange from ONE neighbour -- decided on the global minimum, so
// every rank makes the same choice (the exchange sizes must match).
bool pair_level(const ns_solver* s, int l) {
    const MgLevel& L = s->lv[l];
    if (s->tiled) return false;
    if (s->nranks > 1 && !L.repl) return L.minrows >= nsg::HALO;
    return (long)L.g.nxl * L.g.ny >= s->pair_min_cells;
}

// the smaller (latency-bound) levels that live whole on this rank run their fused passes as
// LDS-tiled kernels (k_tile2); NSGPU_TILE_SMALL=0 keeps single streaming sweeps + separate
// transfers there (A/B)
bool tile_level(const ns_solver* s, int l) {
    const MgLevel& L = s->lv[l];
    if (s->tiled || !s->tile_small || pair_level(s, l)) return false;
    return s->nranks == 1 || L.repl;
}

// the last two pre-smoothing sweeps of level l carry the restriction (k_sweep2<XR> /
// k_tile2<FUSE_R>); NSGPU_FUSED_RESTRICT=0 keeps the separate k_restrict pass (A/B and tests)
bool fused_restrict(const ns_solver* s, int l) {
    return s->fuse_restrict && (pair_level(s, l) || tile_level(s, l)) && s->mg_pre >= 2 && s->mg_pre % 2 == 0;
}

// the prolongation rides on the first two post-smoothing sweeps (k_sweep2 / k_tile2 FUSE_P);
// NSGPU_FUSED_PROLONG=0 keeps the separate k_prolong pass
bool fused_prolong(const ns_solver* s, int l) {
    return s->fuse_prolong && (pair_level(s, l) || tile_level(s, l)) && s->mg_post >= 2;
}

// the finest level's V-cycle boundary may run as one k_sweep4 pass: one rank (the pass reads 9 rows
// past a strip), V(2,2) with both transfers fused on a level of two-sweep passes, and the level
// below taking its iterate as zero (the pass reads that level's phi as the correction; it must not
// also store zeros into it)
bool zero_ok(const ns_solver* s, int l);
bool fuse4_level0(const ns_solver* s) {
    return s->fuse4 && !comm_on(s) && !s->pc_active && s->lv.size() > 1 && !s->lv[0].repl && pair_level(s, 0) &&
           fused_restrict(s, 0) && fused_prolong(s, 0) && s->mg_pre == 2 && s->mg_post == 2 && zero_ok(s, 1);
}

// the Poisson guess may be formed inside the solve's first level-0 restriction pass (GIN): one rank,
// the multigrid solve (no Krylov outflow / masked path), its first pass a streaming FUSE_R
bool gin_ok(const ns_solver* s) {
    return s->gin && s->in_step && !comm_on(s) && s->poisson == NS_POISSON_MG && !s->kv[0] && !s->g.fc &&
           s->lv.size() > 1 && !s->lv[0].repl && pair_level(s, 0) && fused_restrict(s, 0) && s->mg_pre == 2;
}

bool zero_ok(const ns_solver* s, int l) {
    if (l <= 0 || l >= (int)s->lv.size()) return false;
    if (l == (int)s->lv.size() - 1) return s->mg_coarse_lds || s->mg_direct;
    return fused_restrict(s, l) && s->mg_pre == 2;
}

// level l+1 as level l's restriction target / prolongation source: the first replicated
// level is seen through this rank's slab of it (rows gs.i0 .. of the whole level)
struct CoarseView {
    nsg::Geo g;
    double *b, *phi;
    bool gather;   // the distributed -> replicated transition
};
CoarseView coarse_view(ns_solver* s, int l) {
    const MgLevel& F = s->lv[l];
    MgLevel& C = s->lv[l + 1];
    if (C.repl && !F.repl) {
        const ptrdiff_t off = (ptrdiff_t)C.gs.i0 * C.g.ld;
        return CoarseView{C.gs, C.b + off, C.phi + off, true};
    }
    return CoarseView{C.g, C.b, C.phi, false};
}

// agglomeration: every rank's slab of the first replicated level's rhs to every rank, and
// that level's iterate zeroed whole (the restriction zeroed only this rank's rows).  RCCL:
// one group of point-to-point copies (slabs may differ by a row, so not ncclAllGather);
// host transport: an exact sum-allreduce of the level with every foreign row zeroed.
int gather_level(ns_solver* s, MgLevel& C) {
    const size_t ld = C.g.ld;
    // (with C.zero the level's first pass takes its iterate as zero: nothing to clear)
    if (!C.zero)
        HIPCHK(hipMemsetAsync(C.phi - (ptrdiff_t)nsg::HALO * ld, 0,
                              (size_t)(C.g.nx + 2 * nsg::HALO) * ld * sizeof(double), s->st));
    if (s->ht.allreduce) {
        if (s->npiggy) CHK(halo_reqs(s, nullptr, 0));   // (the rows riding along: an exchange of their own)
        const size_t n = (size_t)C.g.nx * ld;
        if (n > (size_t)INT32_MAX) { set_err("agglomerated level too large for the host transport"); return NS_EINVAL; }
        CHK(ensure_stage(s, n));
        HIPCHK(hipMemcpyAsync(s->stage, C.b, n * 8, hipMemcpyDeviceToHost, s->st));
        HIPCHK(hipStreamSynchronize(s->st));
        const size_t r0 = (size_t)C.gs.i0 * ld, r1 = r0 + (size_t)C.gs.nxl * ld;
        std::fill(s->stage, s->stage + r0, 0.0);
        std::fill(s->stage + r1, s->stage + n, 0.0);
        s->x_link += 8.0 * (double)C.gs.nxl * ld;   // (as the RCCL gather: this rank's slab, one link per peer)
        if (s->ht.allreduce(s->ht.user, s->stage, (int32_t)n, 0) != 0) {
            set_err("host transport allreduce failed");
            return NS_ERCCL;
        }
        HIPCHK(hipMemcpyAsync(C.b, s->stage, n * 8, hipMemcpyHostToDevice, s->st));
        return 0;
    }
    NCCLCHK(ncclGroupStart());
    if (s->npiggy) {   // the ghost rows riding along (ns_solver::piggy) join the gather's group
        HaloReq r[4];
        for (int k = 0; k < s->npiggy; k++) r[k] = HaloReq{s->piggy[k].g, s->piggy[k].f, s->piggy[k].w};
        const int n = s->npiggy;
        s->npiggy = 0;
        CHK(halo_rccl(s, r, n, s->st));
    }
    for (int q = 0; q < s->nranks; q++) {
        if (q == s->rank) continue;
        if (s->loopback) {   // virtual slab: the same messages, every peer this process
            const size_t cnt = (size_t)std::min(C.sn[q], C.gs.nxl) * ld;
            NCCLCHK(ncclSend(C.b + (ptrdiff_t)C.gs.i0 * ld, cnt, ncclDouble, 0, s->comm, s->st));
            if (q == (s->rank == 0 ? 1 : 0)) s->x_link += 8.0 * (double)C.gs.nxl * ld;
            NCCLCHK(ncclRecv(C.b + (ptrdiff_t)C.si0[q] * ld, cnt, ncclDouble, 0, s->comm, s->st));
            continue;
        }
        NCCLCHK(ncclSend(C.b + (ptrdiff_t)C.gs.i0 * ld, (size_t)C.gs.nxl * ld, ncclDouble, q, s->comm, s->st));
        if (q == (s->rank == 0 ? 1 : 0)) s->x_link += 8.0 * (double)C.gs.nxl * ld;   // (one link per peer)
        NCCLCHK(ncclRecv(C.b + (ptrdiff_t)C.si0[q] * ld, (size_t)C.sn[q] * ld, ncclDouble, q, s->comm, s->st));
    }
    NCCLCHK(ncclGroupEnd());
    return 0;
}

// level l's implicit zero iterate as stored zeros (a consumer that reads phi)
int zero_phi(ns_solver* s, int l) {
    MgLevel& L = level(s, l);
    if (!L.zero) return 0;
    L.zero = false;
    const size_t ld = L.g.ld;
    HIPCHK(hipMemsetAsync(L.phi - (ptrdiff_t)nsg::HALO * ld, 0, (size_t)(L.g.nxl + 2 * nsg::HALO) * ld * sizeof(double),
                          s->st));
    return 0;
}

// the first consumer of level l's phi in a V-cycle takes an implicit zero (MgLevel::zero): the
// fused restriction pass when it is the level's first pre-smoothing pass, or the LDS coarse solve
bool zero_ok(const ns_solver* s, int l);

int mg_smooth(ns_solver* s, int l, int n, int* tn, int ev0) {
    MgLevel& L = level(s, l);
    if (n > 0) CHK(flush_b(s, l));
    if (n > 0) CHK(zero_phi(s, l));
    for (int k = 0; k < n;) {
        const int w = (n - k >= 2 && pair_level(s, l)) ? 2 : 1;   // two sweeps per HBM pass
        CHK(halo_l(s, l, {L.phi}, 2 * w));
        const bool t = s->timing && l == 0 && (!s->pc_active || s->pc_timing);
        if (t) { CHK(t_begin(s, s->ev[2 * (ev0 + *tn)], s->ev[2 * (ev0 + *tn) + 1])); s->evtag[ev0 + *tn] = 0; }
        const double* sh = l == 0 ? shift0(s) : nullptr;
        if (w == 2) nsg::launch_pois_rbsor2(L.g, L.c, s->mg_omega_s, L.phi, L.tmp, L.b, sh, nullptr, s->st);
        else nsg::launch_pois_rbsor(L.g, L.c, s->mg_omega_s, L.phi, L.tmp, L.b, sh, nullptr, s->st);
        if (t) { CHK(t_end(s, s->ev[2 * (ev0 + *tn)], s->ev[2 * (ev0 + *tn) + 1])); (*tn)++; }
        std::swap(L.phi, L.tmp);
        if (l == 0) { s->arr[NS_ARR_PHI] = L.phi; s->arr[NS_ARR_TMP] = L.tmp; }
        k += w;
    }
    return 0;
}

int mg_coarse(ns_solver* s) {
    const int l = (int)s->lv.size() - 1;
    MgLevel& L = level(s, l);
    CHK(flush_b(s, l));
    if (s->mg_direct) {
        // Y = E o (Vx^-1 b Vy^-T) into the level's spare plane, phi = Vx Y Vy^T (phi is not read:
        // the implicit zero iterate needs nothing)
        L.zero = false;
        const int nx = L.g.nx, ny = L.g.ny, ld = L.g.ld;
        if (nsg::launch_direct(s->dP1, L.b, s->dQ1, s->dE, L.tmp, nx, ny, ld, ld, s->st) != 0 ||
            nsg::launch_direct(s->dP2, L.tmp, s->dQ2, nullptr, L.phi, nx, ny, ld, ld, s->st) != 0) {
            set_err("coarse direct solve does not fit");
            return NS_EINVAL;
        }
        return 0;
    }
    if (s->mg_coarse_lds) {
        const int zin = L.zero ? 1 : 0;
        L.zero = false;
        if (nsg::launch_coarse_vcycle(L.g, s->cvimg, s->cv_n, s->cv_dn, L.phi, L.b, 1, s->mg_pre, s->mg_post,
                                      s->mg_coarse_iters, s->mg_omega_c, s->mg_omega_s, s->out_side == 0,
                                      s->out_side == 1, s->st, zin) != 0) {
            set_err("coarse LDS V-cycle does not fit");
            return NS_EINVAL;
        }
        return 0;
    }
    CHK(zero_phi(s, l));
    for (int k = 0; k < s->mg_coarse_iters; k++) {
        CHK(halo_l(s, l, {L.phi}, 2));
        nsg::launch_pois_rbsor(L.g, L.c, s->mg_omega_c, L.phi, L.tmp, L.b, nullptr, nullptr, s->st);
        std::swap(L.phi, L.tmp);
    }
    return 0;
}

// one V-cycle (pre-smoothing + restriction down to the coarsest level, the coarse solve,
// prolongation + post-smoothing back up).  With `want_check`, `check(nb)` runs after the
// finest level's last post-smoothing pass (r^2 partials of the cycle's output residual in
// s->part, nb of them: the fused prolongation pass computes them in the same HBM pass) and
// returns 1 to end the solve there, 0 to go on, < 0 on error; the preconditioner asks for none.
// (Round 1-2 checked after the NEXT cycle's fused restriction pass, so a converged solve paid
// one restriction pass it then discarded; two more RB sweeps shrink a cycle's output residual
// only ~1.2x -- the post-smoothed residual is smooth -- so the counts stay the same.)
template <class Check>
int mg_vcycle(ns_solver* s, int* tn, int ev0, Check&& check, bool want_check, bool* done) {
    const int nl = (int)s->lv.size();
    *done = false;
    for (int l = 0; l < nl - 1; l++) {
        MgLevel& F = level(s, l);
        MgLevel& C = level(s, l + 1);
        const CoarseView cv = coarse_view(s, l);
        const double* sh = l == 0 ? shift0(s) : nullptr;
        int nb;
        // the coarse level's first pass takes its iterate as zero: the restriction stores no zeros
        const bool czero = zero_ok(s, l + 1);
        double* pcz = czero ? nullptr : cv.phi;
        if (l == 0 && s->gin_pending) {
            // the solve's first restriction pass with its input, the phi extrapolation, formed per
            // row from the history planes (k_sweep2_gin); it writes PHI (extrapolate_phi left the
            // output plane there and TMP free), so no swap
            s->gin_pending = false;
            const bool t = s->timing && (!s->pc_active || s->pc_timing);
            if (t) { CHK(t_begin(s, s->ev[2 * (ev0 + *tn)], s->ev[2 * (ev0 + *tn) + 1])); s->evtag[ev0 + *tn] = 3; }
            nb = nsg::launch_pois_rbsor2_restrict_guess(F.g, F.c, s->mg_omega_s, s->gin_src[0], F.phi, F.b, sh, cv.g,
                                                        cv.b, pcz, s->part, s->gin_src[1], s->gin_src[2],
                                                        s->gin_src[3], s->gin_c, s->st);
            if (nb < 0) { set_err("guess restriction pass does not fit"); return NS_EINVAL; }
            if (t) { CHK(t_end(s, s->ev[2 * (ev0 + *tn)], s->ev[2 * (ev0 + *tn) + 1])); (*tn)++; }
        } else if (l == 0 && s->p_pending) {
            // the previous cycle's prolongation pass (deferred: its output was not checked) and this
            // cycle's restriction pass in one (k_sweep4); level 1's phi still holds that correction
            s->p_pending = false;
            const bool t = s->timing && (!s->pc_active || s->pc_timing);
            if (t) { CHK(t_begin(s, s->ev[2 * (ev0 + *tn)], s->ev[2 * (ev0 + *tn) + 1])); s->evtag[ev0 + *tn] = 2; }
            nb = nsg::launch_pois_sweep4(F.g, F.c, s->mg_omega_s, F.phi, F.tmp, F.b, sh, cv.g, cv.phi, cv.b, nullptr,
                                         s->part, s->st);
            if (nb < 0) { set_err("V-cycle boundary pass does not fit"); return NS_EINVAL; }
            if (t) { CHK(t_end(s, s->ev[2 * (ev0 + *tn)], s->ev[2 * (ev0 + *tn) + 1])); (*tn)++; }
            std::swap(F.phi, F.tmp);
            s->arr[NS_ARR_PHI] = F.phi; s->arr[NS_ARR_TMP] = F.tmp;
        } else if (fused_restrict(s, l)) {
            // last two pre-smoothing sweeps + residual + restriction in one HBM pass
            CHK(mg_smooth(s, l, s->mg_pre - 2, tn, ev0));
            const bool zin = F.zero;   // (then the pass reads neither phi nor its ghost rows)
            F.zero = false;
            const bool t = s->timing && l == 0 && (!s->pc_active || s->pc_timing);
            if (t) { CHK(t_begin(s, s->ev[2 * (ev0 + *tn)], s->ev[2 * (ev0 + *tn) + 1])); s->evtag[ev0 + *tn] = 1; }
            if (tile_level(s, l)) {
                CHK(flush_b(s, l));
                if (!zin) CHK(halo_l(s, l, {F.phi}, 5));
                nb = nsg::launch_pois_tile2_restrict(F.g, F.c, s->mg_omega_s, F.phi, F.tmp, F.b, sh, cv.g, cv.b, pcz,
                                                     s->part, s->st, zin);
            } else if (F.repl) {
                nb = nsg::launch_pois_rbsor2_restrict(F.g, F.c, s->mg_omega_s, F.phi, F.tmp, F.b, sh, cv.g, cv.b,
                                                      pcz, s->part, s->st, zin);
            } else {
                // (the level's rhs ghost rows ride along when owed; a zero iterate has none to send)
                const HaloReq r[2] = {{&F.g, F.phi, 5}, {&F.g, F.b, 4}};
                const HaloReq* rq = zin ? r + 1 : r;
                const int nr = zin ? (F.b_pend ? 1 : 0) : (F.b_pend ? 2 : 1);
                F.b_pend = false;
                auto pass = [&]() {
                    return nsg::launch_pois_rbsor2_restrict(F.g, F.c, s->mg_omega_s, F.phi, F.tmp, F.b, sh, cv.g,
                                                            cv.b, pcz, s->part, s->st, zin);
                };
                nb = nr ? overlapped(s, rq, nr, pass) : pass();
                if (nb < 0) return nb;
                // the pass's output is this level's iterate until its prolongation pass: its ghost
                // rows ride on the next exchange group down the V-cycle (piggy), so that pass needs
                // no exchange of its own for them
                if (comm_on(s) && fused_prolong(s, l) && s->npiggy < 4) {
                    s->piggy[s->npiggy++] = ns_solver::Piggy{&F.g, F.tmp, 5};   // (F.tmp: the output, swapped below)
                    F.phi_ghost = true;
                }
            }
            if (t) { CHK(t_end(s, s->ev[2 * (ev0 + *tn)], s->ev[2 * (ev0 + *tn) + 1])); (*tn)++; }
            std::swap(F.phi, F.tmp);
            if (l == 0) { s->arr[NS_ARR_PHI] = F.phi; s->arr[NS_ARR_TMP] = F.tmp; }
        } else {
            CHK(zero_phi(s, l));
            CHK(mg_smooth(s, l, s->mg_pre, tn, ev0));
            CHK(flush_b(s, l));
            CHK(halo_l(s, l, {F.phi}, 1));
            nb = nsg::launch_restrict(F.g, F.c, F.phi, F.b, sh, cv.g, C.c, cv.b, cv.phi, s->part, s->st);
        }
        (void)nb;   // (the restriction's partials: the pre-smoothed residual, unused)
        // (k_restrict always stores the zeros; the fused passes skip them when the coarse level takes
        // them implicitly)
        C.zero = czero && fused_restrict(s, l);
        if (cv.gather) CHK(gather_level(s, C));
        else if (s->nranks > 1 && s->overlap && s->cst && !C.repl && fused_restrict(s, l + 1) && !tile_level(s, l + 1))
            C.b_pend = true;   // sent with level l+1's FUSE_R exchange
        else CHK(halo_l(s, l + 1, {C.b}, 4));
    }
    CHK(mg_coarse(s));
    int nb_out = -1;   // partials of the finest level's output residual (-1: none yet)
    for (int l = nl - 2; l >= 0; l--) {
        MgLevel& F = level(s, l);
        MgLevel& C = level(s, l + 1);
        const CoarseView cv = coarse_view(s, l);
        if (l == 0 && !want_check && fuse4_level0(s)) {
            // (this cycle's output is not checked, so another cycle follows: the prolongation pass
            // runs fused with its restriction pass, k_sweep4)
            s->p_pending = true;
        } else if (fused_prolong(s, l)) {
            // prolongation + the first two post-smoothing sweeps in one HBM pass; the coarse
            // and fine ghost rows travel in one group
            const bool t = s->timing && l == 0 && (!s->pc_active || s->pc_timing);
            const double* shp = l == 0 ? shift0(s) : nullptr;
            // the finest level's last pass also sums its output residual (the convergence check)
            double* pp = (l == 0 && want_check && s->mg_post == 2) ? s->part : nullptr;
            auto pass = [&]() {
                return (tile_level(s, l) ? nsg::launch_pois_tile2_prolong : nsg::launch_pois_rbsor2_prolong)(
                    F.g, F.c, s->mg_omega_s, F.phi, F.tmp, F.b, shp, cv.g, cv.phi, pp, s->st);
            };
            if (t) { CHK(t_begin(s, s->ev[2 * (ev0 + *tn)], s->ev[2 * (ev0 + *tn) + 1])); s->evtag[ev0 + *tn] = 0; }
            int n;
            if (F.repl) {
                n = pass();
            } else if (tile_level(s, l)) {
                if (cv.gather || C.repl) CHK(halo_l(s, l, {F.phi}, 5));
                else CHK(halo_reqs(s, {HaloReq{&C.g, C.phi, 3}, HaloReq{&F.g, F.phi, 5}}));
                n = pass();
            } else {
                // (the coarse ghost rows are read by the edge strips only; the fine ones were sent
                // after the restriction pass when phi_ghost -- or still ride on this group)
                const bool cx = !(cv.gather || C.repl);
                const HaloReq r[2] = {{&F.g, F.phi, 5}, {&C.g, C.phi, 3}};
                const HaloReq* rq = F.phi_ghost ? r + 1 : r;
                const int nr = F.phi_ghost ? (cx ? 1 : 0) : (cx ? 2 : 1);
                F.phi_ghost = false;
                if (nr == 0 && s->npiggy) CHK(halo_reqs(s, nullptr, 0));   // (rows still riding: send them now)
                n = nr ? overlapped(s, rq, nr, pass) : pass();
                if (n < 0) return n;
            }
            if (pp) nb_out = n;
            if (t) { CHK(t_end(s, s->ev[2 * (ev0 + *tn)], s->ev[2 * (ev0 + *tn) + 1])); (*tn)++; }
            std::swap(F.phi, F.tmp);
            if (l == 0) { s->arr[NS_ARR_PHI] = F.phi; s->arr[NS_ARR_TMP] = F.tmp; }
            CHK(mg_smooth(s, l, s->mg_post - 2, tn, ev0));
        } else {
            if (!cv.gather) CHK(halo_l(s, l + 1, {C.phi}, 1));
            nsg::launch_prolong(F.g, F.phi, cv.g, cv.phi, s->st);
            CHK(mg_smooth(s, l, s->mg_post, tn, ev0));
        }
    }
    if (want_check && nl > 1) {
        if (nb_out < 0) {
            // (unfused or longer post-smoothing: the residual by a restriction pass of its own,
            // whose coarse output the next cycle's restriction overwrites)
            MgLevel& F = level(s, 0);
            const CoarseView cv = coarse_view(s, 0);
            CHK(halo_l(s, 0, {F.phi}, 1));
            nb_out = nsg::launch_restrict(F.g, F.c, F.phi, F.b, shift0(s), cv.g, level(s, 1).c, cv.b, cv.phi,
                                          s->part, s->st);
        }
        const int rc = check(nb_out);
        if (rc < 0) return rc;
        if (rc > 0) *done = true;
    }
    return 0;
}

int pois_solve_mg(ns_solver* s, int* its, double* res, ns_stats* stt) {
    s->p_pending = false;
    const double tol2 = s->rtol * s->rtol;
    const int maxc = std::min(s->max_iters, 1000);
    int cyc = 0, tn = 0, nchk = 0;   // cyc: V-cycles done before the current one
    double tms = 0.0;
    const int per_cycle = s->mg_pre + s->mg_post;
    // residual checks (host syncs): after cycle 0, then where the contraction rate (measured
    // between this solve's checks, else the previous solve's) predicts convergence -- the
    // cycles in between run without a host round trip
    // the first check: at the fewest V-cycles any of the last four solves converged at (consecutive
    // steps converge alike, so the check after cycle 0 would only measure a rate already known;
    // a solve converging earlier than all four costs at most that many partial cycles)
    int next_chk = 0, prev_c = -1;
    if (s->mg_predict && s->mg_rate2 > 0) {
        int m = 1 << 30;
        for (int h : s->mg_hist) m = std::min(m, h);
        if (m > 0) next_chk = m;
    }
    double prev_rr = -1.0;
    if (s->rp_c >= 0) next_chk = s->rp_c;   // virtual slab: the replayed cycle count, one check
    // speculate at the first check when the last four solves all converged by then
    const bool spec_ok = s->speculate && s->in_step && !s->defer_now && s->mg_predict && s->rp_c < 0 && next_chk > 0;
    auto check = [&](int nb) -> int {
        const int cycles = cyc + 1;   // complete cycles (this check ends one)
        if (!(cycles >= next_chk || cycles >= maxc)) return 0;
        // the cycle's output residual: the convergence test (a host sync)
        nsg::launch_reduce_sum(s->part, nb, 1, s->scal + S_RES, s->st);
        CHK(allreduce(s, s->scal + S_RES, 1, ncclSum));
        const bool spec = spec_ok && nchk == 0;
        if (spec) {
            s->cur_cycles = cycles;   // (the guess K5 forms: this solve's count if the check passes)
            CHK(fetch_begin(s));   // (the residual's copy, then K5 behind it)
            CHK(correct_launch(s, s->part + 4 * (size_t)nsg::max_partials(s->g)));
            s->n_spec++;
            CHK(fetch_end(s));
        } else {
            CHK(fetch(s));
        }
        nchk++;
        if (s->timing) {
            for (int k = 0; k < tn; k++) {
                float ms = 0.f;
                HIPCHK(hipEventElapsedTime(&ms, s->ev[2 * k], s->ev[2 * k + 1]));
                if (s->evtag[k] == 2) {
                    if (stt) { stt->t_cycle_kernel_ms += ms; stt->n_cycle_kernels++; }
                } else if (s->evtag[k] == 3) {
                    if (stt) { stt->t_guess_kernel_ms += ms; stt->n_guess_kernels++; }
                } else if (s->evtag[k]) {
                    if (stt) { stt->t_restrict_kernel_ms += ms; stt->n_restrict_kernels++; }
                } else {
                    tms += ms;
                    if (stt) stt->n_poisson_kernels++;
                }
            }
            tn = 0;
        }
        const double r2 = s->hs[S_RES], b2 = s->hs[S_SHIFT + 1];
        *res = b2 > 0 ? std::sqrt(r2 / b2) : std::sqrt(r2);
        if (s->verbose) fprintf(stderr, "nsgpu poisson: after %d V-cycles rel. residual %.3e\n", cycles, *res);
        if (!std::isfinite(r2)) { set_err("Poisson residual is not finite"); *its = cycles; return NS_EDIVERGE; }
        if (r2 <= tol2 * b2 || r2 == 0.0 || cycles >= maxc || s->rp_c >= 0) {
            if (spec) { s->k5_spec = 1; s->n_spec_hit++; }
            return 1;
        }
        if (s->mg_predict) {
            const double rr = r2 / b2;
            double rate = s->mg_rate2;   // per-cycle contraction of r^2
            if (prev_rr > 0 && rr < prev_rr && cycles > prev_c)
                rate = std::pow(rr / prev_rr, 1.0 / (cycles - prev_c));
            int need = 1;
            if (rate > 0 && rate < 0.5) {
                s->mg_rate2 = rate;
                // one check BEFORE the predicted converged cycle: a slower-than-predicted
                // contraction then costs a check, never a wasted V-cycle
                need = (int)std::ceil(std::log(tol2 / rr) / std::log(rate)) - 1;
                need = std::min(std::max(need, 1), 8);
            }
            prev_rr = rr;
            prev_c = cycles;
            next_chk = cycles + need;
        } else {
            next_chk = cycles + 1;
        }
        return 0;
    };
    for (;;) {
        if (s->timing) CHK(ensure_events(s, 2 * (size_t)(tn + per_cycle + 2)));
        bool done = false;
        // (the output residual only on the cycles the check reads: the pass without it keeps 3
        // rows in flight, 97.5 vs 101 us at 4096^2)
        CHK(mg_vcycle(s, &tn, 0, check, cyc + 1 >= next_chk || cyc + 1 >= maxc, &done));
        cyc++;
        if (done) break;
    }
    const int cycles = cyc;
    *its = cycles;
    // history: the cycle count this solve needed -- one fewer when its only check came with a
    // full cycle's contraction to spare (the earlier check point would have passed too)
    int need = cycles;
    if (nchk == 1 && cycles > 0 && s->mg_rate2 > 0) {
        const double rr = s->hs[S_RES] / std::max(s->hs[S_SHIFT + 1], 1e-300);
        if (rr / s->mg_rate2 <= tol2) need = cycles - 1;
    }
    for (int k = 3; k > 0; k--) s->mg_hist[k] = s->mg_hist[k - 1];
    s->mg_hist[0] = need;
    s->last_cycles = s->cur_cycles = cycles;
    s->gin_pending = false;
    if (stt) {
        stt->t_poisson_kernel_ms += tms;
        stt->n_checks += nchk;
    }
    return 0;
}

// ---------------- NEUMANN outflow: BiCGStab on the reference's Poisson matrix
// With an outflow side the matrix (ConstructLHS + AddGhostStencils, FluidSolver.cpp:105-163)
// has rows the red-black smoothers cannot relax (2.5/-2/0.5 ghost, :98-101: not diagonally
// dominant, and coupling a cell to a same-colour cell two rows inward).  The solve is then
// the reference's own method class -- BiCGStab (KSPBCGSL, :73-82) -- on the true matrix,
// right-preconditioned by ONE V-cycle of the wall-closure multigrid (the smoothers' operator:
// outflow faces treated like walls).  The singular system (constant null space, :142-144) is
// solved as P A x = P (b - mean b) with P the mean projection: every residual is kept
// mean-free, as MatNullSpaceRemove does to the reference's Krylov vectors.  All recurrence
// scalars live on the device (k_bicg_scal); one host sync per iteration reads ||r||^2.

// z = M^-1 q: one V-cycle of the preconditioner's multigrid with level-0 rhs q (no mean
// shift), from z = 0 (wall closure) or from the outflow line solve's extension (line closure).  Level 0 is re-pointed at (z, scratch, q) and restored afterwards; the cycle's
// ping-pong may leave the result in either buffer, so z / scratch are swapped to match.
int mg_precond(ns_solver* s, double* q, double*& z, double*& scratch, int* tn = nullptr) {
    double* sv[3] = {s->arr[NS_ARR_PHI], s->arr[NS_ARR_TMP], s->arr[NS_ARR_RPHI]};
    if (s->out_side >= 0) {
        // the outflow side's data: its 1-D line solve (on the side's slab; summed over ranks so
        // every slab has it), extended constantly along x as the cycle's initial iterate, and
        // into the other ping-pong plane's ghost row beyond the side.  The cycle then works on
        // the residual q - D z0, which is O(q), instead of on the O(ny^2 q) Dirichlet data
        const bool mine = s->out_side == 0 ? s->g.i0 == 0 : s->g.i0 + s->g.nxl == s->g.nx;
        const ptrdiff_t ld = s->g.ld;
        const ptrdiff_t row = s->out_side == 0 ? 0 : s->g.nxl - 1, ghost = s->out_side == 0 ? -1 : s->g.nxl;
        if (mine) {
            if (nsg::launch_line_solve(q + row * ld, s->c, s->g.ny, s->lrow, s->st) != 0) {
                set_err("outflow line solve: ny = %d exceeds its LDS capacity", s->g.ny);
                return NS_EINVAL;
            }
        } else {
            HIPCHK(hipMemsetAsync(s->lrow, 0, (size_t)s->g.ny * sizeof(double), s->st));
        }
        CHK(allreduce(s, s->lrow, s->g.ny, ncclSum));
        nsg::launch_line_extend(s->lrow, s->g, z - (ptrdiff_t)nsg::HALO * ld, s->g.nxl + 2 * nsg::HALO,
                                mine ? scratch + ghost * ld : nullptr, s->st);
    } else {
        HIPCHK(hipMemsetAsync(z - (ptrdiff_t)s->hp * s->g.ld, 0, s->plane * sizeof(double), s->st));
    }
    CHK(halo(s, {q}, 5));
    s->arr[NS_ARR_PHI] = z;
    s->arr[NS_ARR_TMP] = scratch;
    s->arr[NS_ARR_RPHI] = q;
    s->pc_active = true;
    s->pc_timing = tn != nullptr;
    int tn0 = 0;
    if (tn) CHK(ensure_events(s, 2 * ((size_t)*tn + 2 * (s->mg_pre + s->mg_post) + 4)));
    bool done = false;
    const int rc = mg_vcycle(s, tn ? tn : &tn0, 0, [](int) { return 0; }, false, &done);
    s->pc_active = false;
    s->pc_timing = false;
    // (level 0's own pointer: a single-level hierarchy relaxes it in mg_coarse, which does not
    // track the swaps in s->arr)
    if (s->lv[0].phi != z) std::swap(z, scratch);
    s->arr[NS_ARR_PHI] = sv[0];
    s->arr[NS_ARR_TMP] = sv[1];
    s->arr[NS_ARR_RPHI] = sv[2];
    return rc;
}

// (r4) z = M^-1 q for a masked domain on one rank whose bounding box admits the direct solve: the
// box's exact Poisson solve (ns_fps.hip: DCT, recurrences, inverse DCT; F in `scratch`) in place of
// one V-cycle of its multigrid -- the same fictitious-domain preconditioner, solved exactly.  q is
// mean-free over the domain and 0 outside it, so the box's mode 0 is consistent: k_bicg_vec keeps every
// Krylov vector 0 outside the domain (it skips those cells; the kv planes are zeroed at ns_create) and
// applies the mean projection P to r, v and t (KV_INIT / KV_V / KV_T), so p and s -- the vectors handed
// here -- inherit both properties
int fps_scan(ns_solver* s, bool backward);
int fps_precond(ns_solver* s, const double* q, double* z, double* scratch, const int32_t* omask = nullptr) {
    const nsg::Geo& g = s->g;
    // ((r5) a masked domain whose box has the E outflow: its row pair transformed eliminated, as the channel's)
    if (nsg::launch_fps_dct(false, q, nullptr, scratch, g.nxl, g.ny, g.ld, s->fps_tw, s->fps_wk, s->st,
                            s->fa.outE ? g.nxl / 2 - 1 : -1) < 0) {
        set_err("direct Poisson preconditioner: ny = %d is not a supported power of two", g.ny);
        return NS_EINVAL;
    }
    nsg::launch_fps_t1b(s->fa, scratch, s->st);
    CHK(fps_scan(s, false));
    nsg::launch_fps_mid(s->fa, scratch, s->st);
    CHK(fps_scan(s, true));
    nsg::launch_fps_t2b(s->fa, scratch, s->st);
    if (omask) {   // (r6: z's masked-domain cells only)
        if (nsg::launch_fps_idct_masked(scratch, z, g.nxl, g.ny, g.ld, s->fps_tw, s->fps_wk, s->st, omask) < 0) {
            set_err("direct Poisson preconditioner: no masked inverse transform for ny = %d", g.ny);
            return NS_EINVAL;
        }
        return 0;
    }
    nsg::launch_fps_dct(true, scratch, nullptr, z, g.nxl, g.ny, g.ld, s->fps_tw, s->fps_wk, s->st);
    return 0;
}

// (r5) z = L_ext^+ q on a masked domain by its capacitance matrix (nsg::CapArgs): two box solves around the
// interface's dense m x m solve -- z1 = L_box^+ q, y = (C + 1 1^T / m)^-1 D^T z1, z = L_box^+ (q - D_w y).  q is mean-
// free over the domain and 0 outside it (the residual k_bicg_vec's KV_INIT leaves); it is modified at the
// interface cells and restored to 0 outside (its domain values are rewritten by the next KV_INIT)
// (r6) xout: the second box solve writes the solution's domain cells straight into xout (its other cells kept) --
// the x = z pass of a solve from zero (k_cap_axpy, 57 us at 4096^2) not needed
int cap_solve(ns_solver* s, double* q, double* z, double* xout = nullptr) {
    CHK(fps_precond(s, q, z, s->kv[8]));
    if (nsg::launch_cap_gemv(s->cap, z, s->st) != hipSuccess) {
        set_err("capacitance solve: k_cap_gemv launch failed (%d interface faces)", s->cap.m + s->cap.border);
        return NS_EHIP;
    }
    nsg::launch_cap_scatter(s->cap, q, 0, s->st);
    if (xout) CHK(fps_precond(s, q, xout, s->kv[8], s->g.fc));
    else CHK(fps_precond(s, q, z, s->kv[8]));
    nsg::launch_cap_scatter(s->cap, q, 1, s->st);
    return 0;
}

// (r5) the capacitance matrix of a masked domain on one rank whose bounding box has the direct solve: the m
// faces between a domain cell and a box cell outside it, then C's columns by m box solves of the faces'
// dipoles w_f d_f (C[g][f] = delta_gf + (D^T L_box^+ w_f d_f)_g, + 1 / m: the regularisation along the domain's
// constant y0 = 1, C y0 = 0) and its inverse by Gauss-Jordan, all on the device.  Not built (BiCGStab with the box
// preconditioner stays): m = 0 or > NSGPU_CAP_MAX (4096; clamped to the gemv's LDS bound, nsg::CAP_LDS_MAX - 1),
// NSGPU_CAP=0, a Gauss-Jordan pivot that is not finite, below 1e-12 in magnitude, or (no border) not positive
int cap_setup(ns_solver* s, const ns_grid_desc* gd, const double* pw, const double* pe, const double* ps,
              const double* pn) {
    const char* ce = getenv("NSGPU_CAP");
    if (ce && std::atoi(ce) == 0) return 0;
    const char* cm = getenv("NSGPU_CAP_MAX");
    const long mmax = std::min(cm ? std::atol(cm) : 4096L, (long)nsg::CAP_LDS_MAX - 1);   // (+ the border row)
    const nsg::Geo& g = s->g;
    const int nx = gd->nx, ny = gd->ny;
    auto inside = [&](int i, int j) { return gd->cell_id[(size_t)i * ny + j] >= 0; };
    std::vector<int> fi, fj;
    std::vector<double> w;
    std::map<int, std::vector<int>> refs;   // plane offset -> signed face references
    const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < ny; j++) {
            if (!inside(i, j)) continue;
            for (int k = 0; k < 4; k++) {
                const int a = i + di[k], b = j + dj[k];
                if (a < 0 || a >= nx || b < 0 || b >= ny || inside(a, b)) continue;
                const int f = (int)fi.size();
                if ((long)f >= mmax) return 0;
                const int oi = (i - g.i0) * g.ld + j, oj = (a - g.i0) * g.ld + b;
                fi.push_back(oi);
                fj.push_back(oj);
                // (the coefficient of this face in the domain cell's row; the same in the outside cell's row on the
                // uniform grids the box's direct solve admits)
                w.push_back(k == 0 ? pw[i] : k == 1 ? pe[i] : k == 2 ? ps[j] : pn[j]);
                refs[oi].push_back(f + 1);
                refs[oj].push_back(-(f + 1));
            }
        }
    const int m = (int)fi.size();
    if (m == 0) return 0;
    std::vector<int> co;
    std::vector<int> cf;
    for (const auto& kv : refs) {
        if (kv.second.size() > 4) return 0;   // (a cell has 4 faces)
        co.push_back(kv.first);
        for (int k = 0; k < 4; k++) cf.push_back(k < (int)kv.second.size() ? kv.second[k] : 0);
    }
    const int nc = (int)co.size();
    // (an E outflow: the bordered system, M = m + 1, and the plane e1 = L_box^+ 1_domain)
    const int border = s->fa.outE ? 1 : 0, M = m + border;
    const size_t ne1 = border ? s->plane : 0;
    // device: cinv (M^2), y, t, u (M each), w (m), flag, e1 (doubles); fi, fj, co, cf (ints)
    // (nd even and the int4 table at a multiple of 4 ints: 16-byte aligned)
    const size_t nd = ((size_t)M * M + 4 * (size_t)M + ne1 + 9) & ~(size_t)1, o4 = (2 * (size_t)m + nc + 3) & ~(size_t)3;
    const size_t ni = o4 + 4 * (size_t)nc;
    HIPCHK(hipMalloc(&s->cap_mem, nd * sizeof(double) + ni * sizeof(int)));
    double* dm = (double*)s->cap_mem;
    double *cinv = dm, *y = cinv + (size_t)M * M, *wd = y + M, *t = wd + M, *u = t + M, *flag = u + M;
    double* e1 = border ? flag + 8 + (size_t)s->hp * g.ld : nullptr;
    int* im = (int*)(dm + nd);
    int *dfi = im, *dfj = dfi + m, *dco = dfj + m;
    int* dcf = im + o4;
    HIPCHK(hipMemcpy(wd, w.data(), m * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemset(flag, 0, sizeof(double)));
    HIPCHK(hipMemcpy(dfi, fi.data(), m * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dfj, fj.data(), m * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dco, co.data(), nc * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dcf, cf.data(), 4 * (size_t)nc * sizeof(int), hipMemcpyHostToDevice));
    nsg::CapArgs& a = s->cap;
    a.m = m; a.ncell = nc; a.border = border; a.e1 = e1;
    a.fi = dfi; a.fj = dfj; a.co = dco; a.cf = (const int4*)dcf; a.w = wd;
    a.cinv = cinv; a.y = y;
    // C by columns: the dipole in the (zeroed) plane kv[0], its box solve into kv[6]
    HIPCHK(hipStreamSynchronize(s->st));   // (the Krylov planes' memset)
    for (int f = 0; f < m; f++) {
        nsg::launch_cap_src(a, s->kv[0], f - 1, f, s->st);
        CHK(fps_precond(s, s->kv[0], s->kv[6], s->kv[8]));
        nsg::launch_cap_col(a, s->kv[6], f, cinv, s->st);
    }
    nsg::launch_cap_src(a, s->kv[0], m - 1, -1, s->st);
    if (border) {   // the border column from e1 = L_box^+ 1_domain (kv[0] zeroed again after)
        nsg::launch_cap_fill(g, s->kv[0], 1.0, s->st);
        CHK(fps_precond(s, s->kv[0], e1, s->kv[8]));
        nsg::launch_cap_fill(g, s->kv[0], 0.0, s->st);
        nsg::launch_cap_col(a, e1, m, cinv, s->st);
    }
    nsg::launch_gj_invert(cinv, M, t, u, flag, border ? 0 : 1, s->st);
    double fl = 0.0;
    HIPCHK(hipMemcpyAsync(&fl, flag, sizeof(double), hipMemcpyDeviceToHost, s->st));
    HIPCHK(hipStreamSynchronize(s->st));
    if (fl != 0.0) {   // (never seen: the preconditioned BiCGStab instead)
        if (s->verbose)
            fprintf(stderr, "nsgpu: capacitance matrix (%d faces): a Gauss-Jordan pivot failed the test of k_gj_prep "
                            "(not finite, tiny%s): BiCGStab\n", m, border ? "" : " or not positive");
        s->cap = nsg::CapArgs{};
        (void)hipFree(s->cap_mem);
        s->cap_mem = nullptr;
        return 0;
    }
    if (s->verbose)
        fprintf(stderr, "nsgpu: masked Poisson by the capacitance matrix: %d interface faces, %d cells%s\n", m, nc,
                border ? ", bordered (E outflow)" : "");
    return 0;
}

// One BiCGStab solve A x = b - shift on this solver's planes (x updated in place).
//   op 0: the Poisson matrix (NEUMANN outflow rows / a masked domain), solved as
//         P A x = P (b - shift) with P the mean projection over the domain's cells;
//   op 1: the Helmholtz matrix I - alpha L_V of a masked domain (regular: no projection).
// Preconditioner: one wall-closure multigrid V-cycle (mg) or diag(A)^-1 (masked domains,
// whose operators the rectangle hierarchy does not represent).  b2 = ||b - shift||^2 (host)
// for the relative test; `name` labels the verbose history.
int bicgstab(ns_solver* s, const KrylovSolve& ks, int* its, double* res) {
    const double tol2 = s->rtol * s->rtol;
    const int maxit = std::min(s->max_iters, ks.mg ? 5000 : 100000);
    double** K = s->kv;   // r, r0, p, v, s, t, ph, sh, scratch
    nsg::KrylovArgs a{};
    a.g = s->g;
    a.x = ks.x;
    a.r = K[0]; a.r0 = K[1]; a.p = K[2]; a.v = K[3]; a.s = K[4]; a.t = K[5];
    a.b = ks.b;
    a.shift = ks.shift;
    a.sc = s->ksc;
    a.part = s->part;
    double* d = s->ksc + nsg::KS_D;
    const double* stop = s->ksc + nsg::KS_STOP;
    // the projection's cell count (k_bicg_scal: mean = sum / n); infinite = no projection
    const double n = ks.op == 0 ? s->ncells : INFINITY;
    auto reduce = [&](int nb, int nv) -> int {
        nsg::launch_reduce_sum(s->part, nb, nv, d, s->st);
        return allreduce(s, d, nv, ncclSum);
    };
    // (r5) the grid apply / Jacobi launches of a converged batch do nothing (KS_STOP); the initial residual's
    // apply always runs
    auto apply = [&](double* x, double* y, const double* q, bool gate = true) -> int {
        CHK(halo(s, {x}, 1));
        const int nb = nsg::launch_apply(ks.op, s->g, s->c, ks.alpha, x, y, q, s->part, s->st, gate ? stop : nullptr);
        return reduce(nb, 2);
    };
    // timed level-0 passes of the preconditioner (events 0 .. tn), read after each host sync
    int tn = 0;
    const bool timed = s->timing && ks.stt && ks.mg;
    auto precond = [&](double* q, int k) -> int {   // K[k] = M^-1 q
        if (ks.mg && ks.op == 0 && s->fps_pc) return fps_precond(s, q, s->kv[k], s->kv[8]);
        if (ks.mg) return mg_precond(s, q, s->kv[k], s->kv[8], timed ? &tn : nullptr);
        nsg::launch_diag_pc(ks.op, s->g, s->c, ks.alpha, q, s->kv[k], s->st, stop);
        return 0;
    };
    // r = P(b - shift - A x), r0 = r, p = v = 0 (also the restart after a breakdown)
    auto init = [&]() -> int {
        CHK(apply(a.x, a.v, nullptr, false));
        nsg::launch_bicg_scal(nsg::KSC_MEAN, d, n, s->ksc, s->st);
        CHK(reduce(nsg::launch_bicg_vec(nsg::KV_INIT, a, s->st), 3));
        nsg::launch_bicg_scal(nsg::KSC_INIT, d, n, s->ksc, s->st);
        return 0;
    };
    auto iteration = [&]() -> int {
        nsg::launch_bicg_scal(nsg::KSC_CHECK, d, n, s->ksc, s->st);      // (the loop head's test, on the device)
        nsg::launch_bicg_scal(nsg::KSC_RHO, d, n, s->ksc, s->st);        // beta, rho
        nsg::launch_bicg_vec(nsg::KV_P, a, s->st);                        // p = r + beta (p - omega v)
        CHK(precond(a.p, 6));                                             // ph = M^-1 p
        a.ph = s->kv[6];
        CHK(apply(a.ph, a.v, a.r0));                                      // y = A ph, r0.y
        nsg::launch_bicg_scal(nsg::KSC_ALPHA, d, n, s->ksc, s->st);      // mean y, alpha
        nsg::launch_bicg_vec(nsg::KV_V, a, s->st);                        // v = P y, s = r - alpha v
        CHK(precond(a.s, 7));                                             // sh = M^-1 s
        a.sh = s->kv[7];
        CHK(apply(a.sh, a.t, nullptr));                                   // y = A sh
        nsg::launch_bicg_scal(nsg::KSC_MEAN, d, n, s->ksc, s->st);
        CHK(reduce(nsg::launch_bicg_vec(nsg::KV_T, a, s->st), 3));       // t = P y; t.s, t.t (3-wide partials)
        nsg::launch_bicg_scal(nsg::KSC_OMEGA, d, n, s->ksc, s->st);      // omega; KS_IT + 1
        CHK(reduce(nsg::launch_bicg_vec(nsg::KV_X, a, s->st), 3));       // x, r; r.r, r0.r, sum r
        return 0;
    };
    // (r5) the convergence test runs on the device at every iteration's head (KSC_CHECK) and freezes the rest of a
    // batch once it stops; the host reads the verdict once per batch -- the first sized from the previous solve of
    // this kind (Poisson, Helmholtz u, v), whose preconditioner launches cost a full iteration when frozen only for
    // the Poisson solve (its multigrid / box-direct preconditioners are not gated): one short there, one over for
    // the gated Helmholtz solves; then 1 (Poisson) or 2 (Helmholtz) at a time.  NSGPU_VERBOSE: every iteration
    const int kind = ks.op == 0 ? 0 : (ks.x == s->arr[NS_ARR_U] ? 1 : 2);
    const bool gated = !ks.mg;
    int batch = s->verbose ? 1 : std::max(1, gated ? s->kpred[kind] + 1 : s->kpred[kind] - 1);
    double kb2 = ks.b2;   // (< 0: not read yet -- the capacitance solve reads it with its residual)
    nsg::launch_bicg_start(s->ksc, tol2 * kb2, kb2, maxit, s->st);
    int its0 = 0;   // (the capacitance solve's refinements before any BiCGStab iteration)
    if (ks.op == 0 && s->cap.m > 0) {
        // (r5) a masked domain with its capacitance matrix: x = L_ext^+ (b - shift) (exact up to round-off; from
        // x = 0: b - shift is the projected residual, no operator application), then the residual -- one host
        // read per solve; a refinement x += L_ext^+ r only at rtol near the round-off (~1e-13).  Stagnating after
        // 3: BiCGStab preconditioned by the box's solve from this x
        nsg::launch_cap_rhs(s->g, ks.b, ks.shift, a.r, s->st);
        // (the rectangle's direct-solve check policy, fps_checks_next: inside steps the first solve and every
        // fps_check-th are checked, and every later one once a check came within 1/100 of rtol; an unchecked solve
        // reports res_phi = -1 and skips the residual pass and its host read)
        const bool check = !s->in_step || fps_checks_next(s);
        if (s->in_step) s->fps_solves++;
        for (;;) {
            // (the first from x = 0 without a border row: the solution's domain cells written straight into x)
            const bool direct_x = its0 == 0 && !s->cap.border && nsg::fps_idct_mask_ok(s->g.ny) && !s->fa.outE;
            if (direct_x) {
                CHK(cap_solve(s, a.r, s->kv[6], a.x));
            } else {
                CHK(cap_solve(s, a.r, s->kv[6]));
                nsg::launch_cap_axpy(s->g, s->cap, a.x, s->kv[6], its0 == 0, s->st);
            }
            if (!check) {
                *its = 1;
                *res = -1.0;
                return 0;
            }
            CHK(init());
            its0++;
            HIPCHK(hipMemcpyAsync(s->scal + S_KRY, d, sizeof(double), hipMemcpyDeviceToDevice, s->st));
            CHK(fetch(s));
            if (kb2 < 0) kb2 = s->hs[S_SHIFT + 1];   // (||b - mean||^2, from K3's reductions)
            const double r2 = s->hs[S_KRY], b2 = kb2;
            *res = b2 > 0 ? std::sqrt(r2 / b2) : std::sqrt(r2);
            *its = its0;
            if (s->verbose)
                fprintf(stderr, "nsgpu %s (capacitance solve): refinement %d rel. residual %.3e\n", ks.name, its0, *res);
            if (!std::isfinite(r2) || (b2 > 0 && r2 > 1e16 * b2)) {
                set_err("%s (capacitance solve) diverged: relative residual %g", ks.name, *res);
                return NS_EDIVERGE;
            }
            if (r2 <= tol2 * b2 || r2 == 0.0) {
                if (s->in_step && (its0 > 1 || *res > 1e-2 * s->rtol)) s->fps_strict = true;
                return 0;
            }
            if (s->in_step) s->fps_strict = true;
            if (its0 >= 3) {   // (BiCGStab from this x: its threshold with b2 known now)
                nsg::launch_bicg_start(s->ksc, tol2 * kb2, kb2, maxit, s->st);
                break;
            }
        }
    } else {
        CHK(init());
    }
    int restarts = 0;
    for (;;) {
        for (int q = 0; q < batch; q++) CHK(iteration());
        nsg::launch_bicg_scal(nsg::KSC_CHECK, d, n, s->ksc, s->st);
        // KS_STOP, KS_R2 / d[0], KS_IT, KS_BRK to the host (one sync per batch)
        HIPCHK(hipMemcpyAsync(s->scal + S_KRY, s->ksc + nsg::KS_STOP, sizeof(double), hipMemcpyDeviceToDevice, s->st));
        HIPCHK(hipMemcpyAsync(s->scal + S_KRY + 1, s->ksc + nsg::KS_BRK, sizeof(double), hipMemcpyDeviceToDevice, s->st));
        HIPCHK(hipMemcpyAsync(s->scal + S_KRY + 2, s->ksc + nsg::KS_IT, sizeof(double), hipMemcpyDeviceToDevice, s->st));
        HIPCHK(hipMemcpyAsync(s->scal + S_KRY + 3, s->ksc + nsg::KS_R2, sizeof(double), hipMemcpyDeviceToDevice, s->st));
        if (s->verbose) {
            HIPCHK(hipMemcpyAsync(s->scal + S_KRY + 4, d, sizeof(double), hipMemcpyDeviceToDevice, s->st));
            HIPCHK(hipMemcpyAsync(s->scal + S_KRY + 5, s->ksc + nsg::KS_ALPHA, 2 * sizeof(double), hipMemcpyDeviceToDevice, s->st));
        }
        CHK(fetch(s));
        for (int k = 0; k < tn; k++) {
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, s->ev[2 * k], s->ev[2 * k + 1]));
            if (s->evtag[k]) { ks.stt->t_restrict_kernel_ms += ms; ks.stt->n_restrict_kernels++; }
            else { ks.stt->t_poisson_kernel_ms += ms; ks.stt->n_poisson_kernels++; }
        }
        tn = 0;
        const bool stopped = s->hs[S_KRY] != 0.0, brk = s->hs[S_KRY + 1] != 0.0;
        const int it = (int)s->hs[S_KRY + 2];
        const double r2 = stopped ? s->hs[S_KRY + 3] : s->hs[S_KRY + 4], b2 = kb2;
        *res = b2 > 0 ? std::sqrt(r2 / b2) : std::sqrt(r2);
        if (s->verbose)
            fprintf(stderr, "nsgpu %s (bicgstab): it %d rel. residual %.3e (alpha %.3e omega %.3e%s)\n", ks.name, it,
                    *res, s->hs[S_KRY + 5], s->hs[S_KRY + 6], brk ? ", breakdown: restart" : "");
        *its = its0 + it;
        if (!stopped) {
            batch = s->verbose ? 1 : (gated ? 2 : 1);
            continue;
        }
        if (!std::isfinite(r2) || (b2 > 0 && r2 > 1e16 * b2)) {
            set_err("%s (BiCGStab) diverged: relative residual %g after %d iterations", ks.name, *res, it);
            return NS_EDIVERGE;
        }
        if (r2 <= tol2 * b2 || r2 == 0.0 || it >= maxit) break;
        // (stopped on a breakdown)
        if (++restarts > 50) { set_err("BiCGStab (%s) broke down 50 times", ks.name); return NS_EDIVERGE; }
        nsg::launch_bicg_scal(nsg::KSC_RESET, d, n, s->ksc, s->st);
        CHK(init());
        batch = 1;
    }
    s->kpred[kind] = *its - its0;
    return 0;
}

// every rank's n values `mine` into `all` (slot q = rank q, n values each).  RCCL: ncclAllGather; host
// transport: an exact sum-allreduce with the foreign slots zeroed; a virtual slab (loopback, nranks > 1):
// the same messages with itself as every peer
int allgather(ns_solver* s, const double* mine, double* all, size_t n) {
    const size_t P = (size_t)s->nranks, r = (size_t)s->rank;
    s->n_allred++;
    s->x_link += 8.0 * (double)n;   // (this rank's slot, one link per peer)
    if (s->ht.allreduce) {
        CHK(ensure_stage(s, P * n));
        // (the stream first: an earlier allreduce's copy back from the stage may still be queued --
        // the stage is written on the host only after the sync)
        HIPCHK(hipMemcpyAsync(s->stage + r * n, mine, n * 8, hipMemcpyDeviceToHost, s->st));
        HIPCHK(hipStreamSynchronize(s->st));
        std::fill(s->stage, s->stage + r * n, 0.0);
        std::fill(s->stage + (r + 1) * n, s->stage + P * n, 0.0);
        if (s->ht.allreduce(s->ht.user, s->stage, (int32_t)(P * n), 0) != 0) {
            set_err("host transport allreduce failed");
            return NS_ERCCL;
        }
        HIPCHK(hipMemcpyAsync(all, s->stage, P * n * 8, hipMemcpyHostToDevice, s->st));
        return 0;
    }
    if (s->loopback) {
        // (a virtual slab: the same ONE ncclAllGather launch as the real call, on the 1-rank communicator --
        // it fills this rank's slot; the others keep their zeros (r4 issued P - 1 self send / recv pairs,
        // which cost the slab's stream far more than one collective launch does).  (r5) NSGPU_VIRTUAL_COPY=1:
        // the slot filled by a device copy instead -- the 1-rank RCCL kernel of a 131 KB allgather runs on one
        // workgroup for ~60 us, a loopback artefact that tools/slab_projection.py's per-collective cost would
        // count twice)
        static const bool vcopy = getenv("NSGPU_VIRTUAL_COPY") && std::atoi(getenv("NSGPU_VIRTUAL_COPY")) != 0;
        if (vcopy) HIPCHK(hipMemcpyAsync(all + r * n, mine, n * 8, hipMemcpyDeviceToDevice, s->st));
        else NCCLCHK(ncclAllGather(mine, all + r * n, n, ncclDouble, s->comm, s->st));
        return 0;
    }
    NCCLCHK(ncclAllGather(mine, all, n, ncclDouble, s->comm, s->st));
    return 0;
}

// every rank's aggregate of one recurrence direction (fps_ragg: 2 x ld, then the deferred mean's sums) into
// fps_gath (slot q = rank q, fps_n doubles each)
int fps_allgather(ns_solver* s) { return allgather(s, s->fps_ragg, s->fps_gath, s->fps_n); }

// the group scan of one direction; multi-rank: this rank's aggregate first (its carries from zero,
// rewritten below), the allgather, the carry-in from the ranks before / after, then the scan from it
int pois_solve_krylov(ns_solver* s, int* its, double* res, ns_stats* stt);
int fps_scan(ns_solver* s, bool backward) {
    if (s->nranks == 1) {
        nsg::launch_fps_scan(s->fa, backward, nsg::FpsRank{}, nullptr, s->st);
        return 0;
    }
    if (s->fps_og) {
        // (r5) ONE allgather per solve: forward, the rank-local passes first -- the forward scan (this rank's
        // (E, P)), k_fps_mid without the chunk stores, the backward scan (its (X0, R) with a zero carry-in) --
        // then the allgather and the real forward scan; backward, the real scan with FpsRank::bq's carry-in
        nsg::FpsRank R{s->fps_gath, s->nranks, s->rank, (int)s->fps_n};
        if (backward) {
            R.bq = s->og_b;
            if (s->fps_og_mean) {   // (the mean was deferred in this solve's forward pass: the same correction)
                R.a1 = s->m0a;
                R.x1 = s->og_x1;
                R.ncells = s->ncells;
            }
            nsg::launch_fps_scan(s->fa, true, R, nullptr, s->st);
            return 0;
        }
        if (s->mean_pend) {
            R.a1 = s->m0a;
            R.ncells = s->ncells;
        }
        const size_t ld = s->g.ld;
        nsg::launch_fps_scan(s->fa, false, nsg::FpsRank{}, s->fps_ragg, s->st);
        nsg::FpsArgs fl = s->fa;
        fl.mid_local = 1;
        nsg::launch_fps_mid(fl, s->arr[NS_ARR_TMP], s->st);
        nsg::launch_fps_scan(s->fa, true, nsg::FpsRank{}, s->fps_ragg + 2 * ld + 8, s->st);
        CHK(fps_allgather(s));
        s->fps_og_mean = s->mean_pend;   // (the backward carry's mode-0 correction needs the same sums)
        if (s->mean_pend) {
            R.ge1 = s->m0g;
            R.shift = s->scal + S_SHIFT;
        }
        nsg::launch_fps_scan(s->fa, false, R, nullptr, s->st);
        return 0;
    }
    nsg::launch_fps_scan(s->fa, backward, nsg::FpsRank{}, s->fps_ragg, s->st);
    CHK(fps_allgather(s));
    // (the other ranks' carry-in is folded inside the scan; r4 had a k_fps_rank_carry launch per direction)
    nsg::FpsRank R{s->fps_gath, s->nranks, s->rank, (int)s->fps_n};
    if (!backward && s->mean_pend) {   // (r5) the deferred mean: its sums came with the aggregates
        R.a1 = s->m0a;
        R.ge1 = s->m0g;
        R.ncells = s->ncells;
        R.shift = s->scal + S_SHIFT;
    }
    nsg::launch_fps_scan(s->fa, backward, R, nullptr, s->st);
    return 0;
}

// (r6) rocBLAS / rocSOLVER for the dense y transforms, loaded on first use (dlopen): the common grids never map the
// libraries (their code objects would add ~20 MB to every process that loads libnsgpu.so)
struct DenseLib {
    bool tried = false, ok = false;
    decltype(&rocblas_create_handle) create = nullptr;
    decltype(&rocblas_destroy_handle) destroy = nullptr;
    decltype(&rocblas_set_stream) set_stream = nullptr;
    decltype(&rocblas_dgemm) dgemm = nullptr;
    decltype(&rocsolver_dstedc) dstedc = nullptr;
};
DenseLib& dense_lib() {
    static DenseLib L;
    if (L.tried) return L;
    L.tried = true;
    void* hb = dlopen("librocblas.so.5", RTLD_NOW | RTLD_GLOBAL);
    if (!hb) hb = dlopen("/opt/rocm/lib/librocblas.so", RTLD_NOW | RTLD_GLOBAL);
    void* hs = dlopen("librocsolver.so.0", RTLD_NOW | RTLD_GLOBAL);
    if (!hs) hs = dlopen("/opt/rocm/lib/librocsolver.so", RTLD_NOW | RTLD_GLOBAL);
    if (!hb || !hs) return L;
    L.create = (decltype(L.create))dlsym(hb, "rocblas_create_handle");
    L.destroy = (decltype(L.destroy))dlsym(hb, "rocblas_destroy_handle");
    L.set_stream = (decltype(L.set_stream))dlsym(hb, "rocblas_set_stream");
    L.dgemm = (decltype(L.dgemm))dlsym(hb, "rocblas_dgemm");
    L.dstedc = (decltype(L.dstedc))dlsym(hs, "rocsolver_dstedc");
    L.ok = L.create && L.destroy && L.set_stream && L.dgemm && L.dstedc;
    return L;
}

// the direct solve (ns_fps.hip): RPHI - shift -> PHI through the transformed plane in TMP; one
// "iteration".  A checked solve computes its residual; speculating, K5 is enqueued before the host
// reads it (as after a predicted multigrid check).  A residual above rtol (never seen: ~1e-14)
// continues with multigrid V-cycles from this phi.
int pois_solve_fps(ns_solver* s, int* its, double* res, ns_stats* stt) {
    const nsg::Geo& g = s->g;
    double* F = s->arr[NS_ARR_TMP];
    // timed steps: the transforms by their dispatch stamps (one rank), the recurrences (five launches,
    // the allgathers on slabs) between marker events
    const bool t = s->timing && s->in_step;
    // (fps_pre: K3's fused launch left this step's coefficients of b in F -- the recurrences take the
    // mean off mode 0 -- and timed itself into kev[2..3])
    const bool pre = s->fps_pre && s->in_step;
    s->fps_pre = false;
    nsg::FpsArgs fa = s->fa;
    // (r5: with an outflow side the mean never enters -- mode 0 takes the projected shift instead, ns_fps.hip
    // mode0_shift -- and the outflow row pair is transformed eliminated)
    const bool oe = s->fa.outE != 0;
    if (pre && !oe) fa.sh0 = s->scal + S_SHIFT;
    // (r5) the mean deferred to the forward allgather: t1b works on b's raw mode 0, k_fps_mid corrects
    // mode 0's chunk aggregates by the response to ny * mean, t2b takes the mean off on the fly
    const bool dm = pre && s->mean_pend;
    nsg::FpsArgs fa1 = fa, fam = fa;
    if (dm) {
        fa1.sh0 = nullptr;
        fam.m0e = s->m0e;
        fam.m0b = s->m0b;
        fam.m0s = s->scal + S_SHIFT;
    }
    if (t) {
        CHK(ensure_kev(s));
        if (!pre && !s->fps_dense) CHK(t_begin(s, s->kev[2], s->kev[3]));
    }
    // (the outflow row pair: the last rank's last local pair -- r6, slabs)
    const int oe_pair = oe && g.i0 + g.nxl == g.nx ? g.nxl / 2 - 1 : -1;
    if (s->fps_dense) {
        // (r6) the dense forward transform: F^T = F (N x N) b^T, one GEMM over the slab's rows (rocBLAS, column-major:
        // the row-major plane is its transpose); the mean comes off mode 0 in the recurrences (sh0, scale sh0s)
        if (t) HIPCHK(hipEventRecord(s->kev[2], s->st));
        const double one = 1.0, zero = 0.0;
        if (dense_lib().dgemm(s->rb, rocblas_operation_none, rocblas_operation_none, g.ny, g.nxl, g.ny, &one, s->dF, g.ny,
                          s->arr[NS_ARR_RPHI], g.ld, &zero, F, g.ld) != rocblas_status_success) {
            set_err("direct Poisson solve: the dense forward transform (rocblas_dgemm) failed");
            return NS_EHIP;
        }
        if (t) HIPCHK(hipEventRecord(s->kev[3], s->st));
        fa.sh0 = fa1.sh0 = fam.sh0 = s->scal + S_SHIFT;
    } else if (!pre && nsg::launch_fps_dct(false, s->arr[NS_ARR_RPHI], oe ? nullptr : s->scal + S_SHIFT, F, g.nxl, g.ny,
                                           g.ld, s->fps_tw, s->fps_wk, s->st, oe_pair, s->fps_tw8) < 0) {
        set_err("direct Poisson solve: ny = %d is not a supported power of two", g.ny);
        return NS_EINVAL;
    }
    if (t) {
        if (!pre && !s->fps_dense) CHK(t_end(s, s->kev[2], s->kev[3]));
        HIPCHK(hipEventRecord(s->kev[4], s->st));
    }
    if (oe && s->nranks > 1) {
        // (r6) slabs: the outflow row lives on the last rank -- its mode-0 shift 2 f'_{n-1} comes to every rank by one
        // scalar all-reduce before the recurrences, which then read it instead of their own last row
        nsg::launch_fps_oe_s0(F, g.nxl - 1, g.ld, g.i0 + g.nxl == g.nx ? 1 : 0, s->scal + S_OE, s->st);
        CHK(allreduce(s, s->scal + S_OE, 1, ncclSum));
        for (nsg::FpsArgs* q : {&fa, &fa1, &fam}) {
            q->s0 = s->scal + S_OE;
            q->s0_given = 1;
        }
    }
    if (s->fps_passes == 3) {   // (A/B: round 4's first form)
        nsg::launch_fps_t1(fa, F, s->st);
        CHK(fps_scan(s, false));
        nsg::launch_fps_t2(fa, F, s->st);
        CHK(fps_scan(s, true));
        nsg::launch_fps_t3(fa, F, s->st);
    } else {
        nsg::launch_fps_t1b(fa1, F, s->st);
        CHK(fps_scan(s, false));
        s->mean_pend = false;
        nsg::launch_fps_mid(fam, F, s->st);
        CHK(fps_scan(s, true));
        nsg::FpsArgs fa2 = fa;
        fa2.ghost = s->deep && s->in_step ? 1 : 0;   // (r5: phi's ghost rows from the solve -- K5 exchanges none)
        nsg::launch_fps_t2b(fa2, F, s->st);
    }
    // (r5) the inverse transform over the ghost rows t2b wrote too (deep slabs): rows [-glo, nxl + ghi)
    const int glo = s->fps_passes != 3 && s->deep && s->in_step && g.i0 > 0 ? 1 : 0;
    const int ghi = s->fps_passes != 3 && s->deep && s->in_step && g.i0 + g.nxl < g.nx ? 1 : 0;
    s->phi_ext = s->fps_passes != 3 && s->deep && s->in_step ? 1 : 0;
    if (t) {
        HIPCHK(hipEventRecord(s->kev[5], s->st));
        if (s->fps_dense) HIPCHK(hipEventRecord(s->kev[6], s->st));
        else CHK(t_begin(s, s->kev[6], s->kev[7]));
    }
    if (s->fps_dense) {   // (r6) phi^T = G (N x N) x^T over the rows the solve wrote
        const double one = 1.0, zero = 0.0;
        if (dense_lib().dgemm(s->rb, rocblas_operation_none, rocblas_operation_none, g.ny, g.nxl + glo + ghi, g.ny, &one,
                          s->dG, g.ny, F - (ptrdiff_t)glo * g.ld, g.ld, &zero,
                          s->arr[NS_ARR_PHI] - (ptrdiff_t)glo * g.ld, g.ld) != rocblas_status_success) {
            set_err("direct Poisson solve: the dense inverse transform (rocblas_dgemm) failed");
            return NS_EHIP;
        }
    } else {
        nsg::launch_fps_dct(true, F - (ptrdiff_t)glo * g.ld, nullptr, s->arr[NS_ARR_PHI] - (ptrdiff_t)glo * g.ld,
                            g.nxl + glo + ghi, g.ny, g.ld, s->fps_tw, s->fps_wk, s->st, -1, s->fps_tw8);
    }
    if (t) {
        if (s->fps_dense) HIPCHK(hipEventRecord(s->kev[7], s->st));
        else CHK(t_end(s, s->kev[6], s->kev[7]));
    }
    auto take_times = [&]() -> int {
        if (!t || !stt) return 0;
        HIPCHK(hipEventSynchronize(s->kev[7]));
        stt->t_fps_dct_ms += kev_ms(s, 2);
        stt->t_fps_tri_ms += kev_ms(s, 4);
        stt->t_fps_idct_ms += kev_ms(s, 6);
        stt->n_fps_solves++;
        return 0;
    };
    *its = 1;
    s->last_cycles = s->cur_cycles = -1;
    // (a standalone solve -- ns_kernel -- is always checked; inside steps every fps_check-th)
    // (fused: the check the launch stored rhs_phi for -- the same prediction, fps_checks_next)
    const bool check = pre ? s->fps_pre_b : !s->in_step || fps_checks_next(s);
    if (s->in_step) s->fps_solves++;
    if (!check) {
        // (not computed on this solve: ns_stats.res_phi = -1, phi_checked = 0 -- a residual the library
        // never measured is not reported as this solve's; the last check's value stays in fps_res)
        *res = -1.0;
        return take_times();
    }
    CHK(halo(s, {s->arr[NS_ARR_PHI]}, 1));   // (slabs: the residual's neighbour rows)
    if (oe) {
        // (r5) the outflow system's residual in the projected sense of the BiCGStab path: ||P (b - A phi)||
        // with A the reference's matrix (k_apply: the outflow rows' 2.5 / -2 / 0.5 ghost) and P the mean
        // projection; into S_RES through (sum r, sum r^2) and k_finish_mean's ||r - mean r||^2 (one rank)
        double* y = s->kv[0];
        nsg::launch_apply(0, g, s->c, 0.0, s->arr[NS_ARR_PHI], y, nullptr, s->part, s->st);
        nsg::launch_axpby(g, 1.0, s->arr[NS_ARR_RPHI], -1.0, y, y, s->st);
        // (r6) in two passes: the mean off r first, then the sums of r - mean -- the one-pass s2 - s^2 / n cancels
        // when r carries a large constant (the projected system's C 1): 5.7e-10 of noise for a ~1e-14 residual at
        // 4096 x 1024 (tools/fps_real_diag.py), which sent a converged solve into the BiCGStab polish
        for (int pass = 0; pass < 2; pass++) {
            if (pass) nsg::launch_cap_rhs(g, y, s->scal + S_AUX, y, s->st);
            const int nb = nsg::launch_sums(g, y, s->part, s->st);
            nsg::launch_reduce_sum(s->part, nb, 2, s->scal + S_AUX + 2, s->st);
            CHK(allreduce(s, s->scal + S_AUX + 2, 2, ncclSum));   // (r6: slabs; one rank: no-op)
            nsg::launch_finish_mean(s->scal + S_AUX + 2, s->ncells, s->scal + S_AUX, s->st);
        }
        HIPCHK(hipMemcpyAsync(s->scal + S_RES, s->scal + S_AUX + 1, sizeof(double), hipMemcpyDeviceToDevice, s->st));
    } else {
        const int nb = nsg::launch_pois_residual(g, s->c, s->arr[NS_ARR_PHI], s->arr[NS_ARR_RPHI], s->scal + S_SHIFT,
                                                 s->part, s->st);
        nsg::launch_reduce_sum(s->part, nb, 1, s->scal + S_RES, s->st);
        CHK(allreduce(s, s->scal + S_RES, 1, ncclSum));
    }
    const bool spec = s->speculate && s->in_step && !s->defer_now;
    if (spec) {
        CHK(fetch_begin(s));
        CHK(correct_launch(s, s->part + 4 * (size_t)nsg::max_partials(s->g)));
        s->n_spec++;
        CHK(fetch_end(s));
    } else {
        CHK(fetch(s));
    }
    if (stt) stt->n_checks++;
    CHK(take_times());
    const double r2 = s->hs[S_RES], b2 = s->hs[S_SHIFT + 1];
    *res = s->fps_res = b2 > 0 ? std::sqrt(r2 / b2) : std::sqrt(r2);
    if (s->verbose) fprintf(stderr, "nsgpu poisson: direct solve, rel. residual %.3e\n", *res);
    if (!std::isfinite(r2)) { set_err("Poisson residual is not finite"); return NS_EDIVERGE; }
    // (a virtual slab's own residual is not the global solve's: it replays, never falls back)
    if (r2 <= s->rtol * s->rtol * b2 || r2 == 0.0 || s->rp_c >= 0) {
        if (spec) { s->k5_spec = 1; s->n_spec_hit++; }
        // the checks are skipped between every fps_check-th solve only while the measured residual sits
        // two orders of magnitude below rtol (the solve's round-off: ~1e-13 of ||b|| at 4096^2 against
        // 1e-8); a residual within 1/100 of rtol (e.g. rtol 1e-12 at 2048^2) makes every later solve checked
        if (s->in_step && s->rp_c < 0 && *res > 1e-2 * s->rtol) s->fps_strict = true;
        return 0;
    }
    // (the speculative K5 wrote only the ping-pong partners: correct() runs it again).  An rtol below
    // the direct solve's round-off (e.g. 1e-12 at 2048^2: 1.25e-12) -- every later solve is checked
    // and refined the same way
    if (s->in_step) s->fps_strict = true;
    s->phi_ext = 0;   // (the refinement below changes phi's own rows only)
    CHK(halo(s, {s->arr[NS_ARR_RPHI]}, 4));   // (the direct solve read no rhs ghost rows)
    int c = 0;
    // (an outflow side: the BiCGStab solve of the true matrix, from this phi)
    CHK(oe ? pois_solve_krylov(s, &c, res, stt)
           : s->poisson == NS_POISSON_MG ? pois_solve_mg(s, &c, res, stt) : pois_solve(s, &c, res, stt));
    s->fps_res = *res;
    *its = 1 + c;
    return 0;
}

int pois_solve_krylov(ns_solver* s, int* its, double* res, ns_stats* stt) {
    // ||b - mean||^2 for the relative test (r5: the capacitance solve reads it with its residual, b2 = -1 here)
    if (!s->cap.m) CHK(fetch(s));
    const KrylovSolve ks{0, 0.0, s->krylov_mg, s->arr[NS_ARR_PHI], s->arr[NS_ARR_RPHI],
                         s->scal + (s->consist ? S_KSHIFT : S_SHIFT), s->cap.m ? -1.0 : s->hs[S_SHIFT + 1], "poisson",
                         stt};
    const int rc = bicgstab(s, ks, its, res);
    // (the capacitance solve: one residual per refinement, none on an unchecked solve)
    if (stt) stt->n_checks += s->cap.m ? (*res >= 0.0 ? *its : 0) : *its + 1;
    // (last_cycles / cur_cycles -1: the quadratic guess -- the channel's BiCGStab took 5.1
    // iterations per step with the cubic against 4.75 with the quadratic, r3)
    s->last_cycles = s->cur_cycles = -1;
    return rc;
}

int pois_solve_any(ns_solver* s, int* its, double* res, ns_stats* stt) {
    // (r5: the direct solve first -- it now covers the E-outflow channel, whose Krylov planes exist too)
    if (s->fps) return pois_solve_fps(s, its, res, stt);
    if (s->kv[0]) return pois_solve_krylov(s, its, res, stt);
    if (s->poisson == NS_POISSON_MG) return pois_solve_mg(s, its, res, stt);
    s->last_cycles = s->cur_cycles = -1;
    return pois_solve(s, its, res, stt);
}

// host tables of the direct solve (ns_create): twiddles, the modes' eigenvalues and every chunk's
// entry pivot.  The pivots p_i(k) of Thomas' recurrence (ns_fps.hip) depend on the operator only:
// the host runs the recurrence over the global rows up to the slab's end and keeps 1 / p of the row
// before each chunk of this slab (0 before global row 0, whose pw is 0)
int fps_setup(ns_solver* s, const std::vector<double>& hy, const double* pw, const double* pe) {
    const nsg::Geo& g = s->g;
    const int N = g.ny, ld = g.ld;
    nsg::FpsArgs& a = s->fa;
    a.nx = g.nx; a.i0 = g.i0; a.nxl = g.nxl; a.ny = N; a.ld = ld;
    a.nch = (g.nxl + nsg::FPS_M - 1) / nsg::FPS_M;
    a.ngrp = (a.nch + nsg::FPS_G - 1) / nsg::FPS_G;
    a.pin = 1;   // (every side of the rectangle is zero-flux for phi: Lx 1 = 0)
    const int nchp = a.ngrp * nsg::FPS_G;   // (t1 / t2 / t3 address whole groups' chunks)
    const size_t n_tab = 4 * (size_t)N + (size_t)N, n_rp0 = (size_t)nchp * ld, n_g = (size_t)a.ngrp * ld;
    // multi-rank: the allgather's own slot and every rank's (fps_n each), and the deferred mean's mode-0
    // tables (chunks' E and BXl, groups', ranks' aggregates of the constant 1)
    {
        const char* e = getenv("NSGPU_FPS_ONEGATHER");
        s->fps_og = s->nranks > 1 && s->nranks <= 64 && s->fps_passes != 3 && !(e && std::atoi(e) == 0);
    }
    s->fps_n = (s->fps_og ? 4 : 2) * (size_t)ld + 8;
    const size_t n_og = s->fps_og ? (size_t)s->nranks * ld + s->nranks : 0;
    const size_t n_mr = s->nranks > 1 ? (size_t)(1 + s->nranks) * s->fps_n + 2 * (size_t)nchp + a.ngrp + s->nranks + n_og
                                      : 0;
    const size_t n_bt = 2 * (size_t)nchp * ld;
    const size_t total = n_tab + n_rp0 + n_bt + 6 * n_g + 5 * (size_t)nchp * ld + n_mr + 8;
    std::vector<double> h(n_tab + n_rp0 + n_bt, 0.0);
    const double pi = 3.14159265358979323846;
    for (int m = 0; m < N; m++) {
        const double t = 2.0 * pi * ((double)m / N);
        h[2 * m] = std::cos(t);
        h[2 * m + 1] = -std::sin(t);
        const double u = pi * ((double)m / (2.0 * N));
        h[2 * N + 2 * m] = std::cos(u);
        h[2 * N + 2 * m + 1] = -std::sin(u);
        const double sn = std::sin(u);
        h[4 * N + m] = -4.0 / (hy[0] * hy[0]) * sn * sn;   // -(2/hy^2)(1 - cos(pi m / N))
    }
    if (s->fps_dense) {
        // (r6) Ly's eigen-decomposition (the Poisson operator along y, ConstructLHS FluidSolver.cpp:113-131: zero-flux
        // faces, 2 / (h (h + h_nb)) toward each neighbour): S = H^1/2 Ly H^-1/2 is symmetric tridiagonal (diagonal
        // -(ps + pn), off-diagonal sqrt(pn_j ps_j+1)); rocSOLVER's divide and conquer gives its eigenpairs, the
        // transforms F = Q^T H^1/2, G = H^-1/2 Q (mode 0 = the zero eigenvalue, its vector H^1/2 1 set exactly)
        std::vector<double> dg(N), of(std::max(N - 1, 1), 0.0), shy(N);
        double sumhy = 0.0;
        for (int j = 0; j < N; j++) {
            const double ps = j > 0 ? 2.0 / (hy[j] * (hy[j] + hy[j - 1])) : 0.0;
            const double pn = j < N - 1 ? 2.0 / (hy[j] * (hy[j] + hy[j + 1])) : 0.0;
            dg[j] = -(ps + pn);
            if (j < N - 1) of[j] = std::sqrt(pn * (2.0 / (hy[j + 1] * (hy[j + 1] + hy[j]))));
            shy[j] = std::sqrt(hy[j]);
            sumhy += hy[j];
        }
        DenseLib& DL = dense_lib();
        if (!DL.ok) { set_err("the dense y transforms need librocblas / librocsolver (dlopen failed)"); return NS_EINVAL; }
        if (DL.create(&s->rb) != rocblas_status_success) { set_err("rocblas_create_handle failed"); return NS_EHIP; }
        if (DL.set_stream(s->rb, s->st) != rocblas_status_success) { set_err("rocblas_set_stream failed"); return NS_EHIP; }
        const size_t nn = (size_t)N * N;
        HIPCHK(hipMalloc(&s->dense_mem, (3 * nn + 3 * (size_t)N + 8) * sizeof(double)));
        s->dF = s->dense_mem;
        s->dG = s->dF + nn;
        double *dC = s->dG + nn, *dD = dC + nn, *dE = dD + N, *dS = dE + N;
        rocblas_int* dinfo = reinterpret_cast<rocblas_int*>(dS + N);
        HIPCHK(hipMemcpy(dD, dg.data(), N * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(dE, of.data(), std::max(N - 1, 1) * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(dS, shy.data(), N * sizeof(double), hipMemcpyHostToDevice));
        if (DL.dstedc(s->rb, rocblas_evect_tridiagonal, N, dD, dE, dC, N, dinfo) != rocblas_status_success) {
            set_err("rocsolver_dstedc failed (ny = %d)", N);
            return NS_EHIP;
        }
        rocblas_int info = 0;
        std::vector<double> lam(N);
        HIPCHK(hipMemcpyAsync(&info, dinfo, sizeof(info), hipMemcpyDeviceToHost, s->st));
        HIPCHK(hipMemcpyAsync(lam.data(), dD, N * sizeof(double), hipMemcpyDeviceToHost, s->st));
        HIPCHK(hipStreamSynchronize(s->st));
        if (info != 0) { set_err("rocsolver_dstedc: info %d (ny = %d)", (int)info, N); return NS_EHIP; }
        // mode k: the (N - 1 - k)-th smallest eigenvalue (ascending from rocSOLVER): mode 0 the zero one
        for (int k = 0; k < N; k++) h[4 * N + k] = k == 0 ? 0.0 : lam[N - 1 - k];
        nsg::launch_dense_mats(dC, dS, 1.0 / std::sqrt(sumhy), N, s->dF, s->dG, s->st);
        HIPCHK(hipStreamSynchronize(s->st));
        a.sh0s = std::sqrt(sumhy);   // (mode 0 of the constant 1: sum_j hy_j / sqrt(sum hy))
    }
    double* rp0 = h.data() + n_tab;
    double* bt = rp0 + n_rp0;   // per chunk: beta (the local back substitution over pi) and BR
    std::vector<double> r(N, 0.0);   // 1 / p of the previous row, per mode
    std::vector<double> crp((size_t)nsg::FPS_M * N), cpi((size_t)nsg::FPS_M * N);   // this chunk's 1/p, pi
    const int iend = g.i0 + g.nxl;
    for (int gi = 0; gi < iend; gi++) {
        const int li = gi - g.i0;
        if (li >= 0 && li % nsg::FPS_M == 0)
            for (int k = 0; k < N; k++) rp0[(size_t)(li / nsg::FPS_M) * ld + k] = r[k];
        const double pem = gi > 0 ? pe[gi - 1] : 0.0;
        const int t = li >= 0 ? li % nsg::FPS_M : 0;
        // (r5: the NEUMANN outflow row eliminated to (-mu / 2, mu): ns_fps.hip piv_next)
        const bool oe = a.outE && gi == g.nx - 1;
        for (int k = 0; k < N; k++) {
            const double gg = (oe ? -0.5 * h[4 * N + k] : pw[gi]) * r[k];
            const double p = std::fma(-gg, pem, oe ? h[4 * N + k] : -(pw[gi] + pe[gi]) + h[4 * N + k]);   // (piv_next's)
            r[k] = (k == 0 && gi == g.nx - 1) ? 0.0 : 1.0 / p;
            if (li >= 0) {
                crp[(size_t)t * N + k] = r[k];
                cpi[(size_t)t * N + k] = -gg * (t ? cpi[(size_t)(t - 1) * N + k] : 1.0);
            }
        }
        if (li >= 0 && (t == nsg::FPS_M - 1 || gi == iend - 1)) {   // the chunk's (beta, BR)
            const int c = li / nsg::FPS_M;
            for (int k = 0; k < N; k++) {
                double b = 0.0, R = 1.0;
                for (int u = t; u >= 0; u--) {
                    const double rr = crp[(size_t)u * N + k], q = -pe[gi - t + u] * rr;
                    b = cpi[(size_t)u * N + k] * rr + q * b;
                    R = q * R;
                }
                bt[(size_t)c * ld + k] = b;
                bt[(size_t)(a.nch + c) * ld + k] = R;
            }
        }
    }
    // (r5) the pivots tabled for t1b / t2b (ns_fps.hip piv_pair): the recurrence of every mode from global row
    // 0 over uniform interior rows reaches its fixed point (to 4 ulp) after c_k rows -- many for the low modes,
    // few for the high ones; whole waves of modes k >= kfast whose c_k are all below prow read 1 / p from
    // the table there and the converged value after it, instead of one fp64 division per row and mode
    // (NSGPU_FPS_PTAB=0: divisions everywhere, A/B)
    std::vector<double> ptab, pinf;
    std::vector<int> prowb;
    int prow = 0, kfast = 1 << 30;
    {
        // NSGPU_FPS_PTAB: 0 divisions everywhere, 1 the table (A/B), 2 (default) per 128-mode block its fixed-point row
        const char* pe_env = getenv("NSGPU_FPS_PTAB");
        const int mode = !s->fps_xuni || s->fps_dense ? 0 : pe_env ? std::atoi(pe_env) : 2;   // (r6: stretched -- none)
        const int PRMAX = std::min(g.nx - 1, mode == 1 ? 1024 : 4096);
        if (mode != 0 && N > 128 && PRMAX > 64) {
            std::vector<double> rr(N, 0.0);
            std::vector<int> conv(N, -1);
            std::vector<char> left(N, 0);
            if (mode == 1) ptab.assign((size_t)PRMAX * ld, 0.0);
            for (int gi = 0; gi < PRMAX; gi++) {
                const double pem = gi > 0 ? pe[gi - 1] : 0.0;
                for (int k = 0; k < N; k++) {
                    const double gg = pw[gi] * rr[k];
                    const double pv = std::fma(-gg, pem, -(pw[gi] + pe[gi]) + h[4 * N + k]);
                    const double rn = 1.0 / pv;
                    // (mode 2: the exact fixed point -- the recurrence returns the same bits from here on, so the
                    // skipped divisions change nothing; mode 1: within 4 ulp)
                    const bool fixed = mode == 2 ? rn == rr[k] : std::fabs(rn - rr[k]) <= 4 * 2.220446049250313e-16 * std::fabs(rn);
                    if (conv[k] < 0 && !left[k] && gi > 1 && fixed) conv[k] = gi;
                    if (mode == 2 && conv[k] >= 0 && rn != rr[k]) {   // (left it again -- an oscillation: never fast)
                        conv[k] = -1;
                        left[k] = 1;
                    }
                    rr[k] = rn;
                    if (mode == 1) ptab[(size_t)gi * ld + k] = rn;
                }
            }
            if (mode == 2) {
                // (each block's row: the last of its modes to converge, + 1; a block with a mode that did not
                // converge within PRMAX rows never takes the fixed point)
                const int nb = (ld + 127) / 128;
                prowb.assign(nb, 1 << 30);
                bool any = false;
                for (int b = 0; b < nb; b++) {
                    int mx = 0;
                    bool ok = b * 128 < N;
                    for (int k = b * 128; k < std::min(N, (b + 1) * 128) && ok; k++) {
                        ok = conv[k] >= 0;
                        mx = std::max(mx, conv[k]);
                    }
                    if (ok) { prowb[b] = mx + 1; any = true; }
                }
                if (any) {
                    pinf.assign(ld, 0.0);
                    for (int k = 0; k < N; k++) pinf[k] = rr[k];
                } else {
                    prowb.clear();
                }
            } else {
            for (int kf = 128; kf < N; kf += 128) {
                int mx = 0;
                bool ok = true;
                for (int k = kf; k < N && ok; k++) {
                    ok = conv[k] >= 0;
                    mx = std::max(mx, conv[k]);
                }
                if (ok) {
                    kfast = kf;
                    prow = std::min(PRMAX, (mx + 1 + 15) / 16 * 16);
                    break;
                }
            }
            if (kfast < N) {
                pinf.assign(ld, 0.0);
                for (int k = 0; k < N; k++) pinf[k] = rr[k];
                ptab.resize((size_t)prow * ld);
            } else {
                ptab.clear();
                kfast = 1 << 30;
            }
            }
        }
    }
    // (the pivot table and pinf, or pinf and the block rows -- ints, in doubles' room)
    const size_t n_pt = !ptab.empty() ? ptab.size() + (size_t)ld : (!prowb.empty() ? (size_t)ld + prowb.size() : 0);
    // (r5) ny = 16384: e^{-2 pi i m / 8192}, m < 8192, after the pivot table (the two-half transforms)
    const size_t n_t8 = nsg::fps_log2(N) < 0 ? (size_t)N : 0;
    HIPCHK(hipMalloc(&s->fps_mem, (total + n_pt + n_t8) * sizeof(double)));
    HIPCHK(hipMemset(s->fps_mem, 0, (total + n_pt + n_t8) * sizeof(double)));
    HIPCHK(hipMemcpy(s->fps_mem, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
    if (n_t8) {
        std::vector<double> t8(n_t8);
        for (int m = 0; m < N / 2; m++) {
            t8[2 * m] = h[4 * m];   // (the 16384-point table's even entries)
            t8[2 * m + 1] = h[4 * m + 1];
        }
        s->fps_tw8 = s->fps_mem + total + n_pt;
        HIPCHK(hipMemcpy(s->fps_mem + total + n_pt, t8.data(), n_t8 * sizeof(double), hipMemcpyHostToDevice));
    }
    if (n_pt && !ptab.empty()) {
        double* pt = s->fps_mem + total;
        HIPCHK(hipMemcpy(pt, ptab.data(), ptab.size() * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(pt + ptab.size(), pinf.data(), (size_t)ld * sizeof(double), hipMemcpyHostToDevice));
        a.ptab = pt;
        a.pinf = pt + ptab.size();
        a.prow = prow;
        a.kfast = kfast;
    } else if (n_pt) {
        double* pt = s->fps_mem + total;
        HIPCHK(hipMemcpy(pt, pinf.data(), (size_t)ld * sizeof(double), hipMemcpyHostToDevice));
        int* pb = reinterpret_cast<int*>(pt + ld);
        HIPCHK(hipMemcpy(pb, prowb.data(), prowb.size() * sizeof(int), hipMemcpyHostToDevice));
        a.pinf = pt;
        a.prowb = pb;
    }
    double* d = s->fps_mem;
    s->fps_tw = d;
    s->fps_wk = d + 2 * (size_t)N;
    a.mu = d + 4 * (size_t)N;
    a.rp0 = d + n_tab;
    a.bt = d + n_tab + n_rp0;
    double* q = d + n_tab + n_rp0 + n_bt;
    a.ga = q; q += 2 * n_g;
    a.gc = q; q += n_g;
    a.gb = q; q += 2 * n_g;
    a.gx = q; q += n_g;
    a.cb = q; q += 2 * (size_t)nchp * ld;
    a.ca = q; q += 2 * (size_t)nchp * ld;
    a.ya = q; q += (size_t)nchp * ld;
    a.s0 = d + total - 8;   // (r5: the outflow's mode-0 shift, k_fps_mid -> t2b)
    if (n_mr) {
        s->fps_ragg = q; q += s->fps_n;
        s->fps_gath = q; q += (size_t)s->nranks * s->fps_n;
        // mode 0's response to the constant 1 (r5, the deferred mean): the same recurrences as the kernels
        // (piv_next, t1b's forward and local back substitution) over f = 1, with mode 0's pivots of the
        // global rows
        const int nx = g.nx;
        std::vector<double> r0(nx);
        {
            double rp = 0.0;
            for (int gi = 0; gi < nx; gi++) {
                const double gg = pw[gi] * rp, pem = gi > 0 ? pe[gi - 1] : 0.0;
                const double p = std::fma(-gg, pem, -(pw[gi] + pe[gi]) + 0.0);
                rp = r0[gi] = gi == nx - 1 ? 0.0 : 1.0 / p;   // (mode 0's pinned last row, a.pin)
            }
        }
        auto fwd = [&](int ga, int gb) {   // forward recurrence from zero over global rows [ga, gb)
            double E = 0.0;
            for (int gi = ga; gi < gb; gi++) E = std::fma(-(pw[gi] * (gi > 0 ? r0[gi - 1] : 0.0)), E, 1.0);
            return E;
        };
        std::vector<double> m0((size_t)2 * nchp + a.ngrp + s->nranks, 0.0);
        for (int c = 0; c < a.nch; c++) {
            const int gi0 = g.i0 + c * nsg::FPS_M, gi1 = std::min(gi0 + nsg::FPS_M, g.i0 + g.nxl);
            std::vector<double> y;
            double E = 0.0;
            for (int gi = gi0; gi < gi1; gi++) {
                E = std::fma(-(pw[gi] * (gi > 0 ? r0[gi - 1] : 0.0)), E, 1.0);
                y.push_back(E);
            }
            double xl = 0.0;
            for (int gi = gi1 - 1; gi >= gi0; gi--) xl = std::fma(y[gi - gi0], r0[gi], -pe[gi] * r0[gi] * xl);
            m0[c] = E;
            m0[(size_t)nchp + c] = xl;
        }
        for (int gq = 0; gq < a.ngrp; gq++)
            m0[2 * (size_t)nchp + gq] = fwd(g.i0 + gq * nsg::FPS_G * nsg::FPS_M,
                                            std::min(g.i0 + (gq + 1) * nsg::FPS_G * nsg::FPS_M, g.i0 + g.nxl));
        for (int rq = 0; rq < s->nranks; rq++) {
            int32_t q0, q1;
            ns_slab_range(g.nx, s->nranks, rq, &q0, &q1);
            m0[2 * (size_t)nchp + a.ngrp + rq] = fwd(q0, q1);
        }
        HIPCHK(hipMemcpy(q, m0.data(), m0.size() * sizeof(double), hipMemcpyHostToDevice));
        s->m0e = q;
        s->m0b = q + nchp;
        s->m0g = q + 2 * (size_t)nchp;
        s->m0a = s->m0g + a.ngrp;
        q += m0.size();
        if (s->fps_og) {
            // (r5) every rank's backward aggregate (x at its first row, zero carry from the ranks after it) as a
            // function of its forward carry-in Y: with f = 0, y_i = Y prod(-g), x_i = y_i r_i - pe_i r_i x_{i+1}, so
            // B_p(k) = sum_i prod_{m <= i}(-g_m) r_i prod_{m < i}(-pe_m r_m) over rank p's rows (piv_next's pivots);
            // X1_p: mode 0's aggregate of f = 1 from zero (the deferred mean's correction)
            const int P = s->nranks;
            std::vector<double> B((size_t)P * ld, 0.0), X1(P, 0.0), rr(N, 0.0), fw(N), bw(N);
            int rq = 0;
            int32_t q0 = 0, q1 = 0;
            ns_slab_range(nx, P, 0, &q0, &q1);
            double y1 = 0.0, bw1 = 1.0;
            for (int gi = 0; gi < nx; gi++) {
                while (gi >= q1) { rq++; ns_slab_range(nx, P, rq, &q0, &q1); }
                if (gi == q0) {
                    std::fill(fw.begin(), fw.end(), 1.0);
                    std::fill(bw.begin(), bw.end(), 1.0);
                    y1 = 0.0;
                    bw1 = 1.0;
                }
                const double pem = gi > 0 ? pe[gi - 1] : 0.0;
                double* Bq = B.data() + (size_t)rq * ld;
                const bool oe = a.outE && gi == nx - 1;   // (r6: the eliminated outflow row, piv_next)
                for (int k = 0; k < N; k++) {
                    const double gg = (oe ? -0.5 * h[4 * N + k] : pw[gi]) * rr[k];
                    const double p = std::fma(-gg, pem, oe ? h[4 * N + k] : -(pw[gi] + pe[gi]) + h[4 * N + k]);
                    rr[k] = (k == 0 && gi == nx - 1) ? 0.0 : 1.0 / p;
                    fw[k] *= -gg;
                    Bq[k] += fw[k] * rr[k] * bw[k];
                    bw[k] *= -pe[gi] * rr[k];
                }
                // (mode 0, f = 1: y_i = 1 - g_i y_{i-1}, the same back substitution)
                y1 = std::fma(-(pw[gi] * (gi > 0 ? r0[gi - 1] : 0.0)), y1, 1.0);
                X1[rq] += y1 * r0[gi] * bw1;
                bw1 *= -pe[gi] * r0[gi];
            }
            HIPCHK(hipMemcpy(q, B.data(), B.size() * sizeof(double), hipMemcpyHostToDevice));
            s->og_b = q;
            q += B.size();
            HIPCHK(hipMemcpy(q, X1.data(), X1.size() * sizeof(double), hipMemcpyHostToDevice));
            s->og_x1 = q;
            q += X1.size();
        }
    }
    a.pw = s->c.pw;
    a.pe = s->c.pe;
    return 0;
}

// coefficient tables of one level: [pw pe bx | ps pn by | hx hy]  (ConstructLHS, FluidSolver.cpp:113-131)
// neu[side]: a NEUMANN outflow side, whose velocity ghost q (:98) adds no Helmholtz wall term
std::vector<double> coef_tables(const std::vector<double>& hx, const std::vector<double>& hy,
                                const int* neu = nullptr) {
    const int nz[4] = {0, 0, 0, 0};
    if (!neu) neu = nz;
    const int nx = (int)hx.size(), ny = (int)hy.size();
    std::vector<double> h(8 * (size_t)nx + 8 * (size_t)ny + 2, 0.0);
    double *pw = h.data(), *pe = pw + nx, *bx = pe + nx, *ps = bx + nx, *pn = ps + ny, *by = pn + ny;
    double *hxo = by + ny, *hyo = hxo + nx;
    double *rhx = hyo + ny, *rhy = rhx + nx, *rsx = rhy + ny, *rsy = rsx + nx + 1;
    double *fwx = rsy + ny + 1, *fex = fwx + nx, *fsy = fex + nx, *fny = fsy + ny;
    // Div_V / GradP face weights r = h / (h_nb + h) (FluidSolver.cpp:389-414, 429-452)
    for (int i = 0; i < nx; i++) {
        fwx[i] = i > 0 ? hx[i] / (hx[i - 1] + hx[i]) : 0.0;
        fex[i] = i < nx - 1 ? hx[i] / (hx[i + 1] + hx[i]) : 0.0;
    }
    for (int j = 0; j < ny; j++) {
        fsy[j] = j > 0 ? hy[j] / (hy[j - 1] + hy[j]) : 0.0;
        fny[j] = j < ny - 1 ? hy[j] / (hy[j + 1] + hy[j]) : 0.0;
    }
    for (int i = 0; i < nx; i++) rhx[i] = 1.0 / hx[i];
    for (int j = 0; j < ny; j++) rhy[j] = 1.0 / hy[j];
    for (int i = 1; i < nx; i++) rsx[i] = 2.0 / (hx[i - 1] + hx[i]);
    for (int j = 1; j < ny; j++) rsy[j] = 2.0 / (hy[j - 1] + hy[j]);
    for (int i = 0; i < nx; i++) {
        const double a = hx[i];
        hxo[i] = a;
        pw[i] = i > 0 ? 2.0 / (a * (a + hx[i - 1])) : 0.0;
        pe[i] = i < nx - 1 ? 2.0 / (a * (a + hx[i + 1])) : 0.0;
        bx[i] = (i == 0 && !neu[0] ? 2.0 / (a * a) : 0.0) + (i == nx - 1 && !neu[1] ? 2.0 / (a * a) : 0.0);
    }
    for (int j = 0; j < ny; j++) {
        const double a = hy[j];
        hyo[j] = a;
        ps[j] = j > 0 ? 2.0 / (a * (a + hy[j - 1])) : 0.0;
        pn[j] = j < ny - 1 ? 2.0 / (a * (a + hy[j + 1])) : 0.0;
        by[j] = (j == 0 && !neu[2] ? 2.0 / (a * a) : 0.0) + (j == ny - 1 && !neu[3] ? 2.0 / (a * a) : 0.0);
    }
    return h;
}

nsg::Coef coef_view(double* d, int nx, int ny) {
    nsg::Coef c{};
    c.pw = d; c.pe = d + nx; c.bx = d + 2 * nx;
    c.ps = d + 3 * nx; c.pn = d + 3 * nx + ny; c.by = d + 3 * nx + 2 * ny;
    c.hx = d + 3 * nx + 3 * ny; c.hy = d + 4 * nx + 3 * ny;
    c.rhx = d + 4 * nx + 4 * ny; c.rhy = d + 5 * nx + 4 * ny;
    c.rsx = d + 5 * nx + 5 * ny; c.rsy = d + 6 * nx + 5 * ny + 1;
    c.fwx = d + 6 * nx + 6 * ny + 2; c.fex = c.fwx + nx; c.fsy = c.fex + nx; c.fny = c.fsy + ny;
    return c;
}

// symmetric eigen-decomposition by cyclic Jacobi rotations: a (n x n, row-major, destroyed) ->
// eigenvalues lam, orthonormal eigenvectors in the columns of v (row-major)
void jacobi_eigen(int n, std::vector<double>& a, std::vector<double>& lam, std::vector<double>& v) {
    v.assign((size_t)n * n, 0.0);
    for (int i = 0; i < n; i++) v[(size_t)i * n + i] = 1.0;
    for (int sweep = 0; sweep < 100; sweep++) {
        double off = 0.0, dg = 0.0;
        for (int p = 0; p < n; p++) {
            dg += a[(size_t)p * n + p] * a[(size_t)p * n + p];
            for (int q = p + 1; q < n; q++) off += a[(size_t)p * n + q] * a[(size_t)p * n + q];
        }
        if (off <= 1e-34 * dg) break;
        for (int p = 0; p < n; p++)
            for (int q = p + 1; q < n; q++) {
                const double apq = a[(size_t)p * n + q];
                if (apq == 0.0) continue;
                // the rotation in (p, q) that zeroes a_pq: t = tan(theta), the smaller root of
                // t^2 + 2 tau t - 1 = 0, tau = (a_qq - a_pp) / (2 a_pq)
                const double tau = (a[(size_t)q * n + q] - a[(size_t)p * n + p]) / (2.0 * apq);
                const double t = (tau >= 0.0 ? 1.0 : -1.0) / (std::fabs(tau) + std::sqrt(1.0 + tau * tau));
                const double c = 1.0 / std::sqrt(1.0 + t * t), sn = t * c;
                for (int k = 0; k < n; k++) {   // A J
                    const double akp = a[(size_t)k * n + p], akq = a[(size_t)k * n + q];
                    a[(size_t)k * n + p] = c * akp - sn * akq;
                    a[(size_t)k * n + q] = sn * akp + c * akq;
                }
                for (int k = 0; k < n; k++) {   // J^T (A J)
                    const double apk = a[(size_t)p * n + k], aqk = a[(size_t)q * n + k];
                    a[(size_t)p * n + k] = c * apk - sn * aqk;
                    a[(size_t)q * n + k] = sn * apk + c * aqk;
                }
                for (int k = 0; k < n; k++) {   // V J
                    const double vkp = v[(size_t)k * n + p], vkq = v[(size_t)k * n + q];
                    v[(size_t)k * n + p] = c * vkp - sn * vkq;
                    v[(size_t)k * n + q] = sn * vkp + c * vkq;
                }
            }
    }
    lam.resize(n);
    for (int i = 0; i < n; i++) lam[i] = a[(size_t)i * n + i];
}

// The exact solve of the coarsest level (k_direct): its 1-D operators from the level's own
// tables (w = pw, e = pe: the outflow closure's pw[0] / pe[n-1] toward a zero ghost included),
// L1 = tridiag(w_i, -(w_i + e_i), e_i); H L1 is symmetric (h_i w_i = 2 / (h_i + h_{i-1}) =
// h_{i-1} e_{i-1}), so S = H^1/2 L1 H^-1/2 = U diag(lam) U^T and L1 = V diag(lam) V^-1 with
// V = H^-1/2 U, V^-1 = U^T H^1/2.  A side without a closure is singular (its null vector
// sqrt(h)); when both are, E's null-mode entry is 0, i.e. the solution with w.x = 0 (w the cell
// areas) of the system projected onto the range -- the LDS V-cycle's bordered last-level solve.
int direct_setup(ns_solver* s, const MgLevel& L) {
    const int nx = L.g.nx, ny = L.g.ny;
    const int n1p = (nx + 15) / 16 * 16, n2p = (ny + 15) / 16 * 16;
    std::vector<double> t(8 * (size_t)nx + 8 * (size_t)ny + 2);
    HIPCHK(hipMemcpy(t.data(), L.coef, t.size() * sizeof(double), hipMemcpyDeviceToHost));
    const nsg::Coef hc = coef_view(t.data(), nx, ny);
    auto decompose = [](int n, const double* w, const double* e, const std::vector<double>& h, std::vector<double>& lam,
                        std::vector<double>& U, bool& singular) {
        std::vector<double> S((size_t)n * n, 0.0);
        for (int i = 0; i < n; i++) {
            S[(size_t)i * n + i] = -(w[i] + e[i]);
            if (i > 0) S[(size_t)i * n + i - 1] = std::sqrt(h[i] / h[i - 1]) * w[i];
            if (i < n - 1) S[(size_t)i * n + i + 1] = std::sqrt(h[i] / h[i + 1]) * e[i];
        }
        for (int i = 0; i + 1 < n; i++) {   // (exactly symmetric: the mean of the two equal products)
            const double m = 0.5 * (S[(size_t)i * n + i + 1] + S[(size_t)(i + 1) * n + i]);
            S[(size_t)i * n + i + 1] = S[(size_t)(i + 1) * n + i] = m;
        }
        jacobi_eigen(n, S, lam, U);
        singular = w[0] == 0.0 && e[n - 1] == 0.0;   // walls on both ends: L1 1 = 0
        if (singular) {
            int k0 = 0;
            for (int k = 1; k < n; k++)
                if (std::fabs(lam[k]) < std::fabs(lam[k0])) k0 = k;
            lam[k0] = 0.0;
            return k0;
        }
        return -1;
    };
    std::vector<double> lx, ly, Ux, Uy;
    bool sx = false, sy = false;
    const int kx0 = decompose(nx, hc.pw, hc.pe, L.hx, lx, Ux, sx);
    const int ky0 = decompose(ny, hc.ps, hc.pn, L.hy, ly, Uy, sy);
    const size_t nP = (size_t)n1p * n1p, nQ = (size_t)n2p * n2p, nE = (size_t)n1p * n2p;
    std::vector<double> img(2 * nP + 2 * nQ + nE, 0.0);
    double *P1 = img.data(), *Q1 = P1 + nP, *E = Q1 + nQ, *P2 = E + nE, *Q2 = P2 + nP;
    for (int i = 0; i < nx; i++)
        for (int k = 0; k < nx; k++) {
            const double u = Ux[(size_t)i * nx + k], r = std::sqrt(L.hx[i]);
            P1[(size_t)k * n1p + i] = u * r;   // V^-1 = U^T H^1/2
            P2[(size_t)i * n1p + k] = u / r;   // V = H^-1/2 U
        }
    for (int j = 0; j < ny; j++)
        for (int m = 0; m < ny; m++) {
            const double u = Uy[(size_t)j * ny + m], r = std::sqrt(L.hy[j]);
            Q1[(size_t)j * n2p + m] = u * r;   // Vy^-T = H^1/2 U
            Q2[(size_t)m * n2p + j] = u / r;   // Vy^T = U^T H^-1/2
        }
    for (int k = 0; k < nx; k++)
        for (int m = 0; m < ny; m++) {
            const double d = lx[k] + ly[m];
            E[(size_t)k * n2p + m] = (sx && sy && k == kx0 && m == ky0) || d == 0.0 ? 0.0 : 1.0 / d;
        }
    HIPCHK(hipMalloc(&s->dmat, img.size() * sizeof(double)));
    HIPCHK(hipMemcpy(s->dmat, img.data(), img.size() * sizeof(double), hipMemcpyHostToDevice));
    s->dP1 = s->dmat;
    s->dQ1 = s->dP1 + nP;
    s->dE = s->dQ1 + nQ;
    s->dP2 = s->dE + nE;
    s->dQ2 = s->dP2 + nP;
    return 0;
}

// multigrid hierarchy: halve while every level stays even; stop at the first level small
// enough for the single-workgroup LDS coarse solve.  With nranks > 1 the first coarse level
// of <= agg_cells cells (NSGPU_AGG_CELLS, default 1024^2; 0 = never), or whose slabs would
// drop below 8 rows on some rank, is agglomerated: it and every coarser level live whole on
// every rank (the single-rank hierarchy from there down, LDS coarse solve included), so the
// latency-bound coarse levels cost no exchanges.  Every decision is made from all ranks'
// slab ranges, so every rank builds the same hierarchy.
int build_levels(ns_solver* s, const std::vector<double>& hx0, const std::vector<double>& hy0) {
    MgLevel L0;
    L0.g = s->g;
    L0.c = s->c;
    L0.hx = hx0;
    L0.hy = hy0;
    // the outflow preconditioner's closure: the side's boundary weight 2/h^2 toward its ghost (face Dirichlet)
    // (0 for a wall) in every level's tables; level 0 gets its own copy (the true operator's
    // tables stay as they are)
    auto close_side = [&](std::vector<double>& t, const std::vector<double>& hx) {
        const size_t nx = hx.size();
        if (s->out_side == 0) t[0] = 2.0 / (hx[0] * hx[0]);                        // pw[0]
        if (s->out_side == 1) t[nx + nx - 1] = 2.0 / (hx[nx - 1] * hx[nx - 1]);   // pe[nx-1]
    };
    if (s->out_side >= 0) {
        L0.g.dsx = s->out_side == 0 ? 1 : 2;   // inherited by every coarse level's Geo
        std::vector<double> t = coef_tables(hx0, hy0, s->g.neu);
        close_side(t, hx0);
        HIPCHK(hipMalloc(&L0.coef, t.size() * sizeof(double)));
        HIPCHK(hipMemcpy(L0.coef, t.data(), t.size() * sizeof(double), hipMemcpyHostToDevice));
        L0.c = coef_view(L0.coef, s->g.nx, s->g.ny);
    }
    std::vector<int> ri0(s->nranks), rn(s->nranks);
    for (int q = 0; q < s->nranks; q++) {
        int32_t a, b;
        ns_slab_range(s->g.nx, s->nranks, q, &a, &b);
        ri0[q] = a;
        rn[q] = b - a;
    }
    L0.minrows = *std::min_element(rn.begin(), rn.end());
    s->lv.push_back(L0);
    long agg_cells = 1024L * 1024L;
    if (const char* e = getenv("NSGPU_AGG_CELLS")) agg_cells = std::atol(e);
    const int agg_min_rows = 8;
    // stop at the first whole coarse level the exact separable solve takes (<= direct_cells, sides
    // <= 128: nsg::direct_fits), else (NSGPU_DIRECT_CELLS=0) at the first whose LDS V-cycle fits (<= ~64^2)
    const size_t lds_cap = 150 * 1024;
    auto direct_fits = [&](const nsg::Geo& g) {
        return s->direct_cells > 0 && (long)g.nx * g.ny <= s->direct_cells && nsg::direct_fits(g.nx, g.ny);
    };
    for (;;) {
        const MgLevel& F = s->lv.back();
        const nsg::Geo& gf = F.g;
        const bool whole = s->nranks == 1 || F.repl;
        if (whole && s->lv.size() > 1 && direct_fits(gf)) break;
        if (whole && s->lv.size() > 1 && nsg::coarse_vcycle_bytes(gf) <= lds_cap) break;
        if (!nsg::mg_can_coarsen(gf.nx, gf.ny)) break;
        nsg::Geo gc = gf;
        gc.fc = nullptr;   // coarse levels are whole boxes (a masked domain's fictitious-domain V-cycle)
        gc.et = nullptr;
        gc.nx /= 2; gc.ny /= 2;
        gc.ld = (gc.ny + 127) / 128 * 128;
        bool repl = F.repl;
        int minrows = gc.nx;
        if (whole) { gc.i0 = 0; gc.nxl = gc.nx; }
        else {
            bool even = true;
            for (int q = 0; q < s->nranks; q++) even = even && ri0[q] % 2 == 0 && rn[q] % 2 == 0;
            if (!even) break;   // a slab edge would split a coarse cell
            for (int q = 0; q < s->nranks; q++) { ri0[q] /= 2; rn[q] /= 2; }
            minrows = *std::min_element(rn.begin(), rn.end());
            gc.i0 /= 2; gc.nxl /= 2;
            repl = agg_cells > 0 && ((long)gc.nx * gc.ny <= agg_cells || minrows < agg_min_rows);
            if (!repl && minrows < 4) break;
        }
        MgLevel C;
        C.repl = repl && s->nranks > 1;
        if (C.repl && !F.repl) {
            C.gs = gc;
            C.si0 = ri0;
            C.sn = rn;
        }
        if (C.repl) { gc.i0 = 0; gc.nxl = gc.nx; minrows = gc.nx; }
        C.minrows = minrows;
        C.g = gc;
        C.hx.resize(gc.nx);
        C.hy.resize(gc.ny);
        for (int i = 0; i < gc.nx; i++) C.hx[i] = F.hx[2 * i] + F.hx[2 * i + 1];
        for (int j = 0; j < gc.ny; j++) C.hy[j] = F.hy[2 * j] + F.hy[2 * j + 1];
        std::vector<double> t = coef_tables(C.hx, C.hy);
        if (s->out_side >= 0) close_side(t, C.hx);
        HIPCHK(hipMalloc(&C.coef, t.size() * sizeof(double)));
        HIPCHK(hipMemcpy(C.coef, t.data(), t.size() * sizeof(double), hipMemcpyHostToDevice));
        C.c = coef_view(C.coef, gc.nx, gc.ny);
        const size_t plane = (size_t)(gc.nxl + 2 * nsg::HALO) * gc.ld;
        HIPCHK(hipMalloc(&C.mem, 3 * plane * sizeof(double)));
        HIPCHK(hipMemsetAsync(C.mem, 0, 3 * plane * sizeof(double), s->st));
        C.phi = C.mem + (size_t)nsg::HALO * gc.ld;
        C.tmp = C.phi + plane;
        C.b = C.tmp + plane;
        s->lv.push_back(C);
    }
    const MgLevel& last = s->lv.back();
    const nsg::Geo& gc = last.g;
    s->mg_direct = (s->nranks == 1 || last.repl) && s->lv.size() > 1 && direct_fits(gc);
    s->mg_coarse_lds = !s->mg_direct && (s->nranks == 1 || last.repl) && s->lv.size() > 1 &&
                       nsg::coarse_vcycle_bytes(gc) <= lds_cap;
    if (s->mg_direct) CHK(direct_setup(s, last));
    if (s->verbose && s->rank == 0) {
        for (size_t l = 0; l < s->lv.size(); l++)
            fprintf(stderr, "nsgpu mg level %zu: %d x %d%s, rows/rank >= %d, %s\n", l, s->lv[l].g.nx, s->lv[l].g.ny,
                    s->lv[l].repl ? " (replicated)" : "", s->lv[l].minrows,
                    pair_level(s, (int)l) ? "2-sweep passes" : (tile_level(s, (int)l) ? "LDS-tiled passes" : "single sweeps"));
        fprintf(stderr, "nsgpu mg coarse solve: %s\n",
                s->mg_direct ? "exact (separable eigen-decomposition)" : (s->mg_coarse_lds ? "LDS V-cycle" : "sweeps"));
    }
    // coarsest relaxation: on the last LDS level (<= 4x4 after the in-LDS coarsening) when the
    // LDS V-cycle is used, else on gc itself by (distributed) sweeps
    int ncx = gc.nx, ncy = gc.ny;
    if (s->mg_coarse_lds)
        while (nsg::mg_can_coarsen(ncx, ncy)) { ncx /= 2; ncy /= 2; }
    const int nc = std::max(ncx, ncy);
    const double pi = 3.14159265358979323846;
    s->mg_omega_c = 2.0 / (1.0 + std::sin(pi / nc));
    s->mg_coarse_iters = 2 * nc + 10;
    if (s->mg_coarse_lds) {
        std::vector<double> img;
        s->cv_n = nsg::cv_image(last.hx.data(), last.hy.data(), gc.nx, gc.ny, s->out_side == 0, s->out_side == 1, img,
                                &s->cv_dn);
        if (s->cv_n < 0) { set_err("coarse V-cycle: the last level's operator is singular"); return NS_EINVAL; }
        HIPCHK(hipMalloc(&s->cvimg, img.size() * sizeof(double)));
        HIPCHK(hipMemcpy(s->cvimg, img.data(), img.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    return 0;
}

// Poisson initial guess: the reference warm-starts from phi^{n-1} (KSPSetInitialGuessNonzero,
// FluidSolver.cpp:54); here from an extrapolation of the last solutions, which is O(dt^k) closer
// to phi^n (the converged answer is the same: both solve to rtol).  PHI (phi^{n-1}), the history
// planes phim, phim2, phim3 and TMP rotate: no copies.
//   linear 2 phi^{n-1} - phi^{n-2};  quadratic 3 phi^{n-1} - 3 phi^{n-2} + phi^{n-3};
//   cubic 4 phi^{n-1} - 6 phi^{n-2} + 4 phi^{n-3} - phi^{n-4}, while the last multigrid solve
//   needed more than one V-cycle (the start-up transient: 3.2 -> 2.9 V-cycles per step over steps
//   6-25 of the 4096^2 cavity); once one cycle suffices (developed flow) the quadratic guess does
//   as well and reads a plane less (both keep the four-plane history).
// The guess is formed by K5 in the same pass (r4, k_cell_s<6>: K5 reads phi^{n-1} anyway) into
// TMP; extrapolate_phi then only rotates the planes.  Elsewhere (masked / NEUMANN grids, the
// quartic A/B, NSGPU_K5_GUESS=0) extrapolate_phi runs k_axpby with the same arithmetic.
struct ExtrapPlan {
    int branch = 0;            // 0: none (phi^{n-1} is the guess: the first step copies it to phim),
                               // 1 linear, 2 quadratic, 3 cubic history, 4 quartic (A/B)
    double c[5] = {0, 0, 0, 0, 0};
    const double* h[4] = {nullptr, nullptr, nullptr, nullptr};
};
ExtrapPlan extrap_plan(const ns_solver* s, int cycles) {
    ExtrapPlan p;
    if (!s->phim || s->phim_valid == 0) return p;
    if (s->phi_extrap >= 4 && s->phim_valid >= 4) {
        p.branch = 4;
        const double c[5] = {5.0, -10.0, 10.0, -5.0, 1.0};
        std::copy(c, c + 5, p.c);
        p.h[0] = s->phim; p.h[1] = s->phim2; p.h[2] = s->phim3; p.h[3] = s->phim4;
    } else if (s->phi_extrap >= 3 && s->phim_valid >= 3) {
        p.branch = 3;
        p.h[0] = s->phim; p.h[1] = s->phim2;
        if (cycles >= 2) {
            p.c[0] = 4.0; p.c[1] = -6.0; p.c[2] = 4.0; p.c[3] = -1.0;
            p.h[2] = s->phim3;
        } else {
            p.c[0] = 3.0; p.c[1] = -3.0; p.c[2] = 1.0;
        }
    } else if (s->phi_extrap >= 2 && s->phim_valid >= 2) {
        p.branch = 2;
        p.c[0] = 3.0; p.c[1] = -3.0; p.c[2] = 1.0;
        p.h[0] = s->phim; p.h[1] = s->phim2;
    } else {
        p.branch = 1;
        p.c[0] = 2.0; p.c[1] = -1.0;
        p.h[0] = s->phim;
    }
    return p;
}

int extrapolate_phi(ns_solver* s) {
    if (!s->phim) return 0;
    const size_t back = (size_t)s->hp * s->g.ld;
    if (s->phim_valid == 0) {
        HIPCHK(hipMemcpyAsync(s->phim - back, s->arr[NS_ARR_PHI] - back, s->plane * sizeof(double),
                              hipMemcpyDeviceToDevice, s->st));
        s->phim_valid = 1;
        s->guess_ready = 0;
        return 0;
    }
    const ExtrapPlan p = extrap_plan(s, s->last_cycles);
    double* prev = s->arr[NS_ARR_PHI];
    s->gin_pending = false;
    if (s->guess_ready && s->guess_branch == p.branch) {
        // (K5 formed it: nothing to launch)
    } else if (p.branch >= 1 && p.branch <= 3 && gin_ok(s)) {
        // the solve's first restriction pass forms it from these planes (the rotation below does
        // not move their contents) and writes its output into TMP, which becomes PHI below
        s->gin_pending = true;
        s->gin_src[0] = prev;
        for (int k = 0; k < 3; k++) s->gin_src[k + 1] = p.h[k];
        for (int k = 0; k < 4; k++) s->gin_c[k] = p.c[k];
    } else {
        nsg::launch_axpby(s->g, p.c[0], prev, p.c[1], p.h[0], s->arr[NS_ARR_TMP], s->st, p.c[2], p.h[1], p.c[3], p.h[2],
                          p.c[4], p.h[3]);
    }
    s->guess_ready = 0;
    s->arr[NS_ARR_PHI] = s->arr[NS_ARR_TMP];
    switch (p.branch) {
    case 4:
        s->arr[NS_ARR_TMP] = s->phim4;
        s->phim4 = s->phim3;
        s->phim3 = s->phim2;
        s->phim2 = s->phim;
        break;
    case 3:
        if (s->phi_extrap >= 4) {
            s->arr[NS_ARR_TMP] = s->phim4;
            s->phim4 = s->phim3;
            s->phim_valid = 4;
        } else {
            s->arr[NS_ARR_TMP] = s->phim3;
        }
        s->phim3 = s->phim2;
        s->phim2 = s->phim;
        break;
    case 2:
        if (s->phi_extrap >= 3) {   // keep phi^{n-3} as the cubic's fourth point; the spare plane becomes scratch
            s->arr[NS_ARR_TMP] = s->phim3;
            s->phim3 = s->phim2;
            s->phim_valid = 3;
        } else {
            s->arr[NS_ARR_TMP] = s->phim2;
        }
        s->phim2 = s->phim;
        break;
    default:
        if (s->phi_extrap >= 2) {   // keep phi^{n-2} as the quadratic's third point
            s->arr[NS_ARR_TMP] = s->phim2;
            s->phim2 = s->phim;
            s->phim_valid = 2;
        } else {
            s->arr[NS_ARR_TMP] = s->phim;
        }
        break;
    }
    s->phim = prev;
    return 0;
}


// stretched grid without an outflow side: move rhs_phi onto the consistent system the oracle's
// PCG solves (k_area_fix); a no-op elsewhere (uniform grids: sum A b = A sum b = 0 already).
// The multigrid keeps subtracting the plain mean S_SHIFT (b' = b - shift is the consistent rhs);
// the Krylov solves project residuals onto mean-free vectors, so they subtract S_KSHIFT = shift +
// mean(b'), which leaves the same solution and a mean-free initial residual.
int consistent_rhs(ns_solver* s) {
    if (!s->consist) return 0;
    const int nb = nsg::launch_area_sum(s->g, s->c, s->arr[NS_ARR_RPHI], s->part, s->st);
    nsg::launch_reduce_sum(s->part, nb, 1, s->scal + S_AUX, s->st);
    CHK(allreduce(s, s->scal + S_AUX, 1, ncclSum));
    nsg::launch_area_fix(s->g, s->c, s->arr[NS_ARR_RPHI], s->scal + S_AUX, s->scal + S_SHIFT, s->area, s->inv_area,
                         s->ncells, s->scal + S_KSHIFT, s->st);
    return 0;
}

// whether the direct solve about to run (inside a step) checks its residual (pois_solve_fps)
bool fps_checks_next(const ns_solver* s) {
    return s->fps_strict || (s->fps_check > 0 && s->fps_solves % s->fps_check == 0);
}

// the (sum, sum^2) partials of rhs_phi -> the sums and the null-space shift (one rank: one launch)
int div_mean(ns_solver* s, int nb) {
    if (s->mean_pend) {   // (r5) the sums ride on the direct solve's forward allgather (fps_scan)
        nsg::launch_reduce_sum(s->part, nb, 2, s->fps_ragg + 2 * (size_t)s->g.ld, s->st);
        return 0;
    }
    if (!comm_on(s)) {
        nsg::launch_reduce_sum_mean(s->part, nb, s->scal + S_DIVSUM, s->ncells, s->scal + S_SHIFT, s->st);
        return 0;
    }
    nsg::launch_reduce_sum(s->part, nb, 2, s->scal + S_DIVSUM, s->st);
    CHK(allreduce(s, s->scal + S_DIVSUM, 2, ncclSum));
    nsg::launch_finish_mean(s->scal + S_DIVSUM, s->ncells, s->scal + S_SHIFT, s->st);
    return 0;
}

// K3 fused into the direct solve's DCT (launch_fps_div): the transformed plane (TMP) and the sums;
// rhs_phi itself only for a checked solve.  Slabs: the interior row pairs while the u*, v* ghost rows
// travel, then the two edge pairs (as overlapped() does for the strip kernels)
int divergence_fps(ns_solver* s) {
    const bool t = s->timing;
    if (t) {
        CHK(ensure_kev(s));
        CHK(t_begin(s, s->kev[2], s->kev[3]));
    }
    double* b = fps_checks_next(s) ? s->arr[NS_ARR_RPHI] : nullptr;
    auto launch = [&](int phase) {
        return nsg::launch_fps_div(s->g, s->c, s->dt, s->arr[NS_ARR_U], s->arr[NS_ARR_V], b, s->arr[NS_ARR_TMP],
                                   s->part, phase, s->fps_tw, s->fps_wk, s->st, s->fa.outE);
    };
    const HaloReq r[2] = {{&s->g, s->arr[NS_ARR_U], 1}, {&s->g, s->arr[NS_ARR_V], 1}};
    int nb;
    if (s->deep && s->u_ext >= 1 && s->in_step) {
        nb = launch(0);   // (r5, deep ghost rows: the residual pass computed u*, v*'s ghost row -- no exchange)
    } else if (!comm_on(s) || !s->overlap || !s->cst) {
        CHK(halo_reqs(s, r, 2, s->st));
        nb = launch(0);
    } else {
        HIPCHK(hipEventRecord(s->xev[0], s->st));
        if (launch(1) < 0) return NS_EINVAL;
        HIPCHK(hipStreamWaitEvent(s->cst, s->xev[0], 0));
        CHK(halo_reqs(s, r, 2, s->cst));
        HIPCHK(hipEventRecord(s->xev[1], s->cst));
        HIPCHK(hipStreamWaitEvent(s->st, s->xev[1], 0));
        nb = launch(2);   // (the partials are per row pair: the same sums as one launch)
    }
    if (nb < 0) {
        set_err("direct Poisson solve: ny = %d is not a supported power of two", s->g.ny);
        return NS_EINVAL;
    }
    if (t) CHK(t_end(s, s->kev[2], s->kev[3]));
    s->fps_pre = true;
    s->fps_pre_b = b != nullptr;
    s->mean_pend = s->fps_defer && s->fps_passes == 2;
    return div_mean(s, nb);
}

// K3 + null-space mean
// K3 with the u*, v* ghost rows, overlapped with the interior strips
int divergence(ns_solver* s) {
    if (s->fps && s->fps_fuse && s->in_step) return divergence_fps(s);
    s->fps_pre = false;
    const HaloReq r[2] = {{&s->g, s->arr[NS_ARR_U], 1}, {&s->g, s->arr[NS_ARR_V], 1}};
    auto launch = [&]() {
        return nsg::launch_div(s->g, s->c, s->dt, s->arr[NS_ARR_U], s->arr[NS_ARR_V], s->arr[NS_ARR_RPHI], s->part,
                               s->st);
    };
    // (r5, deep ghost rows: the residual pass computed u*, v*'s ghost row -- no exchange)
    const int nb = s->deep && s->u_ext >= 1 && s->in_step ? launch() : overlapped(s, r, 2, launch);
    if (nb < 0) return nb;
    return div_mean(s, nb);
}

// sums of an arbitrary RHS_phi -> null-space shift (standalone solves / sweep benchmark)
int rhs_mean(ns_solver* s) {
    const int nb = nsg::launch_sums(s->g, s->arr[NS_ARR_RPHI], s->part, s->st);
    nsg::launch_reduce_sum(s->part, nb, 2, s->scal + S_DIVSUM, s->st);
    CHK(allreduce(s, s->scal + S_DIVSUM, 2, ncclSum));
    nsg::launch_finish_mean(s->scal + S_DIVSUM, s->ncells, s->scal + S_SHIFT, s->st);
    return 0;
}

// ||RHS_u||^2, ||RHS_v||^2 of arbitrary RHS arrays (standalone Helmholtz solve)
int helm_bnorm(ns_solver* s) {
    int nb = nsg::launch_sums(s->g, s->arr[NS_ARR_RU], s->part, s->st);
    nsg::launch_reduce_sum(s->part, nb, 2, s->scal + S_AUX, s->st);
    nb = nsg::launch_sums(s->g, s->arr[NS_ARR_RV], s->part, s->st);
    nsg::launch_reduce_sum(s->part, nb, 2, s->scal + S_AUX + 2, s->st);
    CHK(allreduce(s, s->scal + S_AUX, 4, ncclSum));
    HIPCHK(hipMemcpyAsync(s->scal + S_HBN, s->scal + S_AUX + 1, sizeof(double), hipMemcpyDeviceToDevice, s->st));
    HIPCHK(hipMemcpyAsync(s->scal + S_HBN + 1, s->scal + S_AUX + 3, sizeof(double), hipMemcpyDeviceToDevice, s->st));
    return 0;
}

// K1 with its ghost rows (u, v width 2: MUSCL; phi width 1: grad phi^{n-1} on walls) in one
// exchange group, overlapped with the interior tiles
int rhs(ns_solver* s, bool defer_norm = false) {
    const bool t = s->timing && s->in_step;
    if (t) {
        CHK(ensure_kev(s));
        CHK(t_begin(s, s->kev[0], s->kev[1]));
    }
    int nb;
    if (s->deep && s->in_step) {
        // (r5) deep ghost rows: u, v (e + 2 rows: MUSCL), phi (e + 1: the wall terms' grad phi^{n-1}) and, when
        // not known valid, cu^{n-1}, cv^{n-1} (e) in ONE exchange, overlapped with the strips of the slab's own
        // interior; K1 then computes its rows and e of each neighbour's (their rhs and convective terms), its
        // ||RHS||^2 over its own rows
        const int e = s->deep_e, ld = s->g.ld;
        const HaloReq r[5] = {{&s->g, s->arr[NS_ARR_U], e + 2}, {&s->g, s->arr[NS_ARR_V], e + 2},
                              {&s->g, s->arr[NS_ARR_PHI], e + 1}, {&s->g, s->arr[NS_ARR_CU], e},
                              {&s->g, s->arr[NS_ARR_CV], e}};
        int lo = 0;
        const nsg::Geo gk = deep_geo(s, e, &lo);
        nb = overlapped(s, r, s->cu_ext >= e ? 3 : 5, [&]() {
            return nsg::launch_rhs(gk, s->c, s->dt, s->re, shp(s->arr[NS_ARR_U], lo, ld), shp(s->arr[NS_ARR_V], lo, ld),
                                   shp(s->arr[NS_ARR_PHI], lo, ld), shp(s->arr[NS_ARR_CU], lo, ld),
                                   shp(s->arr[NS_ARR_CV], lo, ld), shp(s->arr[NS_ARR_RU], lo, ld),
                                   shp(s->arr[NS_ARR_RV], lo, ld), s->part, s->st, e + 2);
        });
        s->cu_ext = e;
        s->u_ext = e + 2;
    } else if (s->corr_pend && s->in_step) {
        // (r6) the previous step's CorrectVelocities folded in: U, V hold u*, v*, PHI phi^n; the corrected u, v go to
        // the ping-pong partners (swapped below) and their min / max -- the previous step's monitor -- to S_MM
        double* mm = s->part + 4 * (size_t)nsg::max_partials(s->g);
        nb = nsg::launch_rhs(s->g, s->c, s->dt, s->re, s->arr[NS_ARR_U], s->arr[NS_ARR_V], s->arr[NS_ARR_PHI],
                             s->arr[NS_ARR_CU], s->arr[NS_ARR_CV], s->arr[NS_ARR_RU], s->arr[NS_ARR_RV], s->part, s->st,
                             2, s->arr[NS_ARR_TMPU], s->arr[NS_ARR_TMPV], mm);
        if (nb < 0) { set_err("K1 with the deferred correction: launch refused"); return NS_EHIP; }
        std::swap(s->arr[NS_ARR_U], s->arr[NS_ARR_TMPU]);
        std::swap(s->arr[NS_ARR_V], s->arr[NS_ARR_TMPV]);
        s->corr_pend = 0;
        s->corr_k1 = 1;
        s->cu_ext = 0;
        if (nb < 0) return nb;
        if (t) CHK(t_end(s, s->kev[0], s->kev[1]));
        // (the min / max and ||RHS||^2 partials in one launch; one rank: no bus, no all-reduce)
        nsg::launch_reduce_sum_min(s->part, nb, 2, s->scal + S_HBN, mm, nb, 4, s->scal + S_MM, s->st);
        return 0;
    } else {
        const HaloReq r[3] = {{&s->g, s->arr[NS_ARR_U], 2}, {&s->g, s->arr[NS_ARR_V], 2}, {&s->g, s->arr[NS_ARR_PHI], 1}};
        nb = overlapped(s, r, 3, [&]() {
            return nsg::launch_rhs(s->g, s->c, s->dt, s->re, s->arr[NS_ARR_U], s->arr[NS_ARR_V], s->arr[NS_ARR_PHI],
                                   s->arr[NS_ARR_CU], s->arr[NS_ARR_CV], s->arr[NS_ARR_RU], s->arr[NS_ARR_RV], s->part,
                                   s->st);
        });
        s->cu_ext = 0;
    }
    if (nb < 0) return nb;
    if (t) CHK(t_end(s, s->kev[0], s->kev[1]));
    // (r5, the bus: the rank's norms wait in S_HBNL for the Helmholtz check's allgather)
    const bool ub = defer_norm && bus_on(s);
    nsg::launch_reduce_sum(s->part, nb, 2, s->scal + (ub ? S_HBNL : S_HBN), s->st);
    // (slabs, rectangle: the norms ride on the Helmholtz solve's first residual all-reduce --
    // S_HBN and S_RES are adjacent -- one collective less per step)
    if (ub) {
    } else if (defer_norm && comm_on(s) && !s->g.fc) s->hbn_pend = true;
    else CHK(allreduce(s, s->scal + S_HBN, 2, ncclSum));
    return 0;
}

// u^{n+1} = u* - dt grad phi into the ping-pong partners (no in-place read/write hazard)
// (K5 with phi's ghost rows, overlapped with the interior strips)
// K5 into the ping-pong partners (TMPU, TMPV) and its min/max into scal[S_MM]; `part2`: the
// partial slots (the second half of s->part when speculating: the first half still holds
// the residual partials the check is reducing)
int correct_launch(ns_solver* s, double* part2) {
    const HaloReq r[1] = {{&s->g, s->arr[NS_ARR_PHI], 1}};
    // inside a step: the next step's Poisson guess in the same pass (k_cell_s<6>) into TMP, which the
    // finished solve leaves free (a speculative K5 whose check fails is re-run after the last cycle,
    // with that solve's cycle count: the guess is formed again)
    const ExtrapPlan p = extrap_plan(s, s->cur_cycles);
    const bool guess = s->in_step && s->k5_guess && p.branch >= 1 && p.branch <= 3 && nsg::correct_streams(s->g);
    s->guess_ready = 0;
    // (r5, deep slabs: the direct solve wrote phi's ghost rows -- no exchange)
    const bool have = s->deep && s->phi_ext && s->in_step;
    const bool t5 = s->timing && s->in_step && !guess;   // (r6: the bench's K5 line; read at the next host sync)
    if (t5) {
        CHK(ensure_kev(s));
        CHK(t_begin(s, s->kev[12], s->kev[13]));
    }
    const int nb = have ? [&]() {
        if (guess)
            return nsg::launch_correct_guess(s->g, s->c, s->dt, s->arr[NS_ARR_U], s->arr[NS_ARR_V], s->arr[NS_ARR_TMPU],
                                             s->arr[NS_ARR_TMPV], s->arr[NS_ARR_PHI], part2, p.h[0], p.h[1], p.h[2], p.c,
                                             s->arr[NS_ARR_TMP], s->st);
        return nsg::launch_correct(s->g, s->c, s->dt, s->arr[NS_ARR_U], s->arr[NS_ARR_V], s->arr[NS_ARR_TMPU],
                                   s->arr[NS_ARR_TMPV], s->arr[NS_ARR_PHI], part2, s->st);
    }() : overlapped(s, r, 1, [&]() {
        if (guess)
            return nsg::launch_correct_guess(s->g, s->c, s->dt, s->arr[NS_ARR_U], s->arr[NS_ARR_V], s->arr[NS_ARR_TMPU],
                                             s->arr[NS_ARR_TMPV], s->arr[NS_ARR_PHI], part2, p.h[0], p.h[1], p.h[2], p.c,
                                             s->arr[NS_ARR_TMP], s->st);
        return nsg::launch_correct(s->g, s->c, s->dt, s->arr[NS_ARR_U], s->arr[NS_ARR_V], s->arr[NS_ARR_TMPU],
                                   s->arr[NS_ARR_TMPV], s->arr[NS_ARR_PHI], part2, s->st);
    });
    if (t5 && nb >= 0) {
        CHK(t_end(s, s->kev[12], s->kev[13]));
        s->k5_pend = 1;
    }
    if (guess && nb >= 0) {
        s->guess_ready = 1;
        s->guess_branch = p.branch;
    }
    if (nb < 0) return nb;
    // (r5, the bus: the rank's min / max wait in S_MML for the next collective that carries them --
    // the next step's Helmholtz check, ns_step's closing bus or ns_monitor's)
    const bool ub = bus_on(s);
    nsg::launch_reduce_min(part2, nb, 4, s->scal + (ub ? S_MML : S_MM), s->st);
    if (!ub) CHK(allreduce(s, s->scal + S_MM, 4, ncclMin));
    return 0;
}

int correct(ns_solver* s) {
    if (s->defer_now && s->in_step) {   // (r6: the next step's K1 applies it -- or materialize())
        s->corr_pend = 1;
        s->u_ext = 0;
        return 0;
    }
    if (!s->k5_spec) CHK(correct_launch(s, s->part));
    s->k5_spec = 0;
    std::swap(s->arr[NS_ARR_U], s->arr[NS_ARR_TMPU]);
    std::swap(s->arr[NS_ARR_V], s->arr[NS_ARR_TMPV]);
    s->u_ext = 0;   // (the corrected u, v: the slab's own rows)
    return 0;
}

// (r6) a deferred correction applied now (K5 as in a synchronous step): before any entry point that reads or writes
// the fields, the monitor, or runs kernels on them
int materialize(ns_solver* s) {
    if (!s->corr_pend) return 0;
    s->corr_pend = 0;
    HIPCHK(hipSetDevice(s->device));
    return correct(s);
}

int check_arr(ns_solver* s, int which) {
    if (!s) { set_err("null solver"); return NS_EINVAL; }
    if (which < 0 || which >= NS_NUM_ARR) { set_err("bad array index %d", which); return NS_EINVAL; }
    return 0;
}

}  // namespace

extern "C" {

const char* ns_last_error(void) { return g_err.c_str(); }
int ns_abi_version(void) { return NSGPU_ABI_VERSION; }

int ns_slab_range(int32_t nx, int32_t nranks, int32_t rank, int32_t* i0, int32_t* i1) {
    if (nx <= 0 || nranks <= 0 || rank < 0 || rank >= nranks) { set_err("bad slab arguments"); return NS_EINVAL; }
    // balanced in units of U = 2^k rows (k <= 4, U | nx, at least 8 units per rank so the
    // imbalance stays <= 1/8): a slab edge then never splits a coarse cell of the first k
    // multigrid coarsenings (16384^2 -> 1024^2, where the hierarchy is replicated), whatever
    // the rank count (4096^2 on 3 ranks: 1376 / 1360 / 1360 rows instead of 1366 / 1365 /
    // 1365, whose odd edges stopped the hierarchy at one level)
    int k = 0;
    while (k < 4 && nx % (2 << k) == 0 && (nx >> (k + 1)) >= 8 * nranks) k++;
    const int units = nx >> k;
    if (units < nranks) { set_err("%d rows cannot be split over %d ranks", nx, nranks); return NS_EINVAL; }
    const int base = units / nranks, rem = units % nranks;
    const int a = rank * base + std::min(rank, rem);
    *i0 = a << k;
    *i1 = (a + base + (rank < rem ? 1 : 0)) << k;
    return 0;
}

int ns_nccl_id_size(void) { return (int)sizeof(ncclUniqueId); }

int ns_nccl_get_id(void* out) {
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    std::memcpy(out, &id, sizeof id);
    return 0;
}

int64_t ns_device_bytes(int32_t nxl, int32_t ny) {
    const int64_t ld = ((int64_t)ny + 127) / 128 * 128;
    return (int64_t)NS_NUM_ARR * (nxl + 2 * nsg::HALO) * ld * 8;
}

int ns_create(const ns_grid_desc* gd, const ns_params* p, ns_solver** out) {
    if (!gd || !p || !out) { set_err("null argument"); return NS_EINVAL; }
    *out = nullptr;
    const bool masked = gd->cell_id != nullptr;
    if (masked && !gd->face_edge) { set_err("a cell_id mask needs face_edge (the cells' boundary edges, Grid.h:33)"); return NS_EINVAL; }
    if (gd->nx < 2 || gd->ny < 2) { set_err("one-cell-thick geometry is not supported (FluidSolver.cpp:470-477)"); return NS_EINVAL; }
    if (!gd->hx || !gd->hy) { set_err("hx/hy missing"); return NS_EINVAL; }
    if (!(p->dt > 0)) { set_err("Time step should be positive"); return NS_EINVAL; }
    if (!(p->re > 0)) { set_err("Reynolds number should be positive"); return NS_EINVAL; }
    if (p->nranks < 1 || p->rank < 0 || p->rank >= p->nranks) { set_err("bad rank/nranks"); return NS_EINVAL; }
    const char* lbe = getenv("NSGPU_RCCL_LOOPBACK");
    const bool has_ht = p->host_transport && p->host_transport->exchange && p->host_transport->allreduce;
    const bool loopback = lbe && std::atoi(lbe) != 0 && (p->nranks == 1 || (!p->nccl_id && !has_ht));
    if (p->nranks > 1 && !p->nccl_id && !has_ht && !loopback) {
        set_err("nranks > 1 needs an ncclUniqueId or a host transport");
        return NS_EINVAL;
    }
    if (p->poisson != NS_POISSON_RBSOR && p->poisson != NS_POISSON_JACOBI && p->poisson != NS_POISSON_MG) {
        set_err("unknown Poisson solver %d (NS_POISSON_MG 0, NS_POISSON_JACOBI 1, NS_POISSON_RBSOR 3; ABI %d)",
                p->poisson, NSGPU_ABI_VERSION);
        return NS_EINVAL;
    }

    nsg::Geo g{};
    g.nx = gd->nx;
    g.ny = gd->ny;
    g.ld = (gd->ny + 127) / 128 * 128;
    int32_t i0, i1;
    if (ns_slab_range(gd->nx, p->nranks, p->rank, &i0, &i1)) return NS_EINVAL;
    g.i0 = i0;
    g.nxl = i1 - i0;
    // (the widest exchange outside the 3-sweep passes -- which need slabs of 2*HALO rows, `triple`
    // -- is 6 rows, fed from one neighbour; the overlapped passes want an interior beyond it)
    constexpr int min_slab_rows = 10;
    if (p->nranks > 1 && g.nxl < min_slab_rows) {
        set_err("slab of %d rows is thinner than the %d-row halo exchange", g.nxl, min_slab_rows);
        return NS_EINVAL;
    }
    // ConstructGhostStencils (FluidSolver.cpp:84-103) of one edge
    auto edge_dev = [&](int e, nsg::EdgeDev* D) -> int {
        const ns_edge& E = gd->edges[e];
        *D = nsg::EdgeDev{0, E.nx, E.ny, 0.0, 0.0};
        if (E.type == NS_BC_INLET_UNI) {
            if (E.nx == 0) D->c1 = 2 * E.info; else D->c0 = 2 * E.info;
        } else if (E.type == NS_BC_WALL) {
            if (E.nx != 0) D->c1 = 2 * E.info; else D->c0 = 2 * E.info;
        } else if (E.type == NS_BC_NEUMANN) {
            // outflow: velocity ghost q, phi ghost 2.5 phi_0 - 2 phi_1 + 0.5 phi_2 (:98-101);
            // the Poisson solve becomes BiCGStab on the true matrix (pois_solve_any)
            D->neu = 1;
            if (!masked && p->poisson != NS_POISSON_MG) {
                set_err("NEUMANN outflow edges need the multigrid-preconditioned Krylov Poisson solve "
                        "(NS_POISSON_MG): the RB-SOR / Jacobi sweeps cannot relax the outflow rows");
                return NS_EINVAL;
            }
        } else {
            set_err("edge %d: boundary condition type %d is not supported (INLET_PARABOLIC / PRESSURE / unset "
                    "have no ghost stencil in the reference)", e, E.type);
            return NS_EINVAL;
        }
        return 0;
    };
    std::vector<nsg::EdgeDev> etab(nsg::MAX_EDGES + 1, nsg::EdgeDev{0, 0, 0, 0.0, 0.0});  // [31]: interior faces
    if (masked) {
        if (gd->n_edges > nsg::MAX_EDGES) { set_err("more than %d polygon edges", nsg::MAX_EDGES); return NS_EINVAL; }
        for (int e = 0; e < gd->n_edges; e++)
            if (int rc = edge_dev(e, &etab[e])) return rc;
    } else {
        // sides from edge normals (a rectangle: Grid.cpp:35-63 gives one edge per side)
        const int snx[4] = {-1, 1, 0, 0}, sny[4] = {0, 0, -1, 1};
        int side_edge[4] = {-1, -1, -1, -1};
        for (int e = 0; e < gd->n_edges; e++) {
            const ns_edge& E = gd->edges[e];
            for (int k = 0; k < 4; k++)
                if (E.nx == snx[k] && E.ny == sny[k]) {
                    if (side_edge[k] >= 0) { set_err("side %d has more than one edge: not a rectangle (pass cell_id / face_edge)", k); return NS_EINVAL; }
                    side_edge[k] = e;
                }
        }
        for (int k = 0; k < 4; k++) {
            if (side_edge[k] < 0) { set_err("side %d has no edge: not a rectangle", k); return NS_EINVAL; }
            nsg::EdgeDev D;
            if (int rc = edge_dev(side_edge[k], &D)) return rc;
            g.enx[k] = D.enx;
            g.eny[k] = D.eny;
            g.c0[k] = D.c0;
            g.c1[k] = D.c1;
            g.neu[k] = D.neu;
            if (D.neu && (k < 2 ? gd->nx : gd->ny) < 3) {
                set_err("a NEUMANN side needs >= 3 cells along its normal (its phi ghost reaches 2 inward)");
                return NS_EINVAL;
            }
        }
    }

    // masked domain: the topology plane (this slab's rows and HALO ghost rows on each side)
    // and the global in-domain cell count
    std::vector<int32_t> fch;
    long nin = (long)gd->nx * gd->ny;
    if (masked) {
        const int nx = gd->nx, ny = gd->ny;
        auto inside = [&](int i, int j) { return i >= 0 && i < nx && j >= 0 && j < ny && gd->cell_id[(size_t)i * ny + j] >= 0; };
        nin = 0;
        for (size_t c = 0; c < (size_t)nx * ny; c++) nin += gd->cell_id[c] >= 0;
        if (nin == 0) { set_err("the cell_id mask holds no cell"); return NS_EINVAL; }
        fch.assign((size_t)(g.nxl + 2 * nsg::HALO) * g.ld, 0);
        const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
        for (int li = -nsg::HALO; li < g.nxl + nsg::HALO; li++) {
            const int i = g.i0 + li;
            if (i < 0 || i >= nx) continue;
            for (int j = 0; j < ny; j++) {
                if (!inside(i, j)) continue;
                int code = nsg::FC_IN;
                for (int k = 0; k < 4; k++) {
                    const int t = gd->face_edge[((size_t)i * ny + j) * 4 + k];
                    const bool nb = inside(i + di[k], j + dj[k]);
                    // Grid::inDomain and Cell::edges must agree (the reference mixes both tests)
                    if (nb == (t >= 0) || t >= gd->n_edges) {
                        set_err("cell (%d,%d) face %d: edge tag %d disagrees with the domain mask", i, j, k, t);
                        return NS_EINVAL;
                    }
                    code |= (nb ? nsg::FC_INT : t) << (5 * k);
                    if (!nb && etab[t].neu) {   // the outflow phi ghost's two inward cells
                        const int a1 = i - etab[t].enx, b1 = j - etab[t].eny;
                        if (!inside(a1, b1) || !inside(a1 - etab[t].enx, b1 - etab[t].eny)) {
                            set_err("cell (%d,%d): a NEUMANN face needs two cells inward (FluidSolver.cpp:100)", i, j);
                            return NS_EINVAL;
                        }
                    }
                }
                if (inside(i - 1, j) && inside(i - 2, j) && inside(i + 1, j) && inside(i + 2, j) && inside(i, j - 1) &&
                    inside(i, j - 2) && inside(i, j + 1) && inside(i, j + 2))
                    code |= nsg::FC_DEEP;
                fch[(size_t)(li + nsg::HALO) * g.ld + j] = code;
            }
        }
    }

    // (r6) the masked domain's wall bands (one rank): FC_BAND on the cells within mbw of a boundary face along
    // their row or column (on a rectangle exactly the box bands of helm_band), and the mt kernel's tiles holding one
    std::vector<int32_t> mband;
    if (masked && g.nxl == gd->nx) {
        const int nx = gd->nx, ny = gd->ny, ldh = g.ld;
        int mbw = std::min(nx, ny) > 4096 ? 3 * std::min(nx, ny) / 64 : std::max(32, std::min(nx, ny) / 32);
        if (const char* e = getenv("NSGPU_MASK_BAND_W")) mbw = std::max(1, std::atoi(e));   // (A/B)
        auto code_at = [&](int i, int j) -> int32_t& { return fch[(size_t)(i + nsg::HALO) * ldh + j]; };
        auto bnd = [&](int i, int j) {   // a domain cell with a face that is not interior
            const int32_t c = code_at(i, j);
            if (!(c & nsg::FC_IN)) return false;
            for (int k = 0; k < 4; k++)
                if (nsg::fc_edge(c, k) != nsg::FC_INT) return true;
            return false;
        };
        const int BIG = 1 << 29;
        std::vector<int> dr((size_t)nx * ny, BIG);   // distance along the row / column to a boundary cell
        for (int i = 0; i < nx; i++) {
            int last = -BIG;
            for (int j = 0; j < ny; j++) { if (bnd(i, j)) last = j; dr[(size_t)i * ny + j] = j - last; }
            last = BIG;
            for (int j = ny - 1; j >= 0; j--) {
                if (bnd(i, j)) last = j;
                dr[(size_t)i * ny + j] = std::min(dr[(size_t)i * ny + j], last - j);
            }
        }
        for (int j = 0; j < ny; j++) {
            int last = -BIG;
            for (int i = 0; i < nx; i++) {
                if (bnd(i, j)) last = i;
                dr[(size_t)i * ny + j] = std::min(dr[(size_t)i * ny + j], i - last);
            }
            last = BIG;
            for (int i = nx - 1; i >= 0; i--) {
                if (bnd(i, j)) last = i;
                dr[(size_t)i * ny + j] = std::min(dr[(size_t)i * ny + j], last - i);
            }
        }
        const int nti = (nx + nsg::MT_TI - 1) / nsg::MT_TI, ntj = (ny + nsg::MT_TJ - 1) / nsg::MT_TJ;
        std::vector<char> tb((size_t)nti * ntj, 0);
        for (int i = 0; i < nx; i++)
            for (int j = 0; j < ny; j++)
                if ((code_at(i, j) & nsg::FC_IN) && dr[(size_t)i * ny + j] < mbw) {
                    code_at(i, j) |= nsg::FC_BAND;
                    tb[(size_t)(i / nsg::MT_TI) * ntj + j / nsg::MT_TJ] = 1;
                }
        for (int a = 0; a < nti; a++)
            for (int b = 0; b < ntj; b++)
                if (tb[(size_t)a * ntj + b]) { mband.push_back(a * nsg::MT_TI); mband.push_back(b * nsg::MT_TJ); }
    }

    ns_solver* s = new ns_solver();
    s->g = g;
    if (masked) {
        // compact ids of this slab (i outer, j inner: ids increase along the slab's rows)
        const int32_t* c = gd->cell_id + (size_t)g.i0 * gd->ny;
        const size_t n = (size_t)g.nxl * gd->ny;
        s->cid.assign(c, c + n);
        int64_t lo = -1, cnt = 0;
        for (size_t k = 0; k < n; k++)
            if (c[k] >= 0) {
                if (lo < 0) lo = c[k];
                cnt++;
            }
        s->cid0 = lo < 0 ? 0 : lo;
        s->ncid = cnt;
        for (size_t k = 0; k < n; k++) {
            if (c[k] < 0) continue;
            const int64_t r = c[k] - s->cid0;
            if (r < 0 || r >= cnt) {
                set_err("cell_id is not the compact i-outer / j-inner numbering of Grid.cpp:149-162 (id %d)", c[k]);
                delete s;
                return NS_EINVAL;
            }
            s->cid[k] = (int32_t)r;
        }
    }
    s->dt = p->dt;
    s->re = p->re;
    s->rtol = p->rtol > 0 ? p->rtol : 1e-8;
    s->poisson = p->poisson;
    s->max_iters = p->max_iters > 0 ? p->max_iters : 200000;
    const int nmax = std::max(gd->nx, gd->ny);
    const double pi = 3.14159265358979323846;
    s->omega = p->omega > 0 ? p->omega
                            : (p->poisson != NS_POISSON_JACOBI ? 2.0 / (1.0 + std::sin(pi / nmax)) : 0.9);
    {
        // Helmholtz SOR weight: (I - a L_V) has Jacobi spectral radius
        // rho = 2a(1/hx^2 + 1/hy^2) / (1 + 2a(1/hx^2 + 1/hy^2) + ...) <= that ratio on the finest spacing;
        // optimal SOR omega = 2 / (1 + sqrt(1 - rho^2))
        const double a = p->dt / (2 * p->re);
        const double hxm = *std::min_element(gd->hx, gd->hx + gd->nx), hym = *std::min_element(gd->hy, gd->hy + gd->ny);
        const double t = 2 * a * (1 / (hxm * hxm) + 1 / (hym * hym));
        const double rho = t / (1 + t);
        s->omega_v = p->omega_v > 0 ? p->omega_v : 2.0 / (1.0 + std::sqrt(1.0 - rho * rho));
    }
    s->check_every = p->check_every;
    if (p->check_every > 0) s->pois_batch0 = s->helm_batch0 = p->check_every;
    s->helm_next = s->helm_batch0;
    s->helm_adapt = p->check_every <= 0;
    s->timing = p->timing;
    if (const char* e = getenv("NSGPU_SWEEP")) s->tiled = std::strcmp(e, "tiled") == 0;
    if (const char* e = getenv("NSGPU_SWEEP3")) s->sweep3 = std::atoi(e) != 0;   // A/B: pairs only
    if (const char* e = getenv("NSGPU_HELM_BAND")) s->helm_band = std::atoi(e) != 0;   // A/B: no wall bands
    // the walls' boundary layers span a fixed fraction of the grid: 1/32 of the shorter side (128
    // at 4096^2; 8192^2 with 128 needed 8.5 global sweeps per step, with 256: 4.5 -- 7173 -> 8057
    // MLUPS), at least 32
    s->band_w = std::max(32, std::min(s->g.nx, s->g.ny) / 32);
    // (r5) the Helmholtz operator loses diagonal dominance as the grid grows (alpha / h^2 = n / (16 Re) at
    // dt = h / 8: Jacobi radius 0.51 at 4096^2, 0.67 at 8192^2), so the band needs more sweeps there:
    // 8192^2 with 6 sweeps in 256-wide bands took 4.5 global sweeps per step (4.55 ms), with 9 in 384-wide
    // bands 3.0 (4.47 ms; 9 in 256: 5.8, 6 in 384 / 512: 4.5; profiles/r05/bands_8192.log)
    // (16384^2: 12 sweeps in 768-wide bands 3.0 global sweeps, 31.9 ms per step; 9 in 768: 5.0, 34.1 ms;
    // profiles/r05/bands_16384.log)
    if (std::min(s->g.nx, s->g.ny) > 4096) {
        s->band_sweeps = std::min(s->g.nx, s->g.ny) > 8192 ? 12 : 9;
        s->band_w = 3 * std::min(s->g.nx, s->g.ny) / 64;
    }
    if (const char* e = getenv("NSGPU_BAND_W")) s->band_w = std::max(1, std::atoi(e));   // A/B: band width
    if (const char* e = getenv("NSGPU_BAND_SWEEPS")) s->band_sweeps = std::max(3, std::atoi(e) / 3 * 3);
    if (const char* e = getenv("NSGPU_BAND6")) s->band6 = std::atoi(e) != 0;
    if (const char* e = getenv("NSGPU_SWEEP3_RES")) s->sweep3_res = std::atoi(e) != 0;   // A/B: batches end on pairs
    if (const char* e = getenv("NSGPU_HELM_UV")) s->helm_uv = std::atoi(e);
    // the 3-sweep pass reads HALO ghost rows, which one neighbour feeds only from slabs of
    // >= 2*HALO rows; thinner slabs (the thinnest of all ranks: a global decision) take the
    // same sweeps as a single sweep + pairs
    for (int q = 0; q < s->nranks && s->nranks > 1; q++) {
        int32_t a0, a1;
        ns_slab_range(s->g.nx, s->nranks, q, &a0, &a1);
        if (a1 - a0 < 2 * nsg::HALO) s->triple = false;
    }
    if (const char* e = getenv("NSGPU_FUSED_RESTRICT")) s->fuse_restrict = std::atoi(e) != 0;
    if (const char* e = getenv("NSGPU_FUSED_PROLONG")) s->fuse_prolong = std::atoi(e) != 0;
    if (const char* e = getenv("NSGPU_TILE_SMALL")) s->tile_small = std::atoi(e) != 0;
    if (const char* e = getenv("NSGPU_EXT_TIMING")) s->ext_timing = std::atoi(e) != 0;
    if (const char* e = getenv("NSGPU_PHI_EXTRAP")) s->phi_extrap = std::max(0, std::min(4, std::atoi(e)));
    if (const char* e = getenv("NSGPU_MG_PREDICT")) s->mg_predict = std::atoi(e) != 0;
    if (const char* e = getenv("NSGPU_SPECULATE")) s->speculate = std::atoi(e) != 0;
    if (const char* e = getenv("NSGPU_K5_GUESS")) s->k5_guess = std::atoi(e) != 0;
    if (const char* e = getenv("NSGPU_FUSE4")) s->fuse4 = std::atoi(e) != 0;
    if (const char* e = getenv("NSGPU_GIN")) s->gin = std::atoi(e) != 0;
    if (const char* e = getenv("NSGPU_VERBOSE")) s->verbose = std::atoi(e) != 0;
    if (const char* e = getenv("NSGPU_MASK_HELM")) s->mask_rb = std::strcmp(e, "krylov") != 0;
    if (const char* e = getenv("NSGPU_MASK_RBT")) s->mask_rbt = std::atoi(e) != 0;
    if (const char* e = getenv("NSGPU_MASK_MT")) s->mask_mt = std::atoi(e) != 0;
    if (const char* e = getenv("NSGPU_MASK_BAND")) s->mask_band = std::max(0, std::atoi(e) / 6 * 6);
    if (const char* e = getenv("NSGPU_PAIR_MIN_CELLS")) s->pair_min_cells = std::atol(e);
    if (const char* e = getenv("NSGPU_DIRECT_CELLS")) s->direct_cells = std::max(0L, std::atol(e));
    {
        const char* e = getenv("NSGPU_STRIP_ROWS");  // tuning override; unset = adaptive
        nsg::set_strip_rows(e ? atoi(e) : 0);
    }
    s->rank = p->rank;
    s->nranks = p->nranks;
    s->ncells = (double)nin;
    {
        // a stretched grid (Grid.cpp ratio > 0) with no outflow edge needs the consistent rhs
        bool stretched = false, outflow = false;
        for (int i = 1; i < gd->nx; i++) stretched |= std::fabs(gd->hx[i] - gd->hx[0]) > 1e-12 * gd->hx[0];
        for (int j = 1; j < gd->ny; j++) stretched |= std::fabs(gd->hy[j] - gd->hy[0]) > 1e-12 * gd->hy[0];
        for (int e = 0; e < gd->n_edges; e++) outflow |= gd->edges[e].type == NS_BC_NEUMANN;
        s->consist = stretched && !outflow;
        double a = 0.0, ia = 0.0;
        for (int i = 0; i < gd->nx; i++)
            for (int j = 0; j < gd->ny; j++)
                if (!masked || gd->cell_id[(size_t)i * gd->ny + j] >= 0) {
                    a += gd->hx[i] * gd->hy[j];
                    ia += 1.0 / (gd->hx[i] * gd->hy[j]);
                }
        s->area = a;
        s->inv_area = ia;
        // the direct Poisson solve: a rectangle without an outflow side, uniform hy (the DCT's premise), ny a power
        // of two.  (r6) hx may be stretched (Grid.cpp:87-92): Lx's per-row coefficients enter Thomas' recurrences
        // as they are (ns_fps.hip piv_next), and consistent_rhs makes b - plain mean area-consistent first (mode
        // 0's singular system along x); the fused K3 form (uniform face weights) and the pivot fixed points
        // (uniform interior rows) stay off there
        bool yuni = true, xuni = true;
        for (int j = 1; j < gd->ny; j++) yuni &= gd->hy[j] == gd->hy[0];
        for (int i = 1; i < gd->nx; i++) xuni &= gd->hx[i] == gd->hx[0];
        const char* fe = getenv("NSGPU_FPS");
        // (r5) or a rectangle whose only NEUMANN side is E, on one rank with nx even (the outflow row is
        // the second row of the last row pair, the elimination of ns_fps.hip's piv_next): the channel
        const int nneu_r = masked ? 0 : g.neu[0] + g.neu[1] + g.neu[2] + g.neu[3];
        const char* foe = getenv("NSGPU_FPS_OUTFLOW");
        // (r6) on slabs too: the outflow row pair is the last rank's last local pair (its row count even, >= 4), the
        // mode-0 shift reaches the other ranks by one scalar all-reduce (pois_solve_fps)
        int32_t lq0 = 0, lq1 = gd->nx;
        if (p->nranks > 1) ns_slab_range(gd->nx, p->nranks, p->nranks - 1, &lq0, &lq1);
        const bool out_ok = nneu_r == 1 && g.neu[1] && gd->nx % 2 == 0 && gd->nx >= 4 && (lq1 - lq0) % 2 == 0 &&
                            lq1 - lq0 >= 4 && !(foe && std::atoi(foe) == 0) && xuni;   // (the elimination: uniform hx)
        // (r6) the transforms along y: the FFT (hy uniform, ny a power of two or of 2, 3, 5, 7) or the dense
        // eigenvector transforms (hy stretched, Grid.cpp:87-92, or another ny <= 4096; walls / inlets only)
        const bool fft = yuni && (nsg::fps_log2x(gd->ny) >= 0 || nsg::fps_gen_ok(gd->ny));
        const char* fdn = getenv("NSGPU_FPS_DENSE");
        const bool dense = !fft && !outflow && gd->ny >= 2 && gd->ny <= (yuni ? 4096 : 8192) &&
                           !(fdn && std::atoi(fdn) == 0);
        s->fps = p->poisson == NS_POISSON_MG && !(fe && std::atoi(fe) == 0) && !masked &&
                 (fft ? (!outflow || out_ok) : dense);
        s->fps_dense = s->fps && !fft;
        s->fa.outE = s->fps && outflow ? 1 : 0;
        if (const char* e = getenv("NSGPU_FPS_CHECK")) s->fps_check = std::max(0, std::atoi(e));
        if (const char* e = getenv("NSGPU_FPS_PASSES")) s->fps_passes = std::atoi(e) == 3 && !s->fa.outE ? 3 : 2;
        if (const char* e = getenv("NSGPU_FPS_FUSE")) s->fps_fuse = std::atoi(e) != 0;
        // (r5) ny = 16384 (configs[4]): the two-half transforms have no fused K3 form -- K3, then the DCT; (r6) the
        // one-row transform has (fps_fuse_ok)
        if (!nsg::fps_fuse_ok(gd->ny, s->fa.outE)) s->fps_fuse = false;
        s->fps_xuni = xuni;
        if (!xuni || s->fps_dense) s->fps_fuse = false;   // (r6: K3's general face weights, then the transform)
        if (s->fps) s->phi_extrap = 0;   // (no initial guess: no history planes)
        const char* fpc = getenv("NSGPU_FPS_PC");
        // (r5) or a masked domain whose only NEUMANN edge is its box's whole E column (the backward-facing step):
        // the box's direct solve with the channel's outflow elimination
        bool mask_oe = false;
        if (masked && outflow && gd->nx % 2 == 0 && gd->nx >= 4 && !(foe && std::atoi(foe) == 0) &&
            !(getenv("NSGPU_CAP_OUTFLOW") && std::atoi(getenv("NSGPU_CAP_OUTFLOW")) == 0)) {
            int en = -1, nne = 0;
            for (int e = 0; e < gd->n_edges; e++)
                if (gd->edges[e].type == NS_BC_NEUMANN) { en = e; nne++; }
            bool whole = nne == 1;
            for (int j = 0; j < gd->ny && whole; j++) {
                const size_t c = (size_t)(gd->nx - 1) * gd->ny + j;
                whole = gd->cell_id[c] >= 0 && gd->face_edge[4 * c + 1] == en;
            }
            long faces = 0;
            for (size_t c = 0; c < (size_t)gd->nx * gd->ny && whole; c++)
                for (int f = 0; f < 4; f++) faces += gd->face_edge[4 * c + f] == en;
            mask_oe = whole && faces == gd->ny;
        }
        s->fps_pc = p->poisson == NS_POISSON_MG && !(fe && std::atoi(fe) == 0) && !(fpc && std::atoi(fpc) == 0) &&
                    masked && (!outflow || mask_oe) && yuni && xuni && p->nranks == 1 && nsg::fps_log2(gd->ny) >= 0;
        if (s->fps_pc && outflow) s->fa.outE = 1;
        // (r6) the capacitance solve (cap_setup, unless NSGPU_CAP=0) is exact: BiCGStab takes one iteration from
        // any start, so no phi extrapolation (its k_axpby pass, 87 us at 4096^2, and its four history planes)
        const char* cpe = getenv("NSGPU_CAP");
        if (s->fps_pc && !(cpe && std::atoi(cpe) == 0)) s->phi_extrap = 0;
    }

    auto fail = [&](int rc) { ns_destroy(s); return rc; };
    int dev = p->device;
    if (dev < 0) {
        const char* lr = getenv("LOCAL_RANK");
        dev = lr ? atoi(lr) : 0;
    }
    s->device = dev;
    if (hipSetDevice(dev) != hipSuccess) { set_err("hipSetDevice(%d) failed", dev); return fail(NS_EHIP); }
    {
        // multi-rank, opt-in (NSGPU_COMM_CUS=n): the compute stream leaves n CUs to the comm stream,
        // whose RCCL kernels then run beside the interior strips of an overlapped pass instead of
        // queueing until the strips' resident round drains.  Off by default: the masked compute
        // kernels lost what the exchanges gained (virtual-slab projections, profiles/r03)
        int cus = 0;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const bool comm = p->nranks > 1 || loopback;
        s->comm_cus = 0;
        if (const char* e = getenv("NSGPU_COMM_CUS")) s->comm_cus = std::max(0, std::atoi(e));
        // (a single rank without the loopback has no comm traffic: no masks, every CU computes)
        if (comm && s->comm_cus > 0 && s->comm_cus < cus && cus <= 1024 && cus % 8 == 0) {
            // the reserved CUs spread evenly over the 8 XCDs: workgroups are dispatched round-robin
            // over the XCDs, so an XCD short of CUs would be every launch's straggler (all 8 on one
            // XCD made the strips ~40 % slower).  Bit 32 x + ((x + 8 j) % 32), j < comm_cus / 8: one
            // CU of XCD x per j whether mask bits number the CUs XCD-major or XCD-interleaved
            const int per = cus / 8;
            s->comm_cus = std::max(8, s->comm_cus / 8 * 8);
            std::vector<uint32_t> mc((cus + 31) / 32, 0u), mx((cus + 31) / 32, 0u);
            std::vector<char> comm_cu(cus, 0);
            for (int x = 0; x < 8; x++)
                for (int j = 0; j < s->comm_cus / 8; j++) comm_cu[per * x + (x + 8 * j) % per] = 1;
            for (int k = 0; k < cus; k++) (comm_cu[k] ? mx : mc)[k / 32] |= 1u << (k % 32);
            if (hipExtStreamCreateWithCUMask(&s->st, (uint32_t)mc.size(), mc.data()) != hipSuccess ||
                hipExtStreamCreateWithCUMask(&s->cst, (uint32_t)mx.size(), mx.data()) != hipSuccess) {
                set_err("CU-masked stream create failed");
                return fail(NS_EHIP);
            }
            s->compute_cus = cus - s->comm_cus;
        } else {
            s->comm_cus = 0;
        }
    }
    if (!s->st && hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) != hipSuccess) { set_err("stream create failed"); return fail(NS_EHIP); }
    if (hipEventCreateWithFlags(&s->fev, hipEventDisableTiming) != hipSuccess) { set_err("event create failed"); return fail(NS_EHIP); }
    s->loopback = loopback;
    if (loopback && p->nranks > 1) {
        if (const char* e = getenv("NSGPU_VIRTUAL_ITERS")) {
            for (const char* q = e; *q;) {
                int h = 0, c = 0, used = 0;
                if (std::sscanf(q, "%d:%d%n", &h, &c, &used) != 2 || h < 2 || c < 0) {
                    set_err("NSGPU_VIRTUAL_ITERS: expected sweeps:cycles pairs (sweeps >= 2), got '%s'", q);
                    return fail(NS_EINVAL);
                }
                s->replay.emplace_back(h, c);
                q += used;
                if (*q == ',') q++;
            }
        }
        // (its own residuals would not converge the global problem: never solve to tolerance)
        if (s->replay.empty()) {
            set_err("a virtual slab (NSGPU_RCCL_LOOPBACK with nranks > 1) needs NSGPU_VIRTUAL_ITERS");
            return fail(NS_EINVAL);
        }
    }
    if (p->nranks > 1 || s->loopback) {
        const char* ov = getenv("NSGPU_OVERLAP");
        s->overlap = ov ? std::atoi(ov) != 0 : 1;
        if ((!s->cst && hipStreamCreateWithFlags(&s->cst, hipStreamNonBlocking) != hipSuccess) ||
            hipEventCreateWithFlags(&s->xev[0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&s->xev[1], hipEventDisableTiming) != hipSuccess) {
            set_err("comm stream / event create failed");
            return fail(NS_EHIP);
        }
    }

    {
        // (r5) deep ghost rows (ns_solver::deep): multi-rank rectangles on the direct solve with the wall bands and
        // the residual 3-sweep pass, every rank's slab at least deep_e + 3 rows (one neighbour feeds the exchange)
        const char* de = getenv("NSGPU_DEEP");
        // (E1 = 8 + 6 R: the residual pass's 7-row cone plus the one row of each neighbour it computes for K3)
        const int R = std::max(1, s->band_sweeps / 3), E1 = 8 + 6 * R;
        bool ok = p->nranks > 1 && !masked && s->fps && s->helm_band && s->sweep3 && s->sweep3_res && s->triple &&
                  !(de && std::atoi(de) == 0);
        for (int q = 0; q < p->nranks && ok; q++) {
            int32_t a0, a1;
            ns_slab_range(g.nx, p->nranks, q, &a0, &a1);
            ok = a1 - a0 >= E1 + 3;
        }
        if (ok) {
            s->deep = true;
            s->deep_e = E1;
            s->hp = E1 + nsg::HALO + 2;
        }
        if (s->verbose)
            fprintf(stderr, "nsgpu rank %d/%d: %d x %d, rows %d; direct solve %d (outflow %d, fused K3 %d), wall bands %d "
                    "(%d sweeps, %d wide), 3-sweep passes %d (residual %d, triple %d), deep ghost rows %d (%d)\n",
                    s->rank, s->nranks, g.nx, g.ny, g.nxl, (int)s->fps, s->fa.outE, (int)s->fps_fuse, (int)s->helm_band,
                    s->band_sweeps, s->band_w, (int)s->sweep3, (int)s->sweep3_res, (int)s->triple, (int)s->deep,
                    s->deep_e);
    }
    s->plane = (size_t)(g.nxl + 2 * s->hp) * g.ld;
    if (hipMalloc(&s->base, s->plane * NS_NUM_ARR * sizeof(double)) != hipSuccess) {
        set_err("hipMalloc of %zu bytes failed", s->plane * NS_NUM_ARR * sizeof(double));
        return fail(NS_ENOMEM);
    }
    if (hipMemsetAsync(s->base, 0, s->plane * NS_NUM_ARR * sizeof(double), s->st) != hipSuccess) { set_err("memset failed"); return fail(NS_EHIP); }
    for (int k = 0; k < NS_NUM_ARR; k++) s->arr[k] = s->base + k * s->plane + (size_t)s->hp * g.ld;
    if (s->phi_extrap) {
        const size_t np = (size_t)std::min(s->phi_extrap, 4);
        if (hipMalloc(&s->phim_mem, np * s->plane * sizeof(double)) != hipSuccess) { set_err("hipMalloc phim failed"); return fail(NS_ENOMEM); }
        if (hipMemsetAsync(s->phim_mem, 0, np * s->plane * sizeof(double), s->st) != hipSuccess) { set_err("memset failed"); return fail(NS_EHIP); }
        s->phim = s->phim_mem + (size_t)s->hp * g.ld;
        if (np >= 2) s->phim2 = s->phim + s->plane;
        if (np >= 3) s->phim3 = s->phim2 + s->plane;
        if (np >= 4) s->phim4 = s->phim3 + s->plane;
    }

    if (masked) {
        // (the device edge table padded to 32 entries: k_helm_mt_mask reads the NEUMANN flags of all 31 tags at once)
        std::vector<nsg::EdgeDev> etd(etab.begin(), etab.end());
        if (etd.size() < 32) etd.resize(32, nsg::EdgeDev{});
        if (hipMalloc(&s->fc_mem, fch.size() * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(&s->et_mem, etd.size() * sizeof(nsg::EdgeDev)) != hipSuccess) { set_err("hipMalloc topology failed"); return fail(NS_ENOMEM); }
        if (hipMemcpy(s->fc_mem, fch.data(), fch.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(s->et_mem, etd.data(), etd.size() * sizeof(nsg::EdgeDev), hipMemcpyHostToDevice) != hipSuccess) { set_err("topology upload failed"); return fail(NS_EHIP); }
        s->g.fc = s->fc_mem + (size_t)nsg::HALO * g.ld;
        s->g.et = s->et_mem;
        if (!mband.empty()) {
            if (hipMalloc(&s->mband_tiles, mband.size() * sizeof(int32_t)) != hipSuccess) { set_err("hipMalloc topology failed"); return fail(NS_ENOMEM); }
            if (hipMemcpy(s->mband_tiles, mband.data(), mband.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess) { set_err("topology upload failed"); return fail(NS_EHIP); }
            s->mband_n = (int)(mband.size() / 2);
        }
        std::vector<int32_t> ec;
        for (int li = 0; li < g.nxl; li++)
            for (int j = 0; j < g.ny; j++) {
                const int32_t code = fch[(size_t)(li + nsg::HALO) * g.ld + j];
                if ((code & nsg::FC_IN) && !(code & nsg::FC_DEEP)) ec.push_back(li * g.ld + j);
            }
        if (!ec.empty()) {
            if (hipMalloc(&s->ecell_mem, ec.size() * sizeof(int32_t)) != hipSuccess) { set_err("hipMalloc topology failed"); return fail(NS_ENOMEM); }
            if (hipMemcpy(s->ecell_mem, ec.data(), ec.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess) { set_err("topology upload failed"); return fail(NS_EHIP); }
            s->g.ecell = s->ecell_mem;
            s->g.necell = (int)ec.size();
        }
    }

    // coefficient tables (ConstructLHS, FluidSolver.cpp:113-131)
    std::vector<double> hx0(gd->hx, gd->hx + g.nx), hy0(gd->hy, gd->hy + g.ny);
    for (int i = 0; i < g.nx; i++)
        if (!(hx0[i] > 0)) { set_err("hx[%d] = %g is not positive", i, hx0[i]); return fail(NS_EINVAL); }
    for (int j = 0; j < g.ny; j++)
        if (!(hy0[j] > 0)) { set_err("hy[%d] = %g is not positive", j, hy0[j]); return fail(NS_EINVAL); }
    {
        const std::vector<double> h = coef_tables(hx0, hy0, g.neu);
        if (hipMalloc(&s->coef, h.size() * sizeof(double)) != hipSuccess) { set_err("hipMalloc coef failed"); return fail(NS_ENOMEM); }
        if (hipMemcpy(s->coef, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) { set_err("coef upload failed"); return fail(NS_EHIP); }
        s->c = coef_view(s->coef, g.nx, g.ny);
        s->c.yuni = 1;
        for (int j = 1; j < g.ny; j++) s->c.yuni &= hy0[j] == hy0[0];
        if (s->fps || s->fps_pc)
            if (int rc = fps_setup(s, hy0, h.data(), h.data() + g.nx)) return fail(rc);
    }
    // a masked domain's Poisson preconditioner: one V-cycle of the BOUNDING BOX's wall-closure
    // multigrid (a fictitious-domain preconditioner: the rhs is 0 outside the domain, the
    // outside values of the result are ignored by the masked operator), unless
    if (s->poisson == NS_POISSON_MG) {
        // one NEUMANN side, W or E (a grid row: one slab's, contiguous) of a rectangle: the
        // line-solve preconditioner (NSGPU_OUTFLOW_PC=wall: the round-1 wall closure, A/B)
        const int nneu = g.neu[0] + g.neu[1] + g.neu[2] + g.neu[3];
        const char* ope = getenv("NSGPU_OUTFLOW_PC");
        const bool line_pc = g.ny <= 4096 && !(ope && !std::strcmp(ope, "wall"));
        if (!masked && nneu == 1 && (g.neu[0] || g.neu[1]) && line_pc) s->out_side = g.neu[0] ? 0 : 1;
        if (masked && line_pc) {
            // a polygon whose only NEUMANN edge is exactly the bounding box's W or E column (every
            // cell of it in the domain -- e.g. the backward-facing step's outflow): the box
            // hierarchy takes the same line closure on that side
            int en = -1, nne = 0;
            for (int e = 0; e < gd->n_edges; e++)
                if (gd->edges[e].type == NS_BC_NEUMANN) { en = e; nne++; }
            for (int k = 0; k < 2 && nne == 1 && s->out_side < 0; k++) {
                const int i = k == 0 ? 0 : g.nx - 1;
                bool whole = true;
                for (int j = 0; j < g.ny && whole; j++) {
                    const size_t c = (size_t)i * g.ny + j;
                    whole = gd->cell_id[c] >= 0 && gd->face_edge[4 * c + k] == en;
                }
                long faces = 0;   // the edge must not reach any other cell face
                for (size_t c = 0; c < (size_t)g.nx * g.ny && whole; c++)
                    for (int f = 0; f < 4; f++) faces += gd->face_edge[4 * c + f] == en;
                if (whole && faces == g.ny) s->out_side = k;
            }
        }
        if (p->mg_pre > 0) s->mg_pre = p->mg_pre;
        if (p->mg_omega > 0) s->mg_omega_s = p->mg_omega;
        if (const char* e = getenv("NSGPU_MG_OMEGA")) s->mg_omega_s = std::atof(e);   // smoother over-relaxation (A/B)
        if (p->mg_post > 0) s->mg_post = p->mg_post;
        // (a masked domain preconditioned by the box's direct solve, fps_pc, never runs a V-cycle: its
        // Poisson BiCGStab takes fps_precond, its Helmholtz BiCGStab the Jacobi preconditioner -- no
        // hierarchy is allocated for it)
        if (!s->fps_pc)
            if (int rc = build_levels(s, hx0, hy0)) return fail(rc);
        if (p->mg_coarse_iters > 0) s->mg_coarse_iters = p->mg_coarse_iters;
        if (s->lv.size() < 2 && !s->fps_pc) {
            // nothing to coarsen: plain RB-SOR (O(n) sweeps per solve) -- say so when that is a
            // real grid, not a toy
            if ((long)g.nx * g.ny > 64L * 64L && s->rank == 0)
                fprintf(stderr, "nsgpu: warning: the %d x %d grid cannot be coarsened (odd size%s): the multigrid "
                        "Poisson solve falls back to red-black SOR sweeps\n", g.nx, g.ny,
                        s->nranks > 1 ? " or slab edges" : "");
            s->poisson = NS_POISSON_RBSOR;
        }
        s->krylov_mg = true;
    }
    if (masked || g.neu[0] || g.neu[1] || g.neu[2] || g.neu[3]) {
        // BiCGStab planes (outflow rectangle: the preconditioner is the hierarchy above -- with a
        // single level its coarse relaxation, 2n+10 SOR sweeps from zero; masked domain: Jacobi)
        const size_t nk = sizeof(s->kv) / sizeof(s->kv[0]);
        const size_t kn = nk * s->plane + g.ld;
        if (hipMalloc(&s->kv_mem, kn * sizeof(double)) != hipSuccess) { set_err("hipMalloc Krylov planes failed"); return fail(NS_ENOMEM); }
        if (hipMemsetAsync(s->kv_mem, 0, kn * sizeof(double), s->st) != hipSuccess) { set_err("memset failed"); return fail(NS_EHIP); }
        for (size_t k = 0; k < nk; k++) s->kv[k] = s->kv_mem + k * s->plane + (size_t)s->hp * g.ld;
        s->lrow = s->kv_mem + nk * s->plane;
        if (hipMalloc(&s->ksc, nsg::KS_NUM * sizeof(double)) != hipSuccess) { set_err("hipMalloc failed"); return fail(NS_ENOMEM); }
        if (hipMemsetAsync(s->ksc, 0, nsg::KS_NUM * sizeof(double), s->st) != hipSuccess) { set_err("memset failed"); return fail(NS_EHIP); }
    }
    if (s->fps_pc && s->kv[0]) {   // (r5) the masked domain's capacitance matrix
        const std::vector<double> h = coef_tables(hx0, hy0, g.neu);
        if (int rc = cap_setup(s, gd, h.data(), h.data() + g.nx, h.data() + 3 * g.nx, h.data() + 3 * g.nx + g.ny))
            return fail(rc);
    }
    const int np = nsg::max_partials(g);
    // partials: [0, 4 np) for any kernel's, [4 np, 8 np) for a speculative K5's (correct_launch)
    if (hipMalloc(&s->part, (size_t)np * 8 * sizeof(double)) != hipSuccess) { set_err("hipMalloc partials failed"); return fail(NS_ENOMEM); }
    if (hipMalloc(&s->scal, S_NUM * sizeof(double)) != hipSuccess) { set_err("hipMalloc scalars failed"); return fail(NS_ENOMEM); }
    if (hipMemsetAsync(s->scal, 0, S_NUM * sizeof(double), s->st) != hipSuccess) { set_err("memset failed"); return fail(NS_EHIP); }
    if (hipHostMalloc(&s->hs, S_NUM * sizeof(double), hipHostMallocDefault) != hipSuccess) { set_err("hipHostMalloc failed"); return fail(NS_ENOMEM); }
    // (r5) the scalar bus of multi-rank rectangles (bus())
    {
        const char* be = getenv("NSGPU_BUS");
        s->bus = s->nranks > 1 && !masked && !(be && std::atoi(be) == 0);
        if (s->bus && (hipMalloc(&s->bus_mem, (size_t)BUS_NV * s->nranks * sizeof(double)) != hipSuccess ||
                       hipMemsetAsync(s->bus_mem, 0, (size_t)BUS_NV * s->nranks * sizeof(double), s->st) != hipSuccess)) {
            set_err("hipMalloc of the scalar bus failed");
            return fail(NS_ENOMEM);
        }
        const char* de = getenv("NSGPU_FPS_DEFER");
        // (r6: not with an outflow side -- its mode 0 takes the projected shift, the mean never enters)
    s->fps_defer = s->bus && s->fps && s->fps_fuse && s->m0e && !s->fa.outE && !(de && std::atoi(de) == 0);
    {
        // (r6) K5 deferred into the next async step's K1 (k_rhs_sc): one rank, a rectangle without NEUMANN sides (the
        // streaming K5's domain), the direct solve (no phi-history guess formed by K5), hy uniform (K1's correction
        // takes GradP's y face weights as 0.5); NSGPU_K5_DEFER=0: K5 at every step's end (A/B)
        const char* kd = getenv("NSGPU_K5_DEFER");
        s->k5_defer_ok = !comm_on(s) && !s->g.fc && s->fps && s->c.yuni && !getenv("NSGPU_RHS") && !s->tiled &&
                         nsg::correct_streams(s->g) && !(kd && std::atoi(kd) == 0);
    }
    }

    if (s->loopback) {
        ncclUniqueId id;
        ncclResult_t r = ncclGetUniqueId(&id);
        if (r == ncclSuccess) r = ncclCommInitRank(&s->comm, 1, id, 0);
        if (r != ncclSuccess) { set_err("loopback ncclCommInitRank: %s", ncclGetErrorString(r)); return fail(NS_ERCCL); }
    } else if (s->nranks > 1 && p->host_transport && p->host_transport->exchange) {
        s->ht = *p->host_transport;
    } else if (s->nranks > 1) {
        ncclUniqueId id;
        std::memcpy(&id, p->nccl_id, sizeof id);
        ncclResult_t r = ncclCommInitRank(&s->comm, s->nranks, id, s->rank);
        if (r != ncclSuccess) { set_err("ncclCommInitRank: %s", ncclGetErrorString(r)); return fail(NS_ERCCL); }
    }
    if (hipStreamSynchronize(s->st) != hipSuccess) { set_err("sync failed"); return fail(NS_EHIP); }
    *out = s;
    return 0;
}

void ns_destroy(ns_solver* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->st) (void)hipStreamSynchronize(s->st);
    if (s->comm) (void)ncclCommDestroy(s->comm);
    if (s->mev) (void)hipEventDestroy(s->mev);
    if (s->mm_host) (void)hipHostFree(s->mm_host);
    for (auto e : s->ev) (void)hipEventDestroy(e);
    for (auto e : s->hev) (void)hipEventDestroy(e);
    for (size_t l = 0; l < s->lv.size(); l++) {
        if (l > 0 && s->lv[l].mem) (void)hipFree(s->lv[l].mem);
        if (s->lv[l].coef) (void)hipFree(s->lv[l].coef);
    }
    if (s->base) (void)hipFree(s->base);
    if (s->phim_mem) (void)hipFree(s->phim_mem);
    if (s->kv_mem) (void)hipFree(s->kv_mem);
    if (s->cvimg) (void)hipFree(s->cvimg);
    if (s->dmat) (void)hipFree(s->dmat);
    if (s->fps_mem) (void)hipFree(s->fps_mem);
    if (s->dense_mem) (void)hipFree(s->dense_mem);
    if (s->rb) (void)dense_lib().destroy(s->rb);
    if (s->cap_mem) (void)hipFree(s->cap_mem);
    for (auto e : s->kev)
        if (e) (void)hipEventDestroy(e);
    if (s->f32_mem) (void)hipFree(s->f32_mem);
    if (s->fc_mem) (void)hipFree(s->fc_mem);
    if (s->mband_tiles) (void)hipFree(s->mband_tiles);
    if (s->ecell_mem) (void)hipFree(s->ecell_mem);
    if (s->et_mem) (void)hipFree(s->et_mem);
    if (s->ksc) (void)hipFree(s->ksc);
    if (s->coef) (void)hipFree(s->coef);
    if (s->part) (void)hipFree(s->part);
    if (s->scal) (void)hipFree(s->scal);
    if (s->bus_mem) (void)hipFree(s->bus_mem);
    if (s->hs) (void)hipHostFree(s->hs);
    if (s->stage) (void)hipHostFree(s->stage);
    if (s->cst) (void)hipStreamSynchronize(s->cst);
    for (auto e : s->xev)
        if (e) (void)hipEventDestroy(e);
    if (s->fev) (void)hipEventDestroy(s->fev);
    if (s->cst) (void)hipStreamDestroy(s->cst);
    if (s->st) (void)hipStreamDestroy(s->st);
    delete s;
}

// the step up to CorrectVelocities (its min/max reduced into scal[S_MM], not yet fetched)
static int step_body_(ns_solver* s, ns_stats& st);
static int step_body(ns_solver* s, ns_stats& st) {
    s->n_xchg = s->n_allred = 0;
    s->x_link = 0.0;
    s->k5_spec = 0;
    if (!s->replay.empty()) {
        const auto& r = s->replay[s->replay_k++ % s->replay.size()];
        s->rp_h = r.first;
        s->rp_c = r.second;
    }
    s->in_step = 1;
    s->corr_k1 = 0;
    const int rc = step_body_(s, st);
    s->in_step = 0;
    st.k5_deferred = s->corr_k1;
    st.n_exchanges = s->n_xchg;
    st.n_allreduces = s->n_allred;
    st.x_link_bytes = s->x_link;
    return rc;
}

static int step_body_(ns_solver* s, ns_stats& st) {
    CHK(rhs(s, true));                                             // ConstructRHS_V       (:546)
    // Helmholtz initial guess: u^n.  (The previous step's u* -- kept by correct() in TMPU/TMPV --
    // was measured worse during the cavity's start-up transient: 14.7 vs 11 sweeps/step at 4096^2.)
    // rhs ghost rows (a checked pair pass and the 3-sweep pass read ib-5): multi-rank passes take them with
    // their first overlapped exchange
    if (s->deep) {   // (r5: K1 computed the rhs deep into the neighbours' rows)
    } else if (s->nranks > 1 && s->overlap && s->cst && !s->g.fc && !s->tiled) s->helm_b_pend = 1;
    else CHK(halo(s, {s->arr[NS_ARR_RU], s->arr[NS_ARR_RV]}, 6));
    s->hn = 0;
    // the Poisson initial guess (phi extrapolation) waits to hide the Helmholtz check's host sync
    s->extrap_pending = s->phim ? 1 : 0;
    CHK(helm_solve(s, &st.it_u, &st.res_u, &st.res_v));            // KSPSolve(uSolver) x2 (:547-548)
    if (s->extrap_pending) { s->extrap_pending = 0; CHK(extrapolate_phi(s)); }
    st.it_v = st.it_u;
    for (int k = 0; k < s->hn; k++) {   // (helm_solve's last residual check synchronised the stream)
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, s->hev[2 * k], s->hev[2 * k + 1]));
        st.t_helm_kernel_ms += ms;
        st.n_helm_kernels += (size_t)k < s->hcomp.size() ? s->hcomp[k] : 1;   // (per component: 24 B/cell)
    }
    s->hn = 0;
    if (s->timing && s->kev[0]) {   // (K1 ended before the Helmholtz checks' host syncs)
        st.t_rhs_kernel_ms += kev_ms(s, 0);
        st.n_rhs_kernels++;
    }
    for (int k = 0; k < s->band_timed; k++) {   // (r6: the wall bands, before the same syncs)
        st.t_band_kernel_ms += kev_ms(s, 8 + 2 * k);
        st.n_band_kernels++;
    }
    s->band_timed = 0;
    if (s->k5_pend) {   // (r6: the previous step's K5, ended before this step's first host sync)
        st.t_k5_kernel_ms += kev_ms(s, 12);
        st.n_k5_kernels++;
        s->k5_pend = 0;
    }
    if (!s->k3_spec) CHK(divergence(s));                           // ConstructRHS_phi + mean (:549-550)
    s->k3_spec = 0;
    CHK(consistent_rhs(s));                                        // stretched grids only
    // rhs_phi ghost rows: with the multigrid's first overlapped FUSE_R exchange when it has one
    // (the direct solve reads only the slab's own rows)
    if (s->fps) {
    } else if (s->nranks > 1 && s->overlap && s->cst && s->poisson == NS_POISSON_MG && !s->kv[0] &&
               !s->lv.empty() && !s->lv[0].repl && fused_restrict(s, 0) && !tile_level(s, 0)) {
        level(s, 0).b_pend = true;
    } else {
        CHK(halo(s, {s->arr[NS_ARR_RPHI]}, 4));
    }
    CHK(pois_solve_any(s, &st.it_phi, &st.res_phi, &st));         // KSPSolve(phiSolver)  (:551)
    st.phi_checked = st.res_phi >= 0.0 ? 1 : 0;
    CHK(correct(s));                                               // CorrectVelocities    (:552)
    return 0;
}

static int check_monitor(const ns_stats& st) {
    if (!std::isfinite(st.umin) || !std::isfinite(st.umax) || !std::isfinite(st.vmin) || !std::isfinite(st.vmax)) {
        set_err("velocity field is not finite after the step (scheme diverged; see SURVEY.md section 5 on CFL)");
        return NS_EDIVERGE;
    }
    return 0;
}

int ns_step(ns_solver* s, ns_stats* out) {
    if (!s) { set_err("null solver"); return NS_EINVAL; }
    ns_stats st{};
    HIPCHK(hipSetDevice(s->device));
    nsg::set_compute_cus(s->compute_cus);
    if (s->mm_pending) HIPCHK(hipEventSynchronize(s->mev));   // (an ns_step_async before: its copy lands first)
    s->mm_pending = 0;
    CHK(materialize(s));   // (r6: an ns_step_async before left its correction to this step: K5 first, as ns_step does)
    CHK(step_body(s, st));
    if (s->bus) {   // (r5: K5's min / max went to S_MML; fold them now -- the sync step reports its own)
        CHK(bus(s));
        st.n_allreduces++;
    }
    CHK(fetch(s));                                                 // VecMin/VecMax        (:554-557)
    if (s->k5_pend) {   // (r6: this step's K5 -- the fetch synchronised the stream behind it)
        st.t_k5_kernel_ms += kev_ms(s, 12);
        st.n_k5_kernels++;
        s->k5_pend = 0;
    }
    st.umin = s->hs[S_MM];
    st.umax = -s->hs[S_MM + 1];
    st.vmin = s->hs[S_MM + 2];
    st.vmax = -s->hs[S_MM + 3];
    if (out) *out = st;
    return check_monitor(st);
}

// The same step without the host sync at its end (the reference prints min/max every step:
// FluidSolver.cpp:554-560).  Each step's min/max are copied to pinned memory behind its last
// kernel; they are returned by the NEXT call (the monitor one step late: the same printed
// sequence) or by ns_monitor.  The host is back to launch the next step's K1 while K5 runs.
int ns_step_async(ns_solver* s, ns_stats* out) {
    if (!s) { set_err("null solver"); return NS_EINVAL; }
    ns_stats st{};
    HIPCHK(hipSetDevice(s->device));
    nsg::set_compute_cus(s->compute_cus);
    if (!s->mm_host) {
        HIPCHK(hipHostMalloc(&s->mm_host, 4 * sizeof(double), hipHostMallocDefault));
        HIPCHK(hipEventCreateWithFlags(&s->mev, hipEventDisableTiming));
        for (int k = 0; k < 4; k++) s->mm_host[k] = std::numeric_limits<double>::quiet_NaN();
    }
    if (s->k5_defer_ok) {
        // (r6) K5 deferred into the next step's K1: this step's K1 corrects the previous step's u*, v* (if one is
        // pending) and reduces its min / max into S_MM before the Helmholtz check, whose host read brings them --
        // the previous step's monitor, as before; this step's correction waits in U, V, PHI
        // (the previous async step's monitor: in S_MM from this step's K1, or from a K5 a field read ran since)
        const bool had = s->mm_pending != 0;
        s->defer_now = 1;
        const int rc = step_body(s, st);
        s->defer_now = 0;
        CHK(rc);
        const double nan = std::numeric_limits<double>::quiet_NaN();
        st.umin = had ? s->hs[S_MM] : nan;
        st.umax = had ? -s->hs[S_MM + 1] : nan;
        st.vmin = had ? s->hs[S_MM + 2] : nan;
        st.vmax = had ? -s->hs[S_MM + 3] : nan;
        s->mm_pending = 1;
        if (out) *out = st;
        return had ? check_monitor(st) : 0;
    }
    CHK(step_body(s, st));   // (its residual checks synchronised the stream: the previous copy has landed)
    const bool prev = s->mm_pending != 0;
    const double nan = std::numeric_limits<double>::quiet_NaN();
    if (s->bus) {
        // (r5) the previous step's min / max were folded by this step's Helmholtz-check allgather and
        // fetched with its residuals (hs); this step's wait in S_MML for the next collective
        st.umin = prev ? s->hs[S_MM] : nan;
        st.umax = prev ? -s->hs[S_MM + 1] : nan;
        st.vmin = prev ? s->hs[S_MM + 2] : nan;
        st.vmax = prev ? -s->hs[S_MM + 3] : nan;
        s->mm_pending = 1;
        if (out) *out = st;
        return prev ? check_monitor(st) : 0;
    }
    if (prev) HIPCHK(hipEventSynchronize(s->mev));
    st.umin = prev ? s->mm_host[0] : nan;
    st.umax = prev ? -s->mm_host[1] : nan;
    st.vmin = prev ? s->mm_host[2] : nan;
    st.vmax = prev ? -s->mm_host[3] : nan;
    HIPCHK(hipMemcpyAsync(s->mm_host, s->scal + S_MM, 4 * sizeof(double), hipMemcpyDeviceToHost, s->st));
    HIPCHK(hipEventRecord(s->mev, s->st));
    s->mm_pending = 1;
    if (out) *out = st;
    return prev ? check_monitor(st) : 0;
}

int ns_monitor(ns_solver* s, double* mm) {
    if (!s || !mm) { set_err("null argument"); return NS_EINVAL; }
    if (!s->mm_pending) { set_err("ns_monitor: no ns_step_async since the last ns_step / ns_monitor"); return NS_EINVAL; }
    HIPCHK(hipSetDevice(s->device));
    nsg::set_compute_cus(s->compute_cus);
    ns_stats st{};
    s->mm_pending = 0;
    if (s->k5_defer_ok) {   // (r6: the latest step's correction deferred -- K5 now -- or applied by a field read: S_MM)
        CHK(materialize(s));
        CHK(fetch(s));
        st.umin = mm[0] = s->hs[S_MM];
        st.umax = mm[1] = -s->hs[S_MM + 1];
        st.vmin = mm[2] = s->hs[S_MM + 2];
        st.vmax = mm[3] = -s->hs[S_MM + 3];
        return check_monitor(st);
    }
    if (s->bus) {   // (r5: the latest step's min / max still wait in S_MML -- every rank calls this)
        CHK(bus(s));
        CHK(fetch(s));
        st.umin = mm[0] = s->hs[S_MM];
        st.umax = mm[1] = -s->hs[S_MM + 1];
        st.vmin = mm[2] = s->hs[S_MM + 2];
        st.vmax = mm[3] = -s->hs[S_MM + 3];
        return check_monitor(st);
    }
    HIPCHK(hipEventSynchronize(s->mev));
    st.umin = mm[0] = s->mm_host[0];
    st.umax = mm[1] = -s->mm_host[1];
    st.vmin = mm[2] = s->mm_host[2];
    st.vmax = mm[3] = -s->mm_host[3];
    return check_monitor(st);
}

int ns_set_timing(ns_solver* s, int on) {
    if (!s) { set_err("null solver"); return NS_EINVAL; }
    s->timing = on ? 1 : 0;
    return 0;
}

int ns_get_array(ns_solver* s, int which, double* host) {
    CHK(check_arr(s, which));
    CHK(materialize(s));
    HIPCHK(hipSetDevice(s->device));
    nsg::set_compute_cus(s->compute_cus);
    HIPCHK(hipMemcpy2DAsync(host, (size_t)s->g.ny * 8, s->arr[which], (size_t)s->g.ld * 8, (size_t)s->g.ny * 8,
                            s->g.nxl, hipMemcpyDeviceToHost, s->st));
    HIPCHK(hipStreamSynchronize(s->st));
    return 0;
}

int ns_set_array(ns_solver* s, int which, const double* host) {
    CHK(check_arr(s, which));
    CHK(materialize(s));
    s->guess_ready = 0;   // (TMP / the phi planes may change: the next step forms its guess itself)
    s->cu_ext = s->u_ext = s->phi_ext = 0;   // (r5: the deep ghost rows are stale now)
    HIPCHK(hipSetDevice(s->device));
    nsg::set_compute_cus(s->compute_cus);
    HIPCHK(hipMemcpy2DAsync(s->arr[which], (size_t)s->g.ld * 8, host, (size_t)s->g.ny * 8, (size_t)s->g.ny * 8,
                            s->g.nxl, hipMemcpyHostToDevice, s->st));
    // keep the derived scalars consistent with an injected right-hand side
    if (which == NS_ARR_RPHI) CHK(rhs_mean(s));
    if (which == NS_ARR_PHI || which == NS_ARR_TMP) s->phim_valid = 0;
    if (which == NS_ARR_PHI || which == NS_ARR_TMP || which == NS_ARR_RPHI)
        for (int& h : s->mg_hist) h = -1;   // an injected state: no cycle-count history
    if (which == NS_ARR_RU || which == NS_ARR_RV) CHK(helm_bnorm(s));
    HIPCHK(hipStreamSynchronize(s->st));
    return 0;
}

// the reference's compact Vec order (prevField->u, v, phi: FluidSolver.h:6-18, ids from
// Grid.cpp:149-162): a rectangle's compact order IS the bounding-box plane; a masked domain's
// fields are gathered / scattered through the slab's id map (cells outside stay exactly 0)
static int get_compact(ns_solver* s, int which, double* out) {
    if (s->cid.empty()) return ns_get_array(s, which, out);
    s->hbuf.resize(s->cid.size());
    CHK(ns_get_array(s, which, s->hbuf.data()));
    for (size_t k = 0; k < s->cid.size(); k++)
        if (s->cid[k] >= 0) out[s->cid[k]] = s->hbuf[k];
    return 0;
}

static int set_compact(ns_solver* s, int which, const double* in) {
    if (s->cid.empty()) return ns_set_array(s, which, in);
    s->hbuf.assign(s->cid.size(), 0.0);
    for (size_t k = 0; k < s->cid.size(); k++)
        if (s->cid[k] >= 0) s->hbuf[k] = in[s->cid[k]];
    return ns_set_array(s, which, s->hbuf.data());
}

int ns_local_cells(ns_solver* s, int64_t* first_id, int64_t* count) {
    if (!s) { set_err("null solver"); return NS_EINVAL; }
    if (first_id) *first_id = s->cid.empty() ? (int64_t)s->g.i0 * s->g.ny : s->cid0;
    if (count) *count = s->cid.empty() ? (int64_t)s->g.nxl * s->g.ny : s->ncid;
    return 0;
}

int ns_get_fields(ns_solver* s, double* u, double* v, double* phi) {
    if (!s) { set_err("null solver"); return NS_EINVAL; }
    if (u) CHK(get_compact(s, NS_ARR_U, u));
    if (v) CHK(get_compact(s, NS_ARR_V, v));
    if (phi) CHK(get_compact(s, NS_ARR_PHI, phi));
    return 0;
}

int ns_set_fields(ns_solver* s, const double* u, const double* v, const double* phi, const double* cu0,
                  const double* cv0) {
    if (!s) { set_err("null solver"); return NS_EINVAL; }
    s->guess_ready = 0;   // (TMP / the phi planes may change: the next step forms its guess itself)
    s->cu_ext = s->u_ext = s->phi_ext = 0;   // (r5: the deep ghost rows are stale now)
    if (u) CHK(set_compact(s, NS_ARR_U, u));
    if (v) CHK(set_compact(s, NS_ARR_V, v));
    if (phi) CHK(set_compact(s, NS_ARR_PHI, phi));
    if (cu0) CHK(set_compact(s, NS_ARR_CU, cu0));
    if (cv0) CHK(set_compact(s, NS_ARR_CV, cv0));
    return 0;
}

int ns_kernel(ns_solver* s, int which, int iters, double* out) {
    if (s && s->corr_pend) CHK(materialize(s));   // (r6: a deferred correction first)
    if (!s) { set_err("null solver"); return NS_EINVAL; }
    s->guess_ready = 0;   // (TMP / the phi planes may change: the next step forms its guess itself)
    s->cu_ext = s->u_ext = s->phi_ext = 0;   // (r5: a kernel alone writes the slab's own rows: the deep ghost rows are stale)
    HIPCHK(hipSetDevice(s->device));
    nsg::set_compute_cus(s->compute_cus);
    const double alpha = s->dt / (2 * s->re);
    switch (which) {
    case NS_K_RHS:
        CHK(rhs(s));
        CHK(fetch(s));
        if (out) { out[0] = s->hs[S_HBN]; out[1] = s->hs[S_HBN + 1]; }
        return 0;
    case NS_K_HELMHOLTZ: {
        if (s->g.fc) { set_err("NS_K_HELMHOLTZ sweeps are rectangle-only; use NS_K_HELM_SOLVE on a masked domain"); return NS_EINVAL; }
        // single rank with the 3-sweep pass and iters >= 4: one k_sweep3 pass first; then
        // (rest-1)/2 two-sweep passes, then single sweeps; the residual is of the last sweep's input
        int nb = 0;
        CHK(halo(s, {s->arr[NS_ARR_RU], s->arr[NS_ARR_RV]}, 6));
        const int three = (s->sweep3 && s->nranks == 1 && !s->tiled && iters >= 4) ? 3 : 0;
        if (three) helm_sweep3(s, alpha, 1), helm_sweep3(s, alpha, 2);
        const int pairs = iters - three > 0 ? (iters - three - 1) / 2 : 0;
        for (int k = 0; k < pairs; k++) {
            CHK(halo(s, {s->arr[NS_ARR_U], s->arr[NS_ARR_V]}, 4));
            helm_sweep2(s, alpha, nullptr);
        }
        for (int k = three + 2 * pairs; k < iters; k++) {
            CHK(halo(s, {s->arr[NS_ARR_U], s->arr[NS_ARR_V]}, 2));
            nb = helm_sweep(s, alpha, k == iters - 1 ? s->part : nullptr);
        }
        if (iters > 0) {
            nsg::launch_reduce_sum_segs(s->part, nb, 2, s->scal + S_RES, s->st);
            CHK(allreduce(s, s->scal + S_RES, 2, ncclSum));
        }
        CHK(fetch(s));
        if (out) { out[0] = s->hs[S_RES]; out[1] = s->hs[S_RES + 1]; }
        return 0;
    }
    case NS_K_HELM_BAND: {
        if (s->g.fc || s->tiled) { set_err("NS_K_HELM_BAND needs a rectangle and the streaming sweeps"); return NS_EINVAL; }
        CHK(halo(s, {s->arr[NS_ARR_RU], s->arr[NS_ARR_RV]}, 6));
        CHK(helm_band(s, alpha));
        CHK(fetch(s));
        return 0;
    }
    case NS_K_DIV:
        CHK(divergence(s));
        CHK(fetch(s));
        if (out) { out[0] = s->hs[S_DIVSUM]; out[1] = s->hs[S_DIVSUM + 1]; }
        return 0;
    case NS_K_POISSON: {
        if (s->kv[0]) {
            set_err("NS_K_POISSON sweeps relax the rectangle's wall-closure operator; with a NEUMANN side or a "
                    "masked domain use NS_K_POIS_SOLVE");
            return NS_EINVAL;
        }
        int nb = 0;
        CHK(halo(s, {s->arr[NS_ARR_RPHI]}, 4));
        const int pairs = (s->poisson != NS_POISSON_JACOBI && !s->tiled && iters > 0) ? (iters - 1) / 2 : 0;
        for (int k = 0; k < pairs; k++) {
            CHK(halo(s, {s->arr[NS_ARR_PHI]}, 4));
            nsg::launch_pois_rbsor2(s->g, s->c, s->omega, s->arr[NS_ARR_PHI], s->arr[NS_ARR_TMP], s->arr[NS_ARR_RPHI],
                                    s->scal + S_SHIFT, nullptr, s->st);
            std::swap(s->arr[NS_ARR_PHI], s->arr[NS_ARR_TMP]);
        }
        for (int k = 2 * pairs; k < iters; k++) {
            double* part = k == iters - 1 ? s->part : nullptr;
            CHK(halo(s, {s->arr[NS_ARR_PHI]}, 2));
            nb = pois_sweep(s, part);
        }
        if (iters > 0) {
            nsg::launch_reduce_sum(s->part, nb, 1, s->scal + S_RES, s->st);
            CHK(allreduce(s, s->scal + S_RES, 1, ncclSum));
        }
        CHK(fetch(s));
        if (out) out[0] = s->hs[S_RES];
        return 0;
    }
    case NS_K_CORRECT:
        CHK(correct(s));
        CHK(fetch(s));
        if (out) { out[0] = s->hs[S_MM]; out[1] = -s->hs[S_MM + 1]; out[2] = s->hs[S_MM + 2]; out[3] = -s->hs[S_MM + 3]; }
        return 0;
    case NS_K_HELM_SOLVE: {
        int its = 0;
        double ru = 0, rv = 0;
        CHK(helm_bnorm(s));
        CHK(halo(s, {s->arr[NS_ARR_RU], s->arr[NS_ARR_RV]}, 6));
        CHK(helm_solve(s, &its, &ru, &rv));
        if (out) { out[0] = its; out[1] = std::max(ru, rv); }
        return 0;
    }
    case NS_K_POIS_SOLVE: {
        int its = 0;
        double r = 0;
        CHK(rhs_mean(s));
        CHK(consistent_rhs(s));
        CHK(halo(s, {s->arr[NS_ARR_RPHI]}, 4));
        CHK(pois_solve_any(s, &its, &r, nullptr));
        if (out) { out[0] = its; out[1] = r; }
        return 0;
    }
    case NS_K_RESIDUAL: {
        if (s->kv[0]) {
            set_err("NS_K_RESIDUAL is the rectangle's wall-closure residual; not defined with a NEUMANN side or a mask");
            return NS_EINVAL;
        }
        CHK(halo(s, {s->arr[NS_ARR_PHI]}, 1));
        const int nb = nsg::launch_pois_residual(s->g, s->c, s->arr[NS_ARR_PHI], s->arr[NS_ARR_RPHI],
                                                 s->scal + S_SHIFT, s->part, s->st);
        nsg::launch_reduce_sum(s->part, nb, 1, s->scal + S_AUX, s->st);
        CHK(allreduce(s, s->scal + S_AUX, 1, ncclSum));
        CHK(fetch(s));
        if (out) out[0] = s->hs[S_AUX];
        return 0;
    }
    case NS_K_POISSON32: {
        if (s->kv[0]) { set_err("NS_K_POISSON32 sweeps the rectangle's wall-closure operator (no NEUMANN side, no mask)"); return NS_EINVAL; }
        int nb = 0;
        CHK(to_f32(s));
        for (int k = 0; k < iters; k++) CHK(pois_sweep32(s, k == iters - 1 ? s->part : nullptr, &nb));
        nsg::launch_to_f64(s->g, s->f32[0], s->arr[NS_ARR_PHI], s->st);
        if (iters > 0) {
            nsg::launch_reduce_sum(s->part, nb, 1, s->scal + S_RES, s->st);
            CHK(allreduce(s, s->scal + S_RES, 1, ncclSum));
        }
        CHK(fetch(s));
        if (out) out[0] = s->hs[S_RES];
        return 0;
    }
    default:
        set_err("unknown kernel %d", which);
        return NS_EINVAL;
    }
}

int ns_mg_transfer(ns_solver* s, int op, double* coarse) {
    if (s && s->corr_pend) CHK(materialize(s));   // (r6: a deferred correction first)
    if (!s || !coarse || s->poisson != NS_POISSON_MG || s->lv.size() < 2) {
        set_err("ns_mg_transfer needs a multigrid solver with at least two levels");
        return NS_EINVAL;
    }
    s->guess_ready = 0;   // (TMP / the phi planes may change: the next step forms its guess itself)
    HIPCHK(hipSetDevice(s->device));
    nsg::set_compute_cus(s->compute_cus);
    MgLevel& F = level(s, 0);
    MgLevel& C = level(s, 1);
    const CoarseView cv = coarse_view(s, 0);   // this rank's coarse rows (a slab of a replicated level)
    const size_t w = (size_t)C.g.ny * 8;
    if (op == 0) {
        CHK(halo_g(s, F.g, {F.phi}, 1));
        nsg::launch_restrict(F.g, F.c, F.phi, F.b, s->scal + S_SHIFT, cv.g, C.c, cv.b, cv.phi, s->part, s->st);
        HIPCHK(hipMemcpy2DAsync(coarse, w, cv.b, (size_t)C.g.ld * 8, w, cv.g.nxl, hipMemcpyDeviceToHost, s->st));
    } else {
        HIPCHK(hipMemcpy2DAsync(cv.phi, (size_t)C.g.ld * 8, coarse, w, w, cv.g.nxl, hipMemcpyHostToDevice, s->st));
        if (cv.gather) {
            // the prolongation reads the neighbours' coarse rows too: gather them (the gather
            // moves b, so stage phi through it)
            HIPCHK(hipMemcpyAsync(C.b, C.phi, (size_t)C.g.nx * C.g.ld * 8, hipMemcpyDeviceToDevice, s->st));
            CHK(gather_level(s, C));
            HIPCHK(hipMemcpyAsync(C.phi, C.b, (size_t)C.g.nx * C.g.ld * 8, hipMemcpyDeviceToDevice, s->st));
        } else {
            CHK(halo_g(s, C.g, {C.phi}, 1));
        }
        nsg::launch_prolong(F.g, F.phi, cv.g, cv.phi, s->st);
    }
    HIPCHK(hipStreamSynchronize(s->st));
    return 0;
}

int ns_fill_random(ns_solver* s, uint64_t seed) {
    if (s && s->corr_pend) CHK(materialize(s));   // (r6: a deferred correction first)
    if (!s) { set_err("null solver"); return NS_EINVAL; }
    s->guess_ready = 0;   // (TMP / the phi planes may change: the next step forms its guess itself)
    if (s->g.fc) { set_err("ns_fill_random (the sweep benchmark input) is rectangle-only"); return NS_EINVAL; }
    HIPCHK(hipSetDevice(s->device));
    nsg::set_compute_cus(s->compute_cus);
    nsg::launch_fill_random(s->g, s->arr[NS_ARR_PHI], s->arr[NS_ARR_RPHI], seed, s->st);
    CHK(rhs_mean(s));  // the random rhs's mean becomes the Poisson shift (null-space removal)
    CHK(halo(s, {s->arr[NS_ARR_RPHI]}, 4));
    HIPCHK(hipStreamSynchronize(s->st));
    return 0;
}

int ns_time_poisson(ns_solver* s, int warmup, int iters, double* out) {
    if (s && s->corr_pend) CHK(materialize(s));   // (r6: a deferred correction first)
    if (!s || iters <= 0) { set_err("bad arguments"); return NS_EINVAL; }
    s->guess_ready = 0;   // (TMP / the phi planes may change: the next step forms its guess itself)
    if (s->kv[0]) { set_err("ns_time_poisson times the rectangle's sweeps (no NEUMANN side, no mask)"); return NS_EINVAL; }
    HIPCHK(hipSetDevice(s->device));
    nsg::set_compute_cus(s->compute_cus);
    CHK(ensure_events(s, 2 * (size_t)iters));
    // NSGPU_TIME_PAIRS=1: time the two-sweep (temporally blocked) pass instead of a single sweep
    const bool pairs = getenv("NSGPU_TIME_PAIRS") && s->poisson != NS_POISSON_JACOBI;
    auto one = [&](double* part) -> int {
        if (!pairs) {
            CHK(halo(s, {s->arr[NS_ARR_PHI]}, 2));
            pois_sweep(s, part);
            return 0;
        }
        CHK(halo(s, {s->arr[NS_ARR_PHI]}, part ? 5 : 4));
        nsg::launch_pois_rbsor2(s->g, s->c, s->omega, s->arr[NS_ARR_PHI], s->arr[NS_ARR_TMP], s->arr[NS_ARR_RPHI],
                                s->scal + S_SHIFT, part, s->st);
        std::swap(s->arr[NS_ARR_PHI], s->arr[NS_ARR_TMP]);
        return 0;
    };
    for (int k = 0; k < warmup; k++) CHK(one(nullptr));
    for (int k = 0; k < iters; k++) {
        CHK(t_begin(s, s->ev[2 * k], s->ev[2 * k + 1]));
        CHK(one(k == iters - 1 ? s->part : nullptr));
        CHK(t_end(s, s->ev[2 * k], s->ev[2 * k + 1]));
    }
    HIPCHK(hipStreamSynchronize(s->st));
    double tot = 0.0;
    for (int k = 0; k < iters; k++) {
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, s->ev[2 * k], s->ev[2 * k + 1]));
        tot += ms;
    }
    float span = 0.f;
    HIPCHK(hipEventElapsedTime(&span, s->ev[0], s->ev[2 * iters - 1]));
    if (out) { out[0] = tot / iters; out[1] = tot; out[2] = span; }
    return 0;
}

int ns_time_poisson_fp32(ns_solver* s, int warmup, int iters, double* out) {
    if (s && s->corr_pend) CHK(materialize(s));   // (r6: a deferred correction first)
    if (!s || iters <= 0) { set_err("bad arguments"); return NS_EINVAL; }
    s->guess_ready = 0;   // (TMP / the phi planes may change: the next step forms its guess itself)
    if (s->kv[0]) { set_err("ns_time_poisson_fp32 times the rectangle's sweeps (no NEUMANN side, no mask)"); return NS_EINVAL; }
    HIPCHK(hipSetDevice(s->device));
    nsg::set_compute_cus(s->compute_cus);
    CHK(ensure_events(s, 2 * (size_t)iters));
    CHK(to_f32(s));
    int nb = 0;
    for (int k = 0; k < warmup; k++) CHK(pois_sweep32(s, nullptr, &nb));
    for (int k = 0; k < iters; k++) {
        CHK(t_begin(s, s->ev[2 * k], s->ev[2 * k + 1]));
        CHK(pois_sweep32(s, nullptr, &nb));
        CHK(t_end(s, s->ev[2 * k], s->ev[2 * k + 1]));
    }
    nsg::launch_reduce_sum(s->part, nb, 1, s->scal + S_RES, s->st);
    CHK(allreduce(s, s->scal + S_RES, 1, ncclSum));
    CHK(fetch(s));
    double tot = 0.0;
    for (int k = 0; k < iters; k++) {
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, s->ev[2 * k], s->ev[2 * k + 1]));
        tot += ms;
    }
    float span = 0.f;
    HIPCHK(hipEventElapsedTime(&span, s->ev[0], s->ev[2 * iters - 1]));
    if (out) { out[0] = tot / iters; out[1] = tot; out[2] = span; out[3] = s->hs[S_RES]; }
    return 0;
}

}  // extern "C"
