"""bench.py -- headline benchmark: full incompressible-flow time steps of the lid-driven
cavity (BASELINE.json metric "cell-updates/sec (MLUPS) + Poisson iters/sec, 4096^2 grid at
1/2/4/8 GPUs").

A "step" = one FluidSolver::Solve loop body (/root/reference/SRC/FluidSolver.cpp:546-560):
RHS (K1) -> Helmholtz u, v (K2 sweeps to rtol) -> divergence (K3) -> Poisson (K4 sweeps to
rtol 1e-8, warm start) -> correction + min/max (K5), on the 4096^2 cavity (fp64, Re 1000,
dt = 1/(8n)), inputs resident in HBM.  N > 1: x-slabs, one rank per GPU, RCCL halos
(strong scaling: the global grid is fixed).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--n 4096] [--re 1000] [--no-cpu]
                  [--transport rccl|host]
  (N > 1 under torch.distributed.run; RANK / WORLD_SIZE / LOCAL_RANK from the env; without a
  launcher, --gpus N starts its own N ranks and relays rank 0's JSON line)

--transport host (or NSBENCH_TRANSPORT=host): the N > 1 branch as a rehearsal on ONE GPU -- every
rank on device 0, the ghost rows / gathers / reductions through the host (gloo) instead of RCCL
(libnsgpu.so's ns_host_transport call sites).  The line is then functional evidence for the
multi-rank path (self-launch, slab step, per-rank timing max, local-cell rooflines, rank-0 JSON),
not a scaling number: `config.transport` says so.

--case channel (not the headline line): the n x n/4
channel (square cells h = 4/n, inlet W, walls S / N, the reference's NEUMANN outflow E,
Re 1000, dt = h/8) -- Helmholtz RB-SOR as above; Poisson (r5) by the direct solve with the outflow
row eliminated (one rank, nx even; NSGPU_FPS_OUTFLOW=0 or slabs: BiCGStab on the true outflow operator
preconditioned by the line-closure V-cycle); `roofline` from the same HIP-event timing.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
# the finest multigrid level's two passes per V-cycle, timed with HIP events on the solver's
# stream around every launch in the timed region (ns_params.timing).  Algorithmic bytes per
# cell (24 B/cell for one unfused sweep: read phi, read b, write phi):
#   restriction pass (k_sweep2 FUSE_R): two RB sweeps + residual + restriction:
#       read phi 8 + read b 8 + write phi 8 + write the coarse rhs 8 / 4                = 26
#       (the coarse level's first pass takes its iterate as zero -- ZIN, r3 -- so no coarse phi
#       store; PMC write bytes: phi 134.2 MB + coarse b 33.6 MB at 4096^2)
#   prolongation pass (k_sweep2 FUSE_P): prolongation + two RB sweeps:
#       read phi 8 + read b 8 + write phi 8 + read the coarse correction 8 / 4         = 26
# and the Helmholtz solve's passes (K2, single rank: one velocity component per pass):
#   Helmholtz pass (k_sweep3 / k_sweep2<Helmholtz>): 3 or 2 RB-SOR sweeps: read q 8 + read b 8 + write q 8 = 24
# The one with the largest total time per step is `roofline` (the dominant kernel).
KERNELS = {
    "restrict": ("k_sweep2<Poisson, FUSE_R> (finest pre-smoothing pass: 2 RB sweeps + residual + restriction)", 26),
    "prolong": ("k_sweep2<Poisson, FUSE_P> (finest post-smoothing pass: prolongation + 2 RB sweeps + output residual)", 26),
    # (r4) a V-cycle boundary in one pass, when the cycle's output is not checked: the prolongation
    # + 4 RB sweeps + residual + restriction (k_sweep4): read phi 8 + b 8 + the coarse correction
    # 8 / 4, write phi 8 + the coarse rhs 8 / 4 = 28
    "cycle": ("k_sweep4 (finest V-cycle boundary: prolongation + 4 RB sweeps + residual + restriction, "
              "cycle c's FUSE_P and cycle c+1's FUSE_R in one pass)", 28),
    # (r4) a solve's first FUSE_R pass forming the phi extrapolation on the fly (k_sweep2_gin): FUSE_R's
    # 26 B/cell with 4 history planes read instead of phi (cubic guess; 3 quadratic): 26 + 24 = 50
    "guess": ("k_sweep2_gin (a Poisson solve's first finest restriction pass; its input, the cubic phi "
              "extrapolation, formed from 4 history planes as rows enter)", 50),
    "helmholtz": ("Helmholtz pass of one velocity component of (I - a L_V) u* = RHS (k_sweep3 + residual stage: "
                  "3 RB-SOR sweeps, after the wall bands; or k_sweep2: 2 sweeps; the one-rank two-field "
                  "k_sweep3<FUSE_UV> launch counts as two component passes)", 24),
    # K1 (ConstructRHS_V): read u, v, phi^{n-1}, cu, cv 40 + write cu, cv, ru, rv 32 -- minus the
    # in-place cu / cv reads counted once: 64
    "rhs": ("k_rhs_s (K1, ConstructRHS_V: AB2 MUSCL/Rusanov convection + CN-explicit diffusion + wall terms)", 64),
    # (r4) the direct Poisson solve (ns_fps.hip): the rows' DCT-II read b 8 + write 8; the
    # recurrences along x, two full passes: t1b read 8, t2b read 8 + write 8 (the three-pass form,
    # NSGPU_FPS_PASSES=3: t1 read 8, t2 read 8 + write 8, t3 read 8 + write 8 = 40; chunk / group
    # aggregates ~1-2 B/cell more, not counted) -- one interval over five launches; the inverse DCT
    # read 8 + write 8
    "fps_dct": ("k_fps_dct (direct Poisson solve: DCT-II of every row pair of b - mean, Stockham FFT in LDS)", 16),
    "fps_tri": ("k_fps_t1b + scan + k_fps_mid + scan + k_fps_t2b (direct Poisson solve: the tridiagonal "
                "recurrences along x, one per mode, chunked; five launches timed as one interval)",
                40 if os.environ.get("NSGPU_FPS_PASSES") == "3" else 24),
    "fps_idct": ("k_fps_idct_r (direct Poisson solve: DCT-III of every row -> phi, one row per workgroup as an "
                 "N/2-point complex FFT; k_fps_idct's row pairs outside 1024 <= ny <= 16384)", 16),
    # (r6) K5 (CorrectVelocities + GradP + the min / max monitor): read phi 8 + u*, v* 16, write u, v 16 = 40
    "k5": ("k_cell_s<5> (K5, CorrectVelocities: u = u* - dt grad phi, fused min / max of u, v)", 40),
    # (r6) the Helmholtz wall bands (k_helm_band, 3 RB-SOR sweeps per launch on the cells within 128 of a wall):
    # per band cell u, v read 16 + rhs 16 + write 16 = 48 B; per cell of the grid 48 x the band's fraction
    # (set in run(): BAND_BPC)
    "band": ("k_helm_band (Helmholtz wall bands: 3 RB-SOR sweeps of u, v on the cells within 128 of a wall, "
             "LDS-tiled)", None),
}
# (r4) K3 fused into the DCT (NSGPU_FPS_FUSE, default on): the divergence of u*, v* formed in the
# transform's LDS -- read u*, v* 16 + write the coefficients 8; rhs_phi (8 more) only for a checked solve
FPS_FUSED = os.environ.get("NSGPU_FPS_FUSE", "1") != "0"
if FPS_FUSED:
    KERNELS["fps_dct"] = ("k_fps_dct_div_r (direct Poisson solve: K3's divergence of u*, v* fused into the DCT-II of "
                          "every row, one row per workgroup -- its N reals as an N/2-point complex FFT, radix-8 "
                          "Stockham in LDS; k_fps_dct_div's row pairs outside 1024 <= ny <= 16384)", 24)
# one-launch kernels (the `roofline` candidates; fps_tri is five launches)
SINGLE_LAUNCH = ("restrict", "prolong", "cycle", "guess", "helmholtz", "rhs", "fps_dct", "fps_idct", "k5", "band")
JACOBI_LABEL = "k_jacobi_s<double> (one weighted-Jacobi sweep of the Poisson operator, the north star's roofline kernel)"
SWEEP_BYTES_PER_CELL = 24
# configs[4]'s fp32-field Jacobi sweep: read phi 4 + read b 4 + write phi 4 (fp64 arithmetic / residual)
JACOBI32_LABEL = "k_jacobi_s<float> (one Jacobi sweep on fp32 phi, b; fp64 arithmetic and residual: configs[4])"
SWEEP32_BYTES_PER_CELL = 12


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--case", choices=("cavity", "channel", "stretched", "xstretched"), default="cavity",
                    help="cavity (the headline), channel (NEUMANN outflow), stretched / xstretched (the cavity on a "
                         "geometrically stretched grid, Grid.cpp:87-92: both directions / x only, --ratio)")
    ap.add_argument("--ratio", type=float, default=1.0005,
                    help="--case stretched / xstretched: the face-spacing ratio (Nx / Ny {0 1 n ratio})")
    ap.add_argument("--re", type=float, default=1000.0)
    ap.add_argument("--rtol", type=float, default=1e-8)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-jacobi", action="store_true",
                    help="skip the Jacobi-sweep roofline leg (kernel traces of the step alone)")
    ap.add_argument("--sync-monitor", action="store_true",
                    help="ns_step (host sync at every step's end) instead of ns_step_async")
    ap.add_argument("--transport", choices=("rccl", "host"), default=os.environ.get("NSBENCH_TRANSPORT", "rccl"),
                    help="N > 1: RCCL over xGMI (one GPU per rank), or the host transport (every rank on GPU 0: "
                         "a one-GPU rehearsal of the multi-rank path)")
    ap.add_argument("--time-every", type=int, default=10,
                    help="HIP-event kernel timing on every k-th timed step (each event pair costs a few us of "
                         "GPU idle; 0 = none)")
    return ap.parse_args(argv)


def _sha16(path):
    import hashlib
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _host_threads():
    """The cores this process may use: the box's CPU share (OMP_NUM_THREADS is set to it on
    the GPU pool; os.cpu_count() would name the whole machine), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


HALO = 7   # ghost rows per side (ns_internal.h nsg::HALO)


def helm_passes(n, min_rows):
    """HBM passes of one component's n Helmholtz sweeps (ns_solver.cpp helm_sweeps): 3-sweep
    passes while >= 5 remain; a batch may end on a 3-sweep pass with its residual (3 = 3,
    6 = 3+3; slabs too since HALO = 7), otherwise on a pair (5 = 3+2); an odd remainder otherwise
    starts with a single sweep.  `min_rows` = the thinnest slab's rows: below 2 HALO rows the
    solver allows no 3-sweep pass on any rank (ns_solver::triple), so pairs and single sweeps."""
    triple = min_rows >= 2 * HALO
    p, r = 0, n
    while r > 0:
        if triple and (r >= 5 or r in (3, 6)):
            w = 3
        elif r % 2 and r >= 3:
            w = 1
        else:
            w = min(2, r)
        r -= w
        p += 1
    return p


def cpu_baseline(n, re, dt, omega_v, omega_mg, state, gpu_next=None):
    """The oracle (CPU restatement, -O3, OpenMP) running the SAME algorithm as the GPU path
    (RB-SOR Helmholtz to rtol, multigrid V(2,2) Poisson to rtol 1e-8) for one full time step
    of the same n^2 cavity, from the GPU's own state after its warm-up + timed steps (u, v,
    phi, the convective terms): a steady-state step, not the start-up one.
    Timed at 1 thread (the serial reference) and at the host's cores (a bounded sample:
    ~10-30 s in all).  value = the all-cores rate; value_1thread beside it.
    gpu_next = the GPU's own next step from that state (u, v): the oracle's step must agree with
    it to SURVEY 8(c)'s 1e-6 (both solves to rtol 1e-8) -- parity at the bench's own
    configuration, reported as `parity`."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # CPU baseline leg only

    g = O.OGrid.rectangle(n, n)
    gx, gy = g.grad_phi(state["phi"])
    nt = _host_threads()
    out = {}
    parity = None
    for threads in (1, nt):
        O.set_threads(threads)
        s = O.OSolver(g, dt, re, rtol=1e-8)
        s.use_gpu_algorithm(omega_v, omega_mg)
        s.set(u=state["u"], v=state["v"], phi=state["phi"], cu=state["cu"], cv=state["cv"], gx=gx, gy=gy)
        t0 = time.perf_counter()
        mm, its = s.step()
        out[threads] = (time.perf_counter() - t0, [int(x) for x in its])
        if threads == nt and gpu_next is not None:
            ref = s.get()
            parity = {"max_abs_du": float(np.max(np.abs(gpu_next["u"] - ref["u"]))),
                      "max_abs_dv": float(np.max(np.abs(gpu_next["v"] - ref["v"]))),
                      "oracle_monitor": [float(x) for x in mm], "gpu_monitor": gpu_next["monitor"],
                      "tol": 1e-6}
            parity["ok"] = parity["max_abs_du"] <= 1e-6 and parity["max_abs_dv"] <= 1e-6
        del s
    O.set_threads(1)
    t1, its1 = out[1]
    tn, itsn = out[nt]
    return {
        "value": g.N / tn / 1e6, "unit": "MLUPS", "cores": nt, "kind": "port",
        "value_1thread": g.N / t1 / 1e6,
        "cpu_model": _cpu_model(), "nproc": os.cpu_count(), "threads_used": nt,
        "sample": (f"one full time step of the {n}^2 cavity in the oracle's C restatement (oracle/ns_oracle.c, "
                   f"-O3, OpenMP), started from the GPU's state after its timed steps; same algorithm as the GPU "
                   + ("(the direct Poisson solve: DCT along y, Thomas along x; " if its1[2] == 1 else
                      f"(MG V(2,2) Poisson: {its1[2]} V-cycles from phi^(n-1) -- the GPU's extrapolated guess needs "
                      f"fewer; ")
                   + f"RB-SOR Helmholtz: {its1[0]} sweeps per component), {t1:.1f} s on 1 thread, "
                   f"{tn:.1f} s on {nt} threads"),
        "parity": parity,
    }


def _rccl_version(torch):
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception as e:   # (diagnostic only)
        return f"unknown ({type(e).__name__})"


def self_launch(args) -> int:
    """--gpus N > 1 without a launcher (no WORLD_SIZE in the env): start N ranks, one per GPU,
    under torch.distributed.run on 127.0.0.1 as a CHILD process -- before anything here touches
    the GPU -- and return its exit code.  Rank 0 of the child prints the JSON line."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)]
    env = dict(os.environ)
    # this run's arguments travel in the environment: torch.distributed.run's own parser takes an
    # abbreviation of its options after the script name as its own (--n: ambiguous, --re: --redirects)
    env["NSBENCH_ARGV"] = json.dumps(sys.argv[1:])
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this pool (RCCL)
    env.setdefault("OMP_NUM_THREADS", "1")
    # relay: only whole JSON lines (rank 0's bench line; the launch probe's) reach stdout;
    # everything else the ranks or RCCL print goes to stderr, so no banner can precede or split
    # the line
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    for ln in p.stdout:
        t = ln.strip()
        if t.startswith("{"):
            try:
                json.loads(t)
                print(t, flush=True)
                continue
            except ValueError:
                pass
        sys.stderr.write(ln)
    return p.wait()


METRIC = "cell-updates/sec (MLUPS) + Poisson iters/sec, 4096^2 grid at 1/2/4/8 GPUs"


class Watchdog:
    """Multi-rank runs: a rank that stops making progress -- an RCCL collective
    waiting on a peer that died, a hung communicator set-up -- prints a JSON error line and exits
    non-zero instead of hanging silently; torch.distributed.run then tears the other ranks down.
    `beat(phase, limit_s)`: the next `limit_s` seconds belong to `phase`."""

    def __init__(self, rank, world):
        import threading
        self.rank, self.world = rank, world
        self.phase, self.deadline = "start", time.monotonic() + 600.0
        self._lock = threading.Lock()
        t = threading.Thread(target=self._run, daemon=True)
        t.start()

    def beat(self, phase, limit_s):
        with self._lock:
            self.phase, self.deadline = phase, time.monotonic() + limit_s

    def _run(self):
        while True:
            time.sleep(2.0)
            with self._lock:
                late = time.monotonic() > self.deadline
                phase = self.phase
            if late:
                fail_line(self.rank, self.world, f"rank {self.rank}: no progress in phase '{phase}' (watchdog)")
                os._exit(3)


def fail_line(rank, world, msg):
    """The JSON error line of a failed run (stdout, one write) -- parseable like the bench line."""
    sys.stdout.write("\n" + json.dumps({"metric": METRIC, "value": None, "unit": "MLUPS", "n_gpus": world,
                                        "error": msg, "rank": rank}) + "\n")
    sys.stdout.flush()


def main():
    argv = json.loads(os.environ["NSBENCH_ARGV"]) if "NSBENCH_ARGV" in os.environ and "WORLD_SIZE" in os.environ else None
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        world = max(world, 1)
    if os.environ.get("NSBENCH_LAUNCH_PROBE"):
        # (tests/test_bench_launch.py: the self-launch reached every rank; nothing touches a GPU)
        print(json.dumps({"probe_rank": rank, "world": world, "local_rank": local, "n": args.n, "re": args.re}),
              flush=True)
        return
    wd = Watchdog(rank, world) if world > 1 else None
    try:
        run(args, rank, world, local, wd)
    except Exception as e:   # a failed rank reports and exits non-zero (never hangs its peers silently)
        if world == 1:
            raise
        fail_line(rank, world, f"rank {rank}: {type(e).__name__}: {e}")
        os._exit(1)


def run(args, rank, world, local, wd):
    if os.environ.get("NSBENCH_FAIL_RANK") == str(rank):   # (tests/test_bench_launch.py: the failure path)
        raise RuntimeError("injected failure (NSBENCH_FAIL_RANK)")
    import torch
    import torch.distributed as dist

    import navierstokessolver_amd as nsa

    def beat(phase, limit_s):
        if wd:
            wd.beat(phase, limit_s)

    nccl_id = xport = None
    host = world > 1 and args.transport == "host"
    if world > 1:
        # gloo carries only the bootstrap (RCCL unique id), the barrier and the timing max;
        # the data path (ghost rows, residual / mean / min-max reductions) is RCCL in libnsgpu.so
        # -- or, --transport host, the same call sites through gloo on the host
        from navierstokessolver_amd.dist import TorchHostTransport, nccl_id as make_nccl_id
        dist.init_process_group("gloo", rank=rank, world_size=world)
        if host:
            xport = TorchHostTransport(dist)
        else:
            nccl_id = make_nccl_id(dist)

    n, re = args.n, args.re
    channel = args.case == "channel"
    if channel:
        nyc, h = n // 4, 4.0 / n
        dt = h / 8
        grid = nsa.rectangle(n, nyc, lx=4.0, ly=nyc * h, bc=[(0, 1.0), (2, 0.0), (4, 0.0), (2, 0.0)])
    elif args.case in ("stretched", "xstretched"):
        # (r6) the cavity on the reference's geometric spacing (ratio > 0), dt = 1/(8n) as the
        # uniform cavity (the smallest cell is ~(1 - ratio^(-n/2)) of h: CFL stays < 0.19 for ratio <= 1.0005 at 4096)
        nyc, dt = n, 1.0 / (8 * n)
        grid = nsa.rectangle(n, n, bc=[(nsa.NS_BC_WALL, 0.0), (nsa.NS_BC_WALL, 1.0), (nsa.NS_BC_WALL, 0.0),
                                       (nsa.NS_BC_WALL, 0.0)],
                             xratio=args.ratio, yratio=args.ratio if args.case == "stretched" else -1)
    else:
        nyc, dt = n, 1.0 / (8 * n)
        grid = nsa.cavity(n)
    device = 0 if host else local   # (the host transport's rehearsal: every rank on the one GPU)
    torch.cuda.set_device(device)
    beat("solver set-up (ncclCommInitRank)", 300.0)
    solver = nsa.GpuSolver(grid, dt, re, rtol=args.rtol, device=device, timing=True,
                           rank=rank, nranks=world, nccl_id=nccl_id, host_transport=xport)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # ns_step_async: each step's min/max monitor arrives with the next step (FluidSolver.cpp:554-560
    # prints every step; the values are the same, one call later), so the host enqueues step k+1's
    # K1 while step k's K5 runs instead of waiting for it; the last step's monitor is fetched
    # (ns_monitor) inside the timed region.  --sync-monitor: ns_step, one host sync at each step's end.
    step = solver.step if args.sync_monitor else solver.step_async
    for k in range(args.warmup):
        beat(f"warm-up step {k}", 120.0)
        step()
    if not args.sync_monitor:
        solver.monitor()
    barrier()
    t0 = time.perf_counter()
    stats = []
    for k in range(args.steps):
        beat(f"timed step {k}", 60.0)
        if args.time_every != 1:
            # (r6: steps 1, 1 + k, ...: the first timed step follows the warm-up's monitor() and runs the plain K1;
            # the others fold the previous step's K5 into K1, the K1 the bench line reports)
            solver.set_timing(args.time_every > 0 and k % args.time_every == min(1, args.steps - 1))
        stats.append(step())
    last_monitor = stats[-1] if args.sync_monitor else dict(zip(("umin", "umax", "vmin", "vmax"), solver.monitor()))
    barrier()
    elapsed = time.perf_counter() - t0
    beat("after the timed steps", 300.0)
    per_rank = None
    if world > 1:
        # every rank's own time, slab and per-step communication (the first real
        # multi-GPU line must say where its time went); `value` uses the max over ranks
        mine = {"rank": rank, "ms_per_step": elapsed / args.steps * 1e3, "rows": solver.i1 - solver.i0,
                "exchanges_per_step": sum(s["n_exchanges"] for s in stats) / args.steps,
                "collectives_per_step": sum(s["n_allreduces"] for s in stats) / args.steps,
                "x_link_bytes_per_step": sum(s["x_link_bytes"] for s in stats) / args.steps}
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        elapsed = max(p["ms_per_step"] for p in per_rank) * args.steps / 1e3

    K = args.steps
    timed_steps = K if args.time_every == 1 else (sum(1 for k in range(K) if k % args.time_every == min(1, K - 1))
                                                   if args.time_every > 0 else 0)
    cells = n * nyc
    cycles = sum(s["it_phi"] for s in stats)
    hsweeps = sum(s["it_u"] for s in stats)
    local_cells = (solver.i1 - solver.i0) * nyc
    timed = {"prolong": (sum(s["t_poisson_kernel_ms"] for s in stats), sum(s["n_poisson_kernels"] for s in stats)),
             "restrict": (sum(s["t_restrict_kernel_ms"] for s in stats), sum(s["n_restrict_kernels"] for s in stats)),
             "helmholtz": (sum(s["t_helm_kernel_ms"] for s in stats), sum(s["n_helm_kernels"] for s in stats)),
             "cycle": (sum(s["t_cycle_kernel_ms"] for s in stats), sum(s["n_cycle_kernels"] for s in stats)),
             "guess": (sum(s["t_guess_kernel_ms"] for s in stats), sum(s["n_guess_kernels"] for s in stats)),
             "rhs": (sum(s["t_rhs_kernel_ms"] for s in stats), sum(s["n_rhs_kernels"] for s in stats)),
             "k5": (sum(s["t_k5_kernel_ms"] for s in stats), sum(s["n_k5_kernels"] for s in stats)),
             "band": (sum(s["t_band_kernel_ms"] for s in stats), sum(s["n_band_kernels"] for s in stats))}
    for k in ("dct", "tri", "idct"):
        timed["fps_" + k] = (sum(s[f"t_fps_{k}_ms"] for s in stats), sum(s["n_fps_solves"] for s in stats))
    # the direct Poisson solve ran (one solve per step, no V-cycles) -- or, untimed, no restriction pass
    # (r5: the E-outflow channel takes the direct solve too, with its eliminated outflow row)
    direct = (any(s["n_fps_solves"] for s in stats) or
              (args.time_every == 0 and all(int(s["it_phi"]) == 1 for s in stats)))
    # finest-level sweeps: V(2,2) per cycle (the convergence check rides on each cycle's last pass)
    fine_sweeps = 4 * cycles
    # whole-step algorithmic bytes per cell: K1 64 + K3 24 + K5 40 + the phi
    # extrapolation 32 or 40; Helmholtz 24 per pass of one component (a pass = 2 or 3 sweeps: see
    # helm_passes); multigrid per solve `cycles` FUSE_R and `cycles` FUSE_P passes at 26 each on
    # the finest level (less the fused boundaries below), + 1/3 of that for the coarser levels
    # (each a quarter of the one above)
    min_rows = min(b - a for a, b in (nsa._lib.slab_range(n, world, r) for r in range(world)))
    hpasses = sum(helm_passes(int(s["it_u"]), min_rows) for s in stats)
    # the phi extrapolation: cubic (4 planes read + 1 written = 40 B/cell) after a solve that
    # needed >= 2 V-cycles, else quadratic (32); the solver's `need` may be one less than the
    # cycles a solve ran, so this counts the cubic at most one step too often
    prev_c = [None] + [int(s["it_phi"]) for s in stats[:-1]]
    extrap_bpc = sum(40 if (c is None or c >= 2) else 32 for c in prev_c) / K
    if any(s["n_guess_kernels"] for s in stats) or (args.time_every == 0 and world == 1 and not channel):
        # (r4, GIN: no k_axpby; the solve's first FUSE_R reads 4 / 3 history planes instead of phi:
        # + 24 / 16 B/cell on that pass, counted here in place of the extrapolation's 40 / 32)
        extrap_bpc -= 16
    # the Helmholtz wall bands (two k_helm_band launches) on the cells within 128 of a wall:
    # per launch u, v read 16 + rhs 16 + write 16 -> 96 B per band cell
    bw = max(32, min(n, nyc) // 32)   # the solver's band_w
    if min(n, nyc) > 4096:
        bw = 3 * min(n, nyc) // 64
    band_frac = 1.0 - max(n - 2 * bw, 0) * max(nyc - 2 * bw, 0) / float(n * nyc)
    # (r6) NSGPU_BAND6=1 (one rank, 6 band sweeps, <= 4096): ONE k_helm_band6 launch (48 B per band cell) + the
    # band cells' copy-back (32 B), timed as one interval -- 80 B per band cell per step instead of 2 x 48
    band6 = (world == 1 and min(n, nyc) <= 4096 and os.environ.get("NSGPU_BAND6", "0") != "0"
             and os.environ.get("NSGPU_BAND_SWEEPS", "6") == "6")
    band_bpc = (80 if band6 else 96) * band_frac
    # the finest level: a V-cycle whose output is not checked hands its prolongation pass to the next
    # cycle's restriction pass (one k_sweep4 pass of 28 B/cell instead of 26 + 26): cycles - checks
    # such boundaries per solve (one rank, multigrid)
    fused = sum(max(0, int(s["it_phi"]) - int(s["n_checks"])) for s in stats) if (world == 1 and not channel) else 0
    if not any(s["n_cycle_kernels"] for s in stats) and args.time_every:
        fused = 0   # (NSGPU_FUSE4=0: no boundary pass was timed, none ran)
    step_bpc = (64 + 24 + 40 + extrap_bpc + 2 * 24 * hpasses / K + band_bpc
                + (52 * (cycles - fused) + 28 * fused) / K + 52 * cycles / K / 3.0)
    if direct:
        # the direct solve: 56 B/cell (fps_* above; 72 in the three-pass form; 64 with K3 fused) per solve, plus its
        # residual check (phi 8 + b 8)
        # on the checked solves; no phi extrapolation (no initial guess)
        # (fused K3: no K3 pass (24), the DCT reads u*, v* (24 instead of 16) and stores rhs_phi for the
        # checked solves, 8 more there)
        checks = sum(int(s["n_checks"]) for s in stats)
        fused = FPS_FUSED and args.case != "xstretched"
        if not fused and FPS_FUSED:
            # (r6: an x-stretched grid takes the direct solve unfused -- K3 (24), the consistent rhs's two passes
            # (area sum 8 + fix 16), then the plain DCT of rhs_phi (16))
            KERNELS["fps_dct"] = ("k_fps_dct (direct Poisson solve: DCT-II of every row pair of the consistent "
                                  "rhs_phi - mean, Stockham FFT in LDS)", 16)
        fps_bpc = KERNELS["fps_dct"][1] + KERNELS["fps_tri"][1] + 16 + (0 if fused or not FPS_FUSED else 24 + 24)
        # (the channel's checked residual is the outflow operator's: apply 16 + b - y 24 + sums 8 = 48, vs 16)
        step_bpc = (64 + (0 if FPS_FUSED else 24) + 40 + 2 * 24 * hpasses / K + band_bpc + fps_bpc * cycles / K
                    + ((48 if channel else 16) + (8 if fused else 0)) * checks / K)
    if channel and not direct:
        # BiCGStab iteration (`cycles` = iterations): KV_P 32, two preconditioner applications
        # of (line extension 8 + FUSE_R 28 + FUSE_P 26, x 4/3 for the coarser levels) = 80 each,
        # two operator applications 24 + 16, KV_V 32, KV_T 24, KV_X 64 = 352; start-up (apply +
        # KV_INIT) 64; no phi extrapolation
        step_bpc = 64 + 24 + 40 + 64 + 2 * 24 * hpasses / K + 352 * cycles / K
    value = cells * K / elapsed / 1e6
    # (r6) ns_step_async with K5 deferred into the next step's K1: a step whose K1 applied the previous step's
    # correction (k5_deferred) moves 88 B/cell in K1 and runs no K5 of its own; the first timed step follows the
    # warm-up's solver.monitor() (which applied the pending correction), so its K1 is the plain one; the last
    # step's K5 runs once inside the timed region, in the closing solver.monitor()
    n_def = sum(int(s.get("k5_deferred", 0)) for s in stats)
    deferred = n_def > 0 and not args.sync_monitor
    if deferred:
        step_bpc += ((64 * (K - n_def) + 88 * n_def + 40) - (64 + 40) * K) / K
        timed["rhs"] = (sum(s["t_rhs_kernel_ms"] for s in stats if s["k5_deferred"]),
                        sum(s["n_rhs_kernels"] for s in stats if s["k5_deferred"]))

    # the north star's roofline kernel: one Jacobi sweep of this rank's slab (random phi, b;
    # 10 warm-up + 50 timed launches, HIP events), single rank only
    jacobi = jacobi32 = None
    if world == 1 and args.case == "cavity" and not args.no_jacobi:
        js = nsa.GpuSolver(nsa.cavity(n), dt, re, poisson=nsa.NS_POISSON_JACOBI, omega=1.0, device=device)
        js.fill_random(0x5EED)
        t = js.time_poisson(10, 50)
        jacobi = t["avg_ms"] * 1e-3
        try:
            js.fill_random(0x5EED)
            jacobi32 = js.time_poisson_fp32(10, 50)["avg_ms"] * 1e-3
        except AttributeError:   # a library without the fp32 sweep (A/B against an older build)
            jacobi32 = None
        js.close()
    if rank != 0:
        return
    # roofline.traffic: HBM bytes per launch from rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE
    # cannot be read inside this run); profiles/pmc_traffic.json names the run that measured them
    # and the sha256 of the libnsgpu.so it ran, and `traffic_source` says whether that is this
    # run's library
    traffic, tsrc = {}, None
    prof = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(prof) and world == 1:
        try:
            d = json.load(open(prof))
            if d.get("n") == n and args.case == "cavity":
                traffic = {k: v.get("kernel_bytes_per_launch") for k, v in d.get("kernels", {}).items()}
                tri = [traffic.get(k) for k in (("fps_t1", "fps_t2", "fps_t3")
                                                if os.environ.get("NSGPU_FPS_PASSES") == "3" else ("fps_t1b", "fps_t2b"))]
                if all(x is not None for x in tri):
                    traffic["fps_tri"] = sum(tri)
                traffic["fps_dct"] = traffic.get("fps_dct_div") if FPS_FUSED else traffic.get("fps_dct")
                src = dict(d.get("source") or {})
                src["file"] = "profiles/pmc_traffic.json"
                src["same_library_as_this_run"] = (src.get("libnsgpu_sha16") is not None and
                                                   src.get("libnsgpu_sha16") == _sha16(nsa._lib.LIB_PATH))
                tsrc = src
        except Exception:
            traffic = {}

    def roof(key, label, bpc, avg_s, launches):
        achieved = bpc * local_cells / avg_s / 1e9
        tkey = "rhs_sc" if (key == "rhs" and deferred) else key   # (r6: K1 with the deferred K5 folded in)
        r = {"bound": "hbm", "kernel": label, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": achieved / HBM_PEAK_GBS, "traffic": traffic.get(tkey), "avg_kernel_us": avg_s * 1e6,
             "launches_timed": launches, "bytes_per_launch": bpc * local_cells, "bytes_per_cell": bpc}
        if r["traffic"] is not None:
            r["traffic_source"] = tsrc
        return r

    kern = {}
    for key, (label, bpc) in KERNELS.items():
        if key == "band":
            bpc = 48 * band_frac
            if band6:
                label, bpc = ("k_helm_band6 + k_band_copy (Helmholtz wall bands: 6 RB-SOR sweeps of u, v on the cells "
                              "near a wall in one launch of 64 x 64 tiles with their 12-cell cone in LDS, then the "
                              "band cells' copy-back)", band_bpc)
        if key == "rhs" and deferred:
            # (r6) K1 with the previous step's K5 folded in (k_rhs_sc): read u*, v*, phi^n, cu, cv 40 + write u, v,
            # cu, cv, ru, rv 48
            label, bpc = ("k_rhs_sc (K1 + the previous step's K5 folded in: CorrectVelocities on the fly, then "
                          "ConstructRHS_V: AB2 MUSCL/Rusanov convection + CN-explicit diffusion + wall terms)", 88)
        ms, cnt = timed[key]
        if cnt:
            kern[key] = roof(key, label, bpc, ms / cnt / 1e3, cnt)
            # (launches are timed on every --time-every'th step: scale to all K steps)
            kern[key]["ms_per_step"] = ms / max(1, timed_steps)
            if key == "rhs" and deferred:   # (one K1 per step; its average over the deferred steps timed)
                kern[key]["ms_per_step"] = ms / cnt
    single = [k for k in kern if k in SINGLE_LAUNCH]
    dominant = max(single, key=lambda k: kern[k]["ms_per_step"]) if single else None
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "MLUPS",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (lid-driven cavity from rest, no input files)",
        "config": {"workload": (f"{n}x{nyc} channel (inlet W, NEUMANN outflow E), Re={re:g}, dt=h/8, fp64, "
                                + ("direct Poisson solve (DCT along y; the outflow row eliminated into tridiagonal "
                                   "recurrences along x, mode 0 in the projected sense; residual checked on every "
                                   "16th solve)" if direct else
                                   "BiCGStab Poisson with the line-closure V-cycle preconditioner")
                                + f" + RB-SOR Helmholtz, both to rtol {args.rtol:g}") if channel else
                               (f"{n}x{n} lid-driven cavity"
                                + (f" on a stretched grid (ratio {args.ratio:g} along x"
                                   + (" and y)" if args.case == "stretched" else ", y uniform)")
                                   if args.case != "cavity" else "")
                                + f", Re={re:g}, dt=1/{8 * n}, fp64, "
                                + ("direct Poisson solve (DCT along y + tridiagonal recurrences along x; residual "
                                   "checked on every 16th solve)" if direct else
                                   "multigrid Poisson (RB-GS smoother; V-cycles to rtol)")
                                + f" + RB-SOR Helmholtz, both to rtol {args.rtol:g}"),
                   "case": args.case, "nx": n, "ny": nyc, "re": re, "dt": dt, "parallelism": f"x-slab x{world}",
                   "ratio": args.ratio if args.case in ("stretched", "xstretched") else None,
                   "step_api": "ns_step" if args.sync_monitor else "ns_step_async",
                   "transport": ("none (one rank)" if world == 1 else
                                 "RCCL over xGMI, one GPU per rank" if not host else
                                 f"host (gloo): a rehearsal of the multi-rank path with all {world} ranks on one GPU "
                                 "-- functional evidence, not a scaling number"),
                   "local_rows_rank0": solver.i1 - solver.i0},
        "ranks": per_rank,
        "monitor_last_step": {k: last_monitor[k] for k in ("umin", "umax", "vmin", "vmax")},
        ("poisson_direct_solves_per_s" if direct else "poisson_bicgstab_its_per_s" if channel else
         "poisson_vcycles_per_s"): cycles / elapsed,
        ("poisson_direct_solves_per_step" if direct else "poisson_bicgstab_its_per_step" if channel else
         "poisson_vcycles_per_step"): cycles / K,
        "poisson_fine_sweeps_per_s": fine_sweeps / elapsed,
        "poisson_fine_sweeps_per_step": fine_sweeps / K,
        "helmholtz_sweeps_per_step": hsweeps / K,
        "helmholtz_passes_per_step": 2 * hpasses / K,
        "poisson_checks_per_step": sum(s["n_checks"] for s in stats) / K,
        "roofline": kern.get(dominant),
        "step_roofline": {"bound": "hbm", "bytes_per_cell": step_bpc, "bytes_per_step": step_bpc * cells,
                          "achieved": step_bpc * cells / (elapsed / K) / 1e9, "peak": HBM_PEAK_GBS * world,
                          "unit": "GB/s", "frac": step_bpc * cells / (elapsed / K) / 1e9 / (HBM_PEAK_GBS * world),
                          "note": "every kernel's algorithmic bytes of a step / ms_per_step (host syncs, "
                                  "kernel boundaries and latency-bound coarse levels included)"},
        "kernels": dict(kern),
    }
    # (r6) the share of the step's wall time the timed kernels account for (their per-step ms over ms_per_step;
    # the unlisted rest: the scans / carries of fps_tri are inside it, the small reductions and kernel boundaries
    # are not)
    line["kernels_ms_per_step"] = sum(k["ms_per_step"] for k in kern.values())
    line["kernels_share_of_step"] = line["kernels_ms_per_step"] / (elapsed / K * 1e3)
    if jacobi is not None:
        line["kernels"]["jacobi_sweep"] = roof("jacobi_sweep", JACOBI_LABEL, SWEEP_BYTES_PER_CELL, jacobi, 50)
    if jacobi32 is not None:
        line["kernels"]["jacobi_sweep_fp32"] = roof("jacobi_sweep_fp32", JACOBI32_LABEL, SWEEP32_BYTES_PER_CELL,
                                                    jacobi32, 50)
    if channel or direct:
        for k in ("poisson_fine_sweeps_per_s", "poisson_fine_sweeps_per_step"):
            line.pop(k)
    if channel:
        line["data"] = "synthetic (channel from rest, uniform inlet, no input files)"
    if world > 1:
        line["comm"] = {"collectives_per_step": sum(s["n_allreduces"] for s in stats) / K,
                        "exchanges_per_step": sum(s["n_exchanges"] for s in stats) / K,
                        "x_link_bytes_per_step": sum(s["x_link_bytes"] for s in stats) / K,
                        "rccl_version": _rccl_version(torch) if not host else None,
                        "note": "collectives = all-reduces + allgathers issued per step by rank 0 (r5: the "
                                "Helmholtz check's scalar bus and the direct solve's one allgather -- two with "
                                "NSGPU_FPS_ONEGATHER=0 -- + 1 on a checked solve); exchanges = ghost-row send/recv "
                                "groups"}
    else:
        line.pop("ranks")
    if world == 1 and not args.no_cpu and args.case == "cavity" and n & (n - 1) == 0:
        try:
            state = {k: solver.get(a).ravel() for k, a in (("u", nsa.NS_ARR_U), ("v", nsa.NS_ARR_V),
                                                           ("phi", nsa.NS_ARR_PHI), ("cu", nsa.NS_ARR_CU),
                                                           ("cv", nsa.NS_ARR_CV))}
            # the GPU's own next step from that state (after the timed region), for the oracle to match
            st_next = solver.step()
            gpu_next = {"u": solver.get(nsa.NS_ARR_U).ravel(), "v": solver.get(nsa.NS_ARR_V).ravel(),
                        "monitor": [st_next[k] for k in ("umin", "umax", "vmin", "vmax")]}
            line["cpu_baseline"] = cpu_baseline(n, re, dt, solver.omega_v, solver.mg_omega, state, gpu_next)
            line["parity_vs_oracle"] = line["cpu_baseline"].get("parity")
        except Exception as e:  # the baseline must never hide the GPU line
            line["cpu_baseline"] = {"error": repr(e)}
    # one write: the line cannot be split by other output of this process
    sys.stdout.write("\n" + json.dumps(line) + "\n")
    sys.stdout.flush()


if __name__ == "__main__":
    main()
