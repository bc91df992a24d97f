"""Strong-scaling projection for configs[3] (8192^2 over 1/2/4/8 MI355X) from ONE GPU.

For P = 1 the single-rank step is timed as bench.py does (ns_step_async, W warm-up + K timed
steps).  For P > 1 one rank's share is timed as a VIRTUAL slab (NSGPU_RCCL_LOOPBACK=1,
nranks = P, no ncclUniqueId; ns_solver.cpp): the process builds rank r's slab (an interior
rank), its hierarchy (distributed levels + the replicated coarse levels every rank runs) and
issues every RCCL group of the real step -- ghost-row send/recv pairs on the comm stream
overlapped with the interior strips, the agglomeration gather, the all-reduces -- with itself
as every peer.  What this does not contain is the xGMI part: the transfer of a 64 KB-per-row
message between two GPUs and the latency of a P-GPU all-reduce.  The projection adds those
as stated per-event costs (--allreduce-us, --exchange-us), counted from the step's own
n_allreduces / n_exchanges.  Reductions cover the slab only, so the slab's iteration counts
can differ from the global solve's by a cycle; both are printed.

  python tools/slab_projection.py [--n 8192] [--ranks 1,2,4,8] [--warmup 5] [--steps 10]
  python tools/slab_projection.py --weak-rows 2048 --ny 8192      # configs[3]'s weak scaling

--weak-rows W: weak scaling, W rows per rank on a (W P) x ny grid (configs[3]: 2048 x 8192 per GPU).
For each P the single-rank run of the global (W P) x ny grid gives the replayed counts (its own
problem: the grid grows with P); the row reports the virtual slab's ms/step, the projected one, and
the weak-scaling efficiency t(P = 1) / t(P).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(n, P, warmup, steps, re, replay=None, ny=None):
    """One configuration; P > 1 replays the single-rank run's per-step (Helmholtz sweeps,
    V-cycles) sequence `replay` (NSGPU_VIRTUAL_ITERS): the same work per step as the global
    solve, which the 8-slab tests show the P-rank run reproduces exactly."""
    import navierstokessolver_amd as nsa
    ny = ny or n
    dt = 1.0 / (8 * max(n, ny))
    kw = {}
    if P > 1:
        os.environ["NSGPU_RCCL_LOOPBACK"] = "1"
        os.environ["NSGPU_VIRTUAL_ITERS"] = ",".join(f"{h}:{c}" for h, c in replay)
        kw = dict(rank=P // 2, nranks=P)
    grid = nsa.cavity(n) if ny == n else nsa.rectangle(n, ny, lx=1.0, ly=ny / n)
    gs = nsa.GpuSolver(grid, dt, re, device=0, **kw)
    os.environ.pop("NSGPU_RCCL_LOOPBACK", None)
    os.environ.pop("NSGPU_VIRTUAL_ITERS", None)
    seq = []
    for _ in range(warmup):
        s = gs.step_async()
        seq.append((s["it_u"], s["it_phi"]))
    gs.monitor()
    t0 = time.perf_counter()
    st = [gs.step_async() for _ in range(steps)]
    gs.monitor()
    t = (time.perf_counter() - t0) / steps
    seq += [(s["it_u"], s["it_phi"]) for s in st]
    i0, i1 = gs.i0, gs.i1
    gs.close()
    return seq, {"P": P, "nx": n, "ny": ny, "rank": P // 2 if P > 1 else 0, "rows": i1 - i0, "ms_per_step": t * 1e3,
            "vcycles_per_step": sum(s["it_phi"] for s in st) / steps,
            "helm_sweeps_per_step": sum(s["it_u"] for s in st) / steps,
            "exchanges_per_step": sum(s["n_exchanges"] for s in st) / steps,
            "allreduces_per_step": sum(s["n_allreduces"] for s in st) / steps,
            "link_mb_per_step": sum(s.get("x_link_bytes", 0.0) for s in st) / steps / 1e6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--re", type=float, default=1000.0)
    ap.add_argument("--replay", default="", help="h:c,... per-step counts for P > 1 instead of a P = 1 run's")
    ap.add_argument("--allreduce-us", type=float, default=25.0,
                    help="assumed latency of one small (<= 4 doubles) RCCL all-reduce over P GPUs (xGMI)")
    ap.add_argument("--exchange-us", type=float, default=5.0,
                    help="assumed exposed cost of one ghost-row exchange group beyond the self-copy measured "
                         "here (64 KB per row per side over one 153 GB/s-class xGMI link, overlapped with the "
                         "interior strips)")
    ap.add_argument("--link-gbs", type=float, default=50.0,
                    help="assumed sustained one-direction bandwidth of one GPU-to-GPU xGMI link (GB/s): the "
                         "upper projection adds every byte the rank sends over its busiest link (ghost rows "
                         "and agglomeration gathers, ns_stats.x_link_bytes) as exposed transfer time")
    ap.add_argument("--weak-rows", type=int, default=0, help="weak scaling: rows per rank (grid (W P) x ny)")
    ap.add_argument("--ny", type=int, default=0, help="columns of the weak-scaling grid (default --n)")
    a = ap.parse_args()
    rows = []
    if a.weak_rows:
        ny = a.ny or a.n
        t1 = None
        for P in (int(x) for x in a.ranks.split(",")):
            n = a.weak_rows * P
            seq, r1 = run(n, 1, a.warmup, a.steps, a.re, ny=ny)   # the global problem's counts
            if P == 1:
                r = r1
            else:
                _, r = run(n, P, a.warmup, a.steps, a.re, seq, ny=ny)
            extra = 0.0 if P == 1 else (r["allreduces_per_step"] * a.allreduce_us + r["exchanges_per_step"] * a.exchange_us) * 1e-3
            r["projected_ms_per_step"] = r["ms_per_step"] + extra
            r["projected_mlups"] = n * ny / (r["projected_ms_per_step"] * 1e-3) / 1e6
            r["single_gpu_ms_per_step_of_this_grid"] = r1["ms_per_step"]
            t1 = t1 or r["projected_ms_per_step"]
            r["weak_efficiency"] = t1 / r["projected_ms_per_step"]
            rows.append(r)
            print(json.dumps(r), flush=True)
        print(json.dumps({"weak_rows": a.weak_rows, "ny": ny, "assumptions": {"allreduce_us": a.allreduce_us,
                          "exchange_us": a.exchange_us},
                          "weak_efficiency": {r["P"]: round(r["weak_efficiency"], 3) for r in rows}}), flush=True)
        return
    replay = [tuple(int(x) for x in t.split(":")) for t in a.replay.split(",")] if a.replay else None
    for P in (int(x) for x in a.ranks.split(",")):
        if P > 1 and replay is None:
            replay, _ = run(a.n, 1, a.warmup, a.steps, a.re)
        seq, r = run(a.n, P, a.warmup, a.steps, a.re, replay)
        if P == 1:
            replay = seq
        extra = 0.0 if P == 1 else (r["allreduces_per_step"] * a.allreduce_us + r["exchanges_per_step"] * a.exchange_us) * 1e-3
        r["projected_ms_per_step"] = r["ms_per_step"] + extra
        r["projected_mlups"] = a.n * a.n / (r["projected_ms_per_step"] * 1e-3) / 1e6
        # upper bound: every link byte exposed at --link-gbs (no overlap with the interior strips)
        r["projected_ms_per_step_link"] = r["projected_ms_per_step"] + (0.0 if P == 1 else r["link_mb_per_step"] / a.link_gbs)
        rows.append(r)
        print(json.dumps(r), flush=True)
    base = rows[0]["projected_ms_per_step"] if rows and rows[0]["P"] == 1 else None
    if base:
        for r in rows:
            r["projected_speedup"] = base / r["projected_ms_per_step"]
            r["projected_speedup_link"] = base / r["projected_ms_per_step_link"]
        print(json.dumps({"n": a.n, "assumptions": {"allreduce_us": a.allreduce_us, "exchange_us": a.exchange_us,
                                                    "link_gbs": a.link_gbs,
                                                    # (r5) the measured share's collectives: RCCL's 1-rank loopback
                                                    # kernels, or device copies (NSGPU_VIRTUAL_COPY=1)
                                                    "virtual_collectives": "copy" if os.environ.get(
                                                        "NSGPU_VIRTUAL_COPY", "0") not in ("", "0") else "rccl-loopback"},
                          "speedup": {r["P"]: round(r["projected_speedup"], 2) for r in rows},
                          "speedup_link_bytes_exposed": {r["P"]: round(r["projected_speedup_link"], 2) for r in rows}}),
              flush=True)


if __name__ == "__main__":
    main()
