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
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(n, P, warmup, steps, re, replay=None):
    """One configuration; P > 1 replays the single-rank run's per-step (Helmholtz sweeps,
    V-cycles) sequence `replay` (NSGPU_VIRTUAL_ITERS): the same work per step as the global
    solve, which the 8-slab tests show the P-rank run reproduces exactly."""
    import navierstokessolver_amd as nsa
    dt = 1.0 / (8 * n)
    kw = {}
    if P > 1:
        os.environ["NSGPU_RCCL_LOOPBACK"] = "1"
        os.environ["NSGPU_VIRTUAL_ITERS"] = ",".join(f"{h}:{c}" for h, c in replay)
        kw = dict(rank=P // 2, nranks=P)
    gs = nsa.GpuSolver(nsa.cavity(n), dt, re, device=0, **kw)
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
    return seq, {"P": P, "rank": P // 2 if P > 1 else 0, "rows": i1 - i0, "ms_per_step": t * 1e3,
            "vcycles_per_step": sum(s["it_phi"] for s in st) / steps,
            "helm_sweeps_per_step": sum(s["it_u"] for s in st) / steps,
            "exchanges_per_step": sum(s["n_exchanges"] for s in st) / steps,
            "allreduces_per_step": sum(s["n_allreduces"] for s in st) / steps}


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
    a = ap.parse_args()
    rows = []
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
        rows.append(r)
        print(json.dumps(r), flush=True)
    base = rows[0]["projected_ms_per_step"] if rows and rows[0]["P"] == 1 else None
    if base:
        for r in rows:
            r["projected_speedup"] = base / r["projected_ms_per_step"]
        print(json.dumps({"n": a.n, "assumptions": {"allreduce_us": a.allreduce_us, "exchange_us": a.exchange_us},
                          "speedup": {r["P"]: round(r["projected_speedup"], 2) for r in rows}}), flush=True)


if __name__ == "__main__":
    main()
