"""A/B: single RB sweep vs the two-sweep pass (per sweep), Jacobi, at several sizes, one process."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import navierstokessolver_amd as nsa
for n in [int(x) for x in sys.argv[1:]] or [4096, 2048, 1024]:
    res = {}
    for rnd in range(2):
        for name, pairs, solver, L in [("rb1", 0, 0, 0), ("rb2", 1, 0, 0), ("rb2-L16", 1, 0, 16), ("rb2-L64", 1, 0, 64),
                                       ("jacobi", 0, 1, 0)]:
            os.environ.pop("NSGPU_TIME_PAIRS", None); os.environ.pop("NSGPU_STRIP_ROWS", None)
            if pairs: os.environ["NSGPU_TIME_PAIRS"] = "1"
            if L: os.environ["NSGPU_STRIP_ROWS"] = str(L)
            gs = nsa.GpuSolver(nsa.cavity(n), 1.0 / (8 * n), 1000.0, poisson=solver, omega=1.0)
            gs.fill_random(3)
            t = gs.time_poisson(5, 30)["avg_ms"] * 1e3 / (2 if pairs else 1)
            gs.close()
            res.setdefault(name, []).append(t)
    print(n, "  ".join(f"{k}={min(v):6.1f}us/sweep({24*n*n/(min(v)*1e-6)/1e9:5.0f}GB/s-eq)" for k, v in res.items()), flush=True)
