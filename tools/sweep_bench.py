"""A/B timing of the Poisson sweep kernels at one grid size, all variants in ONE process
(cdna_hip_programming.md 5.4 rule 24).  Prints avg kernel microseconds and GB/s at the
algorithmic 24 B/cell."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import navierstokessolver_amd as nsa

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
variants = []
for impl in ("stream", "tiled"):
    for solver in (nsa.NS_POISSON_RBSOR, nsa.NS_POISSON_JACOBI):
        rows = (16, 32, 64, 128) if impl == "stream" else (0,)
        for L in rows:
            variants.append((impl, solver, L))
res = {}
for rnd in range(2):
    for impl, solver, L in variants:
        os.environ["NSGPU_SWEEP"] = impl
        if L:
            os.environ["NSGPU_STRIP_ROWS"] = str(L)
        gs = nsa.GpuSolver(nsa.cavity(n), 1.0 / (8 * n), 1000.0, poisson=solver, omega=1.9 if solver == 0 else 1.0)
        gs.fill_random(0x5EED)
        t = gs.time_poisson(10, iters)
        gs.close()
        key = f"{impl}-{'rb' if solver == 0 else 'jacobi'}-L{L}"
        res.setdefault(key, []).append(t["avg_ms"])
for k, v in res.items():
    us = min(v) * 1e3
    print(f"{k:24s} {us:9.1f} us  {24 * n * n / (us * 1e-6) / 1e9:8.1f} GB/s  (rounds: {', '.join(f'{x*1e3:.1f}' for x in v)})")
