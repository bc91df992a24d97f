"""Strip-height sweep of the RB smoother over multigrid level sizes (one process)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import navierstokessolver_amd as nsa
for n in (4096, 2048, 1024, 512, 256):
    line = []
    for L in (4, 8, 16, 32, 64):
        os.environ["NSGPU_STRIP_ROWS"] = str(L)
        gs = nsa.GpuSolver(nsa.cavity(n), 1.0 / (8 * n), 1000.0, poisson=nsa.NS_POISSON_RBSOR, omega=1.0)
        gs.fill_random(1)
        t = min(gs.time_poisson(5, 30)["avg_ms"] for _ in range(2)) * 1e3
        gs.close()
        line.append(f"L{L}={t:7.1f}us({24*n*n/(t*1e-6)/1e9:5.0f}GB/s)")
    print(n, " ".join(line), flush=True)
