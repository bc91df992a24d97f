"""Strip height x size for the single and the two-sweep RB pass (per-sweep us), one process."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import navierstokessolver_amd as nsa
for n in (4096, 2048, 1024, 512, 256):
    for pairs in (0, 1):
        line = []
        for L in (0, 4, 8, 16, 32, 48, 64):
            if pairs and L == 4: continue
            os.environ["NSGPU_STRIP_ROWS"] = str(L)   # 0 = the residency rule
            if pairs: os.environ["NSGPU_TIME_PAIRS"] = "1"
            else: os.environ.pop("NSGPU_TIME_PAIRS", None)
            gs = nsa.GpuSolver(nsa.cavity(n), 1.0 / (8 * n), 1000.0, poisson=nsa.NS_POISSON_RBSOR, omega=1.0)
            gs.fill_random(1)
            t = min(gs.time_poisson(5, 20)["avg_ms"] for _ in range(2)) * 1e3 / (2 if pairs else 1)
            gs.close()
            line.append(f"{'auto' if L == 0 else 'L%d' % L}={t:6.1f}")
        print(n, "rb2" if pairs else "rb1", " ".join(line), "us/sweep", flush=True)
