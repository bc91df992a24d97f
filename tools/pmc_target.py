"""Profiling target: only the finest-level Poisson smoother (k_sweep<Poisson,RB>) at n^2,
so rocprofv3 --pmc passes see one kernel.  python tools/pmc_target.py [n] [iters]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import navierstokessolver_amd as nsa
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
it = int(sys.argv[2]) if len(sys.argv) > 2 else 50
gs = nsa.GpuSolver(nsa.cavity(n), 1.0 / (8 * n), 1000.0, poisson=nsa.NS_POISSON_RBSOR, omega=1.0)
gs.fill_random(0x5EED)
t = gs.time_poisson(5, it)
print(f"n={n} avg kernel {t['avg_ms']*1e3:.1f} us", flush=True)
