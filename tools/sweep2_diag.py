"""Time the two-sweep streaming pass (k_sweep2, Poisson operator, no residual) at 4096^2 with
HIP events: 10 warm-up + 50 timed passes on random input (ns_time_poisson, NSGPU_TIME_PAIRS=1).
Run against diagnostic builds (SWEEP2_DIAG=1: the memory stream only; 2: no shuffles) under
NSGPU_LIB to split the pass's time into memory stream and compute.
  NSGPU_LIB=abl/libnsgpu_diag1.so python tools/sweep2_diag.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NSGPU_TIME_PAIRS"] = "1"
import navierstokessolver_amd as nsa

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
s = nsa.GpuSolver(nsa.cavity(n), 1.0 / (8 * n), 1000.0, poisson=nsa.NS_POISSON_RBSOR, device=0)
s.fill_random(0x5EED)
t = s.time_poisson(10, 50)
us = t["avg_ms"] * 1e3
print(f"{os.environ.get('NSGPU_LIB', 'default')}: k_sweep2 pass {us:.1f} us = {24 * n * n / us / 1e3:.0f} GB/s algorithmic")
