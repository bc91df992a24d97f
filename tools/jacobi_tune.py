"""Jacobi sweep (the north star's roofline kernel) at 4096^2 vs streaming-strip height and
store / load policy: one GpuSolver per setting, 10 warm-up + 50 timed sweeps (HIP events)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import navierstokessolver_amd as nsa

n = 4096
for env in [{}, {"NSGPU_STRIP_ROWS": "8"}, {"NSGPU_STRIP_ROWS": "16"}, {"NSGPU_STRIP_ROWS": "32"},
            {"NSGPU_STRIP_ROWS": "64"}, {"NSGPU_NT_LOADS": "1"}, {"NSGPU_NT_STORES": "0"}, {"NSGPU_ALT_DIR": "0"}]:
    for k in ("NSGPU_STRIP_ROWS", "NSGPU_NT_LOADS", "NSGPU_NT_STORES", "NSGPU_ALT_DIR"):
        os.environ.pop(k, None)
    os.environ.update(env)
    js = nsa.GpuSolver(nsa.cavity(n), 1.0 / (8 * n), 1000.0, poisson=nsa.NS_POISSON_JACOBI, omega=1.0, device=0)
    js.fill_random(0x5EED)
    t = js.time_poisson(10, 50)
    js.close()
    us = t["avg_ms"] * 1e3
    print(f"{env or 'default'}: {us:.1f} us  {24 * n * n / us / 1e3:.0f} GB/s", flush=True)
