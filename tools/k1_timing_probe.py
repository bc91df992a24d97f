"""K1 event timing vs the kernel trace (r6: k_rhs_sc read 286 us by the bench's dispatch-stamped events and 338 us in
rocprofv3's trace).  Runs 5 + 20 async 4096^2 steps with every step's kernels timed and prints each step's K1 (and
the Helmholtz / direct-solve intervals); run it plain and under rocprofv3 --kernel-trace to compare.
    python tools/k1_timing_probe.py [n]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import navierstokessolver_amd as nsa  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
s = nsa.GpuSolver(nsa.cavity(n), 1.0 / (8 * n), 1000.0, timing=True, device=0)
for _ in range(5):
    s.step_async()
s.monitor()
torch.cuda.synchronize()
t0 = time.perf_counter()
st = [s.step_async() for _ in range(20)]
s.monitor()
torch.cuda.synchronize()
el = time.perf_counter() - t0
k1 = [x["t_rhs_kernel_ms"] * 1e3 for x in st]
print(f"ms/step {el / 20 * 1e3:.3f}  deferred {[x['k5_deferred'] for x in st].count(1)}/20")
print("K1 us per step:", " ".join(f"{v:.1f}" for v in k1))
print(f"K1 mean {sum(k1) / len(k1):.1f} us; band {sum(x['t_band_kernel_ms'] for x in st) / 20 * 1e3:.1f} us/step; "
      f"K5 {sum(x['t_k5_kernel_ms'] for x in st) / max(1, sum(x['n_k5_kernels'] for x in st)) * 1e3:.1f} us")
