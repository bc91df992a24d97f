"""Phase timing of the one-workgroup LDS coarse V-cycle (k_coarse_vcycle) from a diagnostic
build (CV_DIAG=1: thread 0 stamps the 100 MHz wall clock at each phase boundary):
  make -C navierstokessolver_amd/csrc cvdiag                                      (CPU)
  NSGPU_LIB=abl/libnsgpu_cvdiag.so python tools/cv_diag.py [n]                                   (GPU)
Runs a few cavity steps (the last launch's stamps are read back) and prints each phase in us."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import navierstokessolver_amd as nsa

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
s = nsa.GpuSolver(nsa.cavity(n), 1.0 / (8 * n), 1000.0, device=0)
for _ in range(4):
    s.step()
lib = ctypes.CDLL(os.environ["NSGPU_LIB"])
buf = (ctypes.c_ulonglong * 64)()
assert lib.nsg_cv_diag(buf) == 0
t = np.array(buf[:22], dtype=np.float64)
names = {0: "start", 1: "layout + load", 2: "tables"}
names.update({3 + k: f"down level {k} (pre + restrict)" for k in range(9)})
names[12] = "coarsest solve"
names.update({13 + k: f"up level {k} (prolong + post)" for k in range(8)})
names[21] = "store"
prev = t[0]
for k in (1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 20, 19, 18, 17, 16, 15, 14, 13, 21):
    if t[k] == 0 or t[k] < t[0]:
        continue
    print(f"{names[k]:32s} {(t[k] - prev) * 0.01:7.2f} us")
    prev = t[k]
print(f"{'total':32s} {(t[21] - t[0]) * 0.01:7.2f} us")
