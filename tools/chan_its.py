"""Per-step Poisson BiCGStab iteration counts of the outflow channel (A/B of the apply / cell kernels):
   TAG=x python tools/chan_its.py nx ny steps"""
import os, sys, json
sys.path.insert(0, "/root/repo")
import numpy as np
import navierstokessolver_amd as nsa
BC_CHANNEL = [(0, 1.0), (2, 0.0), (4, 0.0), (2, 0.0)]
nx, ny = int(sys.argv[1]), int(sys.argv[2])
h = 4.0 / nx
g = nsa.rectangle(nx, ny, lx=4.0, ly=ny * h, bc=BC_CHANNEL)
gs = nsa.GpuSolver(g, h / 8, 1000.0)
its = []; res = []
for k in range(int(sys.argv[3])):
    st = gs.step()
    its.append(st["it_phi"]); res.append(st["res_phi"])
u, v, phi = gs.fields()
print(os.environ.get("TAG", ""), "its", its, "sum", sum(its), "u0", float(u.ravel()[12345]), "maxres", max(res), flush=True)
gs.close()
