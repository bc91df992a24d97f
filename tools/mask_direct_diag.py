"""Masked-domain Poisson (BiCGStab preconditioned by the bounding box's V-cycle): iterations per step
and the full-step errors against the oracle, with the exact coarsest-level solve (default) and with
round 3's LDS V-cycle (NSGPU_DIRECT_CELLS=0).  python tools/mask_direct_diag.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    from polygons import ALL
    from test_gpu_mask import pair
    import navierstokessolver_amd as gpu
    from oracle import OSolver
    for name, steps, re in (("step", 15, 100.0), ("lshape", 12, 400.0), ("split", 10, 100.0)):
        P = ALL[name]
        n = max(P["xspec"][-1][2], P["yspec"][-1][2])
        dt = 1.0 / (16 * n)
        og, gs, m = pair(gpu, name, dt, re)
        osv = OSolver(og, dt, re, rtol=1e-13)
        its = []
        for _ in range(steps):
            st = gs.step(); osv.step(); its.append(st["it_phi"])
        ref = osv.get()
        u, v, phi = (a.ravel() for a in gs.fields())
        p, q = phi[m] - phi[m].mean(), ref["phi"] - ref["phi"].mean()
        print(os.environ.get("NSGPU_DIRECT_CELLS", "default"), name, "its", its,
              "du %.2e" % np.max(np.abs(u[m] - ref["u"])), "ephi %.2e" % (np.linalg.norm(p - q) / np.linalg.norm(q)), flush=True)
    sys.exit(0)
for dc in (None, "0"):
    env = dict(os.environ)
    if dc is not None:
        env["NSGPU_DIRECT_CELLS"] = dc
    subprocess.run([sys.executable, os.path.abspath(__file__), "child"], env=env, check=True)
