"""Per-step Helmholtz / Poisson counts and residuals of the 4096^2 cavity from rest; run with
NSGPU_VERBOSE=1 for the solvers' residual histories on stderr.  python tools/verbose_steps.py"""
import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import navierstokessolver_amd as nsa
n = 4096
gs = nsa.GpuSolver(nsa.cavity(n), 1.0/(8*n), 1000.0, device=0)
for k in range(int(os.environ.get("STEPS", "14"))):
    st = gs.step()
    print("step", k + 1, st["it_u"], st["it_phi"], st["res_u"], st["res_v"], flush=True)
