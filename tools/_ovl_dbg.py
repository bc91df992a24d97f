import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
os.environ["NSGPU_PAIR_MIN_CELLS"] = "0"
os.environ["NSGPU_STRIP_ROWS"] = "16"
import navierstokessolver_amd as nsa
n, ny = 192, 160
res = {}
for lb in ("0", "1"):
    os.environ["NSGPU_RCCL_LOOPBACK"] = lb
    gs = nsa.GpuSolver(nsa.rectangle(n, ny), 1.0 / (8 * n), 100.0, rtol=1e-11, device=0)
    st = [gs.step() for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1)]
    res[lb] = (gs.fields(), [(s["it_u"], s["it_phi"]) for s in st])
    gs.close()
print(res["0"][1], res["1"][1])
for k, name in enumerate(("u", "v", "phi")):
    a, b = res["0"][0][k], res["1"][0][k]
    d = np.abs(a - b)
    rows = np.nonzero(d.max(axis=1) > 0)[0]
    print(name, d.max(), "rows differing:", rows[:20], len(rows), "mean diff", float((a - b).mean()))
