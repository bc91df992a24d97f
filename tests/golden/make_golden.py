"""Generate the committed oracle fixtures (small .npz) -- run from the repo root:
    python tests/golden/make_golden.py
Each case: a rectangle, its BCs, dt, Re, steps; stored: per-step (umin, umax, vmin, vmax)
and the final u, v, phi of the converged oracle (oracle/ns_oracle.c, rtol 1e-13)."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
from oracle import OGrid, OSolver  # noqa: E402

CASES = [
    dict(name="cavity16_re100", nx=16, ny=16, bc=[[2, 0.0], [2, 1.0], [2, 0.0], [2, 0.0]], xratio=-1, yratio=-1,
         dt=1 / 128, re=100.0, steps=10),
    dict(name="cavity32_re400", nx=32, ny=32, bc=[[2, 0.0], [2, 1.0], [2, 0.0], [2, 0.0]], xratio=-1, yratio=-1,
         dt=1 / 256, re=400.0, steps=8),
    dict(name="channel24x40_inlets", nx=24, ny=40, bc=[[0, 1.0], [2, 0.0], [0, 1.0], [2, 0.5]], xratio=-1,
         yratio=-1, dt=1 / 320, re=100.0, steps=6),
]


def main():
    idx = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/ns_oracle.c", "cases": []}
    for c in CASES:
        g = OGrid.rectangle(c["nx"], c["ny"], bc=c["bc"], xratio=c["xratio"], yratio=c["yratio"])
        s = OSolver(g, c["dt"], c["re"], rtol=1e-13)
        mms = [s.step()[0] for _ in range(c["steps"])]
        st = s.get()
        f = c["name"] + ".npz"
        np.savez_compressed(os.path.join(HERE, f), mm=np.array(mms), u=st["u"], v=st["v"], phi=st["phi"])
        idx["cases"].append(dict(c, file=f))
    json.dump(idx, open(os.path.join(HERE, "index.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
