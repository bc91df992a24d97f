"""One virtual slab's step (tools/slab_projection.py's method) for a rocprofv3 kernel trace:
python tools/vslab_trace.py N P [helm_sweeps] -- rank P/2 of an N^2 cavity on P x-slabs, the loopback
communicator, every step replaying (helm_sweeps, 1 Poisson solve)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from slab_projection import run

n, P = int(sys.argv[1]), int(sys.argv[2])
h = int(sys.argv[3]) if len(sys.argv) > 3 else 3
seq, r = run(n, P, 5, 20, 1000.0, replay=[(h, 1)] * 25)
print(r)
