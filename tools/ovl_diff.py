"""Where do the overlapped and plain-exchange slab runs differ?  (debug aid for the
test_overlapped_exchange_is_bit_identical test: prints the per-step monitor and the rows / columns
of the first differing field)  NSGPU_LIB selects the library.  python tools/ovl_diff.py [nproc]"""
import os, sys, pathlib, tempfile
import numpy as np
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from test_gpu_multirank import launch
nproc = int(sys.argv[1]) if len(sys.argv) > 1 else 2
args = ["--xport", "host", "--size", "192", "--size-y", "160", "--nsteps", os.environ.get("NSTEPS", "4"), "--tol", "1e-11"]
os.environ["NSGPU_PAIR_MIN_CELLS"] = "0"
os.environ["NSGPU_STRIP_ROWS"] = "16"
tmp = pathlib.Path(tempfile.mkdtemp())
res = {}
for ov in ("1", "0"):
    os.environ["NSGPU_OVERLAP"] = ov
    (tmp / ov).mkdir()
    res[ov] = launch(tmp / ov, *args, nproc=nproc, port=29641 + int(ov))
a, b = res["1"], res["0"]
print("mm overlap\n", a["mm"], "\nmm plain\n", b["mm"])
for k in ("u", "v", "phi"):
    d = np.abs(a[k] - b[k])
    print(k, "max diff", d.max(), "shape", d.shape)
    if d.max() > 0:
        rows = np.where(d.max(axis=1) > 0)[0]
        cols = np.where(d.max(axis=0) > 0)[0]
        print(" rows", rows[:40], "...", len(rows), " cols", cols[:20], "...", len(cols))
