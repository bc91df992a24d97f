"""Per-kernel, per-grid-size time from a rocprofv3 kernel trace (csv).
python tools/trace_summary.py <kernel_trace.csv> [steps] [first-kernel]
first-kernel: count only from the first launch whose name contains it (e.g. k_rhs: the first time
step; k_rhs@5: the sixth, after 5 warm-up steps), so one-time set-up work -- RCCL's communicator init (~260 copies and ~520 fills,
tools/rccl_loopback_probe.cpp), solver creation -- is not divided over the steps."""
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
if len(sys.argv) > 3:
    # name@K: from the K-th (0-based) launch whose name contains `name` (skip K warm-up steps)
    key, _, nth = sys.argv[3].partition("@")
    hits = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
    k0 = hits[min(int(nth or 0), len(hits) - 1)] if hits else 0
    rows = rows[k0:]
agg = collections.defaultdict(lambda: [0, 0.0])
def g(r, k):
    for key in (k, k.replace("_", "")):
        if key in r: return r[key]
    return "?"
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:40]
    grid = g(r, "Grid_Size_X") if "Grid_Size_X" in r else g(r, "Grid_Size")
    gy = r.get("Grid_Size_Y", "")
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = agg[(name, f"{grid}x{gy}")]
    a[0] += 1; a[1] += dur
tot = sum(v[1] for v in agg.values())
print(f"total GPU time per step: {tot/steps/1e3:.3f} ms")
for (n, gsz), (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
    print(f"{n:40s} grid={gsz:>14s} calls/step={c/steps:7.1f} avg={t/c:8.1f}us per-step={t/steps/1e3:7.3f}ms {100*t/tot:5.1f}%")
