"""Per-kernel summary of a rocprofv3 rocpd database (`--kernel-trace` without `--output-format csv`):
kernel, calls, total / average microseconds, VGPRs and scratch, for the dispatches after the last launch of
`--after` (e.g. the last set-up kernel) or all of them.  Usage: rocpd_summary.py results.db [--after NAME]
[--steps N] (per-step columns: totals / N)."""
import argparse
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--after", default=None)
ap.add_argument("--steps", type=int, default=1)
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = list(c.execute("select name, start, end, vgpr_count, scratch_size from kernels order by start"))
if a.after:
    rows = rows[max(i for i, r in enumerate(rows) if a.after in r[0]) + 1:]
d = defaultdict(lambda: [0, 0.0, 0, 0])
for n, s, e, v, sc in rows:
    k = n.split("(")[0].replace("(anonymous namespace)::", "")
    d[k][0] += 1
    d[k][1] += (e - s) / 1e3
    d[k][2], d[k][3] = v, sc
tot = sum(x[1] for x in d.values())
print(f"dispatches {len(rows)}, span {(rows[-1][2] - rows[0][1]) / 1e3:.1f} us, busy {tot:.1f} us; per step "
      f"(/{a.steps}): span {(rows[-1][2] - rows[0][1]) / 1e3 / a.steps:.1f} us, busy {tot / a.steps:.1f} us")
print(f"{'kernel':64s} {'calls':>6s} {'total_us':>10s} {'avg_us':>8s} {'per_step_us':>11s} {'vgpr':>5s} {'scratch':>7s}")
for k, x in sorted(d.items(), key=lambda t: -t[1][1]):
    print(f"{k[:64]:64s} {x[0]:6d} {x[1]:10.1f} {x[1] / x[0]:8.2f} {x[1] / a.steps:11.1f} {x[2]:5d} {x[3]:7d}")
