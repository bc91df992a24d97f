"""Idle gaps between consecutive kernels in a rocprofv3 kernel trace, grouped by the kernel
pair (the dependent-kernel boundary cost; tools/profile_round.sh makes the trace).
  python tools/gaps.py <kernel_trace.csv> [max_gap_us]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
cap = float(sys.argv[2]) if len(sys.argv) > 2 else 500.0
gaps = collections.defaultdict(list)
for a, b in zip(rows, rows[1:]):
    g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000
    if 0 < g < cap:
        gaps[(a["Kernel_Name"].split("(")[0][-26:], b["Kernel_Name"].split("(")[0][-26:])].append(g)
print(f"total gap {sum(sum(v) for v in gaps.values()):.0f} us over {len(rows)} kernels")
for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:12]:
    print(f"{k[0]:28s} -> {k[1]:28s} n={len(v):4d} sum={sum(v):8.0f} med={sorted(v)[len(v) // 2]:6.1f}")
