"""Kernels between the marker launches of tools/rccl_loopback_probe.cpp (rocprofv3 kernel trace):
per phase, each kernel name's count and mean duration.  python tools/probe_phases.py <kernel_trace.csv>"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
phase, agg = 0, collections.defaultdict(lambda: [0, 0.0])
names = {0: "RCCL init (before the first marker)", 1: "allreduce x10", 2: "send+recv self x10", 3: "7 send/recv pairs x10", 4: "end"}
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if n.startswith("marker"):
        phase += 1
        continue
    a = agg[(phase, n[:60])]
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for (p, n), (c, t) in sorted(agg.items()):
    label = names.get(0 if p == 0 else (p - 1) % 4 + 1, "?")
    print(f"phase {p} ({label}): {n:60s} x{c:3d} avg {t / c:8.1f} us")
