"""Per-kernel VGPRs / scratch / occupancy of ns_kernels.hip (hipcc -Rpass-analysis), one line per kernel.
python tools/resources.py [filter]"""
import re
import subprocess
import sys

src = "navierstokessolver_amd/csrc"
out = subprocess.run(["make", "-s", "-C", src, "resources"], capture_output=True, text=True).stdout
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
        continue
    for key in ("VGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0]] = int(m.group(1))
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if flt in r["name"]:
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('ScratchSize', '?'):>3} scr {r.get('Occupancy', '?'):>2} w/simd "
              f"{r.get('LDS', '?'):>6} lds  {r['name']}")
