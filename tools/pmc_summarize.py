"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the bench into
profiles/pmc_traffic.json (read by bench.py for each kernel's roofline.traffic).
  python tools/pmc_summarize.py <n> <fetch_dir> <write_dir> <out.json> key=regex=bytes_per_cell ...
For each key: the dispatches whose kernel name matches `regex`, restricted to the largest grid
among them (the finest multigrid level), median over dispatches.
gfx950 corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts half the bytes of a wide
coalesced stream -> x2; WRITE_SIZE is exact for 16-B/lane stores; both in KiB."""
import csv, glob, json, re, sys

if sys.argv[1] == "--valu":
    # python tools/pmc_summarize.py --valu <n> <valu_dir> <out.json> key=regex ...: SQ_INSTS_VALU
    # (wave-instructions, summed over the dispatch) per finest-level cell, median over dispatches
    import statistics
    n, d, out = int(sys.argv[2]), sys.argv[3], sys.argv[4]
    res = {"n": n, "kernels": {}, "note": "SQ_INSTS_VALU wave-instructions per dispatch / n^2 cells (finest-level dispatches, median)"}
    for spec in sys.argv[5:]:
        key, rx = spec.split("=", 1)
        pat = re.compile(rx)
        vals = {}
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if pat.search(r.get("Kernel_Name", "")) and r.get("Counter_Name") in ("SQ_INSTS_VALU", "SQ_WAVES"):
                    g = int(r.get("Grid_Size", r.get("Grid_Size_X", "0")) or 0)
                    vals.setdefault((r.get("Dispatch_Id"), g), {})[r["Counter_Name"]] = float(r["Counter_Value"])
        if not vals:
            continue
        gmax = max(g for _, g in vals)
        v = [x["SQ_INSTS_VALU"] for (_, g), x in vals.items() if g == gmax and "SQ_INSTS_VALU" in x]
        w = [x["SQ_WAVES"] for (_, g), x in vals.items() if g == gmax and "SQ_WAVES" in x]
        med = statistics.median(v)
        res["kernels"][key] = {"regex": rx, "dispatches": len(v), "valu_wave_insts": med, "waves": statistics.median(w) if w else None,
                               "valu_per_cell": med / (n * n), "lane_ops_per_cell": 64 * med / (n * n)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))
    sys.exit(0)

n = int(sys.argv[1]); fetch_dir, write_dir, out = sys.argv[2], sys.argv[3], sys.argv[4]


def per_dispatch(d, counter, pat):
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat.search(r.get("Kernel_Name", "")) and r.get("Counter_Name") == counter:
                g = int(r.get("Grid_Size", r.get("Grid_Size_X", "0")) or 0)
                rows.append((g, float(r["Counter_Value"])))
    if not rows:
        return []
    gmax = max(g for g, _ in rows)
    return [v for g, v in rows if g == gmax]


def _sha16(path):
    import hashlib
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
res = {"n": n, "kernels": {},
       "note": "median over the finest-level dispatches; FETCH_SIZE x2 (gfx950 wide-stream correction), KiB -> bytes",
       # the stamp bench.py copies into each roofline.traffic: which run and which library measured it
       "source": {"fetch_dir": fetch_dir, "write_dir": write_dir,
                  "command": os.environ.get("PMC_COMMAND", "rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) -- "
                                            "python3 bench.py --steps 3 --warmup 1 --no-cpu"),
                  "libnsgpu_sha16": _sha16(os.path.join(ROOT, "navierstokessolver_amd", "libnsgpu.so"))}}
for spec in sys.argv[5:]:
    key, rx, bpc = spec.split("=")
    pat = re.compile(rx)
    fv, wv = per_dispatch(fetch_dir, "FETCH_SIZE", pat), per_dispatch(write_dir, "WRITE_SIZE", pat)
    fetch = sorted(fv)[len(fv) // 2] * 1024 * 2 if fv else None
    write = sorted(wv)[len(wv) // 2] * 1024 if wv else None
    res["kernels"][key] = {"regex": rx, "dispatches": [len(fv), len(wv)], "fetch_bytes_corrected": fetch,
                           "write_bytes": write, "kernel_bytes_per_launch": (fetch + write) if fetch and write else None,
                           "algorithmic_bytes_per_launch": float(bpc) * n * n}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
