"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes for one kernel into
profiles/pmc_traffic.json (read by bench.py for roofline.traffic).
  python tools/pmc_summarize.py <n> <fetch_dir> <write_dir> <out.json> <kernel regex> <alg bytes/cell> [label]
gfx950 corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts half the bytes of a wide
coalesced stream -> x2; WRITE_SIZE is exact for 16-B/lane stores; both in KiB."""
import csv, glob, json, re, sys
n = int(sys.argv[1]); fetch_dir, write_dir, out = sys.argv[2], sys.argv[3], sys.argv[4]
pat = re.compile(sys.argv[5]); bpc = float(sys.argv[6])
label = sys.argv[7] if len(sys.argv) > 7 else sys.argv[5]


def per_dispatch(d, counter):
    vals = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat.search(r.get("Kernel_Name", "")) and r.get("Counter_Name") == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


fv, wv = per_dispatch(fetch_dir, "FETCH_SIZE"), per_dispatch(write_dir, "WRITE_SIZE")
fetch = sorted(fv)[len(fv) // 2] * 1024 * 2 if fv else None
write = sorted(wv)[len(wv) // 2] * 1024 if wv else None
res = {"n": n, "kernel": label, "dispatches": [len(fv), len(wv)],
       "fetch_bytes_corrected": fetch, "write_bytes": write,
       "kernel_bytes_per_launch": (fetch + write) if fetch and write else None,
       "algorithmic_bytes_per_launch": bpc * n * n,
       "note": "median over dispatches; FETCH_SIZE x2 (gfx950 wide-stream correction), KiB -> bytes"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
