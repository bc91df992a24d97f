"""One summary line of a bench.py JSON log: label MLUPS ms/step V-cycles (or direct solves) Helmholtz-sweeps
checks/step and each timed kernel's average (A/B scripts).  python tools/bench_line.py <label> <log>"""
import json
import sys

d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = " ".join(f"{n}={v['avg_kernel_us']:.1f}us" for n, v in d["kernels"].items())
pois = d.get("poisson_vcycles_per_step", d.get("poisson_direct_solves_per_step"))
print(sys.argv[1], round(d["value"]), round(d["ms_per_step"], 3), pois,
      d["helmholtz_sweeps_per_step"], d.get("poisson_checks_per_step"), ks, flush=True)
