#!/bin/bash
# bench.py at several multigrid smoother over-relaxations (ms/step, V-cycles/step)
for w in 1.0 1.1 1.15 1.2 1.25 1.3; do
  echo -n "omega=$w "
  NSGPU_MG_OMEGA=$w timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step", d["poisson_vcycles_per_step"], "V-cycles/step", round(d["value"]), "MLUPS")' || exit 1
done
