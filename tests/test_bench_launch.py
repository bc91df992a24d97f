"""bench.py --gpus N starts its own N ranks when no launcher set WORLD_SIZE (the
driver's `python3 bench.py --gpus N` form must reach every rank).  CPU only: the probe hook
(NSBENCH_LAUNCH_PROBE) makes each rank report its rank / world and exit before any GPU call."""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_self_launches_n_ranks():
    env = dict(os.environ, NSBENCH_LAUNCH_PROBE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    # (the ranks share the child's stdout: their lines may interleave)
    probes = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", r.stdout)]
    assert sorted(p["probe_rank"] for p in probes) == [0, 1, 2]
    assert all(p["world"] == 3 for p in probes)
    assert sorted(p["local_rank"] for p in probes) == [0, 1, 2]
