"""bench.py --gpus N starts its own N ranks when no launcher set WORLD_SIZE (the
driver's `python3 bench.py --gpus N` form must reach every rank).  CPU: the probe hook
(NSBENCH_LAUNCH_PROBE) makes each rank report its rank / world and exit before any GPU call.
GPU: the whole N = 2 branch on one GPU through the host transport."""
import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_self_launches_n_ranks():
    env = dict(os.environ, NSBENCH_LAUNCH_PROBE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    # (--n and --re are abbreviations of torch.distributed.run options: they must reach the ranks)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--steps", "1", "--n", "512",
                        "--re", "100"], capture_output=True, text=True, env=env, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    # (the ranks share the child's stdout: their lines may interleave)
    probes = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", r.stdout)]
    assert sorted(p["probe_rank"] for p in probes) == [0, 1, 2]
    assert all(p["world"] == 3 for p in probes)
    assert sorted(p["local_rank"] for p in probes) == [0, 1, 2]
    assert all(p["n"] == 512 and p["re"] == 100.0 for p in probes)


def test_bench_failed_rank_reports_and_exits_nonzero():
    """a rank that fails (an RCCL init or collective error raises NsError) prints a JSON
    error line and exits non-zero, and the job ends instead of leaving its peers hanging in a collective.
    CPU: NSBENCH_FAIL_RANK injects the failure on rank 1 before any GPU call; rank 0 is left waiting in
    the process-group set-up until torch.distributed.run tears it down."""
    env = dict(os.environ, NSBENCH_FAIL_RANK="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "NSBENCH_LAUNCH_PROBE"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--n", "64"],
                       capture_output=True, text=True, env=env, timeout=240, cwd=ROOT)
    assert r.returncode != 0
    errs = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", r.stdout)]
    assert any(e.get("error") and e.get("rank") == 1 and e.get("value") is None for e in errs), r.stdout[-2000:]


def _bench(args, timeout=300):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "NSBENCH_LAUNCH_PROBE"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       env=env, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return r


@pytest.mark.gpu
def test_bench_two_ranks_host_transport():
    """bench.py's N > 1 branch end to end on one GPU (--transport host: both
    ranks on device 0, ghost rows / gathers / reductions through gloo) -- the self-launch, the slab
    step, the per-rank timing max and the rank-0 JSON line.  stdout holds exactly ONE line (the
    relay sends everything that is not a JSON line to stderr), it says n_gpus 2 and the host
    transport, and its last monitor equals one rank's run of the same workload (the slab step
    matches one rank: tests/test_gpu_multirank.py; tolerance 1e-9)."""
    common = ["--n", "512", "--steps", "4", "--warmup", "3", "--no-cpu", "--time-every", "1"]
    r2 = _bench(["--gpus", "2", "--transport", "host", *common])
    lines = [ln for ln in r2.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r2.stdout[-2000:]
    d2 = json.loads(lines[0])
    assert d2["n_gpus"] == 2 and d2["config"]["transport"].startswith("host")
    assert d2["config"]["local_rows_rank0"] == 256
    assert d2["value"] > 0 and d2["roofline"] is not None
    #  the multi-rank line says where its time went: every rank's ms / step and slab,
    # the per-step collectives (r5: 2 on an unchecked direct solve -- the Helmholtz check's scalar bus and
    # the recurrences' one allgather) and exchange groups, the link bytes; the RCCL version on the RCCL transport
    ranks = d2["ranks"]
    assert [x["rank"] for x in ranks] == [0, 1] and [x["rows"] for x in ranks] == [256, 256]
    assert all(x["ms_per_step"] > 0 for x in ranks)
    assert abs(max(x["ms_per_step"] for x in ranks) - d2["ms_per_step"]) <= 1e-6 * d2["ms_per_step"]
    c = d2["comm"]
    assert 2 <= c["collectives_per_step"] <= 5 and c["exchanges_per_step"] >= 1 and c["x_link_bytes_per_step"] > 0
    assert "rccl_version" in c
    d1 = json.loads([ln for ln in _bench(common).stdout.splitlines() if ln.strip()][-1])
    assert d1["n_gpus"] == 1 and "ranks" not in d1 and "comm" not in d1
    for k in ("umin", "umax", "vmin", "vmax"):
        assert abs(d2["monitor_last_step"][k] - d1["monitor_last_step"][k]) <= 1e-9, (k, d2["monitor_last_step"],
                                                                                         d1["monitor_last_step"])
