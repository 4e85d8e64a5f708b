"""bench.py --gpus N launches its own N ranks (one process per GPU, extract.py:101-117 pattern) when no external
launcher set WORLD_SIZE: rehearsed on the CPU with gloo through --selftest-launch (the same self-launch, rendezvous,
barrier-bracketed timing, SUM/MAX reduction and rank-0 JSON line; a host loop stands in for the device step)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("extra", [[], ["--config", "c4"]])
def test_bench_self_launches_two_ranks(extra):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["RVCX_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--selftest-launch", "--steps",
                        "3"] + extra, env=env, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["backend"] == "gloo"
    ranks = sorted(tuple(x) for x in rec["ranks"])
    assert [x[0] for x in ranks] == [0, 1] and [x[2] for x in ranks] == [0, 1]  # RANK and LOCAL_RANK per worker
    assert ranks[0][1] != ranks[1][1]  # two processes


def test_bench_worker_failure_propagates():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["RVCX_DIST_BACKEND"] = "no-such-backend"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--selftest-launch"], env=env,
                       capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode != 0
