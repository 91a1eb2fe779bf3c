"""bench.py's rank plumbing on the CPU (no GPU call is made): --gpus N
starts N rank processes itself when no launcher is present, agrees with a
launcher's WORLD_SIZE, and refuses a disagreement (the driver's
scaling run uses `bench.py --gpus N`)."""
import json
import os
import subprocess
import sys

import pytest

from _paths import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _env():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    return e


def test_rank_check():
    assert bench.rank_check(1, {}) == 1
    assert bench.rank_check(4, {}) is None            # bench starts the ranks
    assert bench.rank_check(4, {"WORLD_SIZE": "4"}) == 4
    assert bench.rank_check(1, {"WORLD_SIZE": "1"}) == 1
    with pytest.raises(SystemExit):
        bench.rank_check(2, {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        bench.rank_check(8, {"WORLD_SIZE": "1"})


def test_launch_plan():
    plan = bench.launch_plan(4, {"FOO": "1"}, 12345)
    assert [p["RANK"] for p in plan] == ["0", "1", "2", "3"]
    assert [p["LOCAL_RANK"] for p in plan] == ["0", "1", "2", "3"]
    for p in plan:
        assert p["WORLD_SIZE"] == "4"
        assert p["MASTER_ADDR"] == "127.0.0.1"
        assert p["MASTER_PORT"] == "12345"
        assert p["FOO"] == "1"


def test_mismatch_exits_nonzero():
    env = _env()
    env["WORLD_SIZE"] = "4"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"),
                        "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0
    assert "must agree" in r.stderr
    assert r.stdout == ""


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_ranks(n):
    """No launcher: bench.py --gpus N runs N ranks that meet over gloo; rank
    0 alone prints one JSON line, with n_gpus = N."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"),
                        "--gpus", str(n), "--probe-launch"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["gpus_arg"] == n
    assert d["ranks"] == list(range(n))


def test_config4_refuses_ranks():
    env = _env()
    env["WORLD_SIZE"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"),
                        "--config4", "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "one process" in r.stderr
