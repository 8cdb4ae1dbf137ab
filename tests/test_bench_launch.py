"""bench.py's multi-GPU entry point on CPU: ``--gpus N`` starts N rank processes itself when
no launcher set WORLD_SIZE, and every rank checks the world it joined (``--dry-run`` replaces
the GPU body with a gloo barrier and a rank count)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _bench(*args, env=None, timeout=120):
    e = {k: v for k, v in os.environ.items()
         if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=e,
                          capture_output=True, text=True, timeout=timeout)


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 3])
def test_gpus_flag_starts_n_ranks(n):
    r = _bench("--gpus", str(n), "--dry-run")
    assert r.returncode == 0, r.stderr
    d = _line(r.stdout)
    assert d["n_gpus"] == n and d["ranks_seen"] == n and d["gpus_flag"] == n


def test_rank_refuses_a_world_that_disagrees_with_gpus():
    r = _bench("--gpus", "2", "--dry-run",
               env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "--gpus 2 but the launcher started 1 ranks" in r.stderr


def test_under_torch_distributed_run():
    """The driver's form: torch.distributed.run starts the ranks, bench.py joins them."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", "29517", os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2
