"""`bench.py --gpus N` launches N ranks itself when no launcher set WORLD_SIZE (the driver may run
it either way); a --gpus that disagrees with WORLD_SIZE is refused.  CPU/gloo dry run."""
import json
import os
import subprocess
import sys

from conftest import REPO


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          timeout=240, cwd=REPO, env=env)


def test_gpus_n_spawns_n_ranks():
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    assert lines[0]["n_gpus"] == 2 and lines[0]["world_size"] == 2 and lines[0]["rank_sum"] == 1


def test_mismatched_world_is_refused():
    r = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
