"""`bench.py --gpus N` launches N ranks itself when no launcher set WORLD_SIZE (the driver may run
it either way); a --gpus that disagrees with WORLD_SIZE is refused.  CPU/gloo dry run, which also
rehearses the viewsplit step's rank layout, Philox offsets, megabatch all-gather and tooHigh
all_reduce (bench.py:dry_run_viewsplit): the final megabatch must be bit-identical at N = 1, 2, 4."""
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


def test_viewsplit_dry_run_is_bit_identical_across_world_sizes():
    """N ranks own 4 views each of one 4N-view megabatch; the same 4N views run as one process must
    end in the same bits (--views 4 per rank vs --views 4N on one rank)."""
    digests = {}
    for n in (1, 2, 4):
        args = ["--gpus", str(n), "--dry-run", "--steps", "6", "--views", "4"]
        r = _run(args)
        assert r.returncode == 0, r.stderr[-2000:]
        line = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")][0]
        assert line["world_size"] == n and line["rank_sum"] == n * (n - 1) // 2
        digests[n] = line["viewsplit_sha256"]
        one = _run(["--dry-run", "--steps", "6", "--views", str(4 * n)])
        assert one.returncode == 0, one.stderr[-2000:]
        ref = [json.loads(l) for l in one.stdout.splitlines() if l.startswith("{")][0]["viewsplit_sha256"]
        assert digests[n] == ref, n


def test_mismatched_world_is_refused():
    r = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
