"""bench.py's multi-rank plumbing on the CPU: ``--gpus N`` without a launcher spawns N ranks itself
(torch.distributed.run on 127.0.0.1), the ranks rendezvous, time with a barrier and a
max-over-ranks reduction, and rank 0 prints ONE JSON line whose n_gpus is the world size the
process group actually saw (--gpus used to be parsed and ignored).  The GPU work is
replaced by a trivial loop (--selftest-launch); the real run is the same code path up to there."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env=None):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=180, cwd=ROOT, env=env)


def test_bench_self_launches_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = _run("--gpus", "2", "--selftest-launch", "--steps", "5", env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout        # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 5


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = _run("--gpus", "2", "--selftest-launch", env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
