"""bench.py's multi-rank launch: ``python bench.py --gpus N``
without a torch.distributed environment starts N ranks itself (a
torch.distributed.run child process) and the line reports the N ranks the
all-reduce saw.  CPU only: --dry-run with the gloo backend."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_spawns_two_ranks():
    out = _run("--gpus", "2", "--backend", "gloo", "--dry-run", "--steps", "5", "--warmup", "1")
    assert out["n_gpus"] == 2 and out["ranks_seen"] == 2 and out["steps"] == 5


def test_bench_single_rank_dry_run():
    out = _run("--dry-run", "--steps", "3", "--warmup", "1")
    assert out["n_gpus"] == 1 and out["ranks_seen"] == 1
