"""bench.py's multi-rank launcher on CPU: `--gpus 2` without WORLD_SIZE starts torch.distributed.run
with two ranks as a child process; the ranks shard the pairs and all-gather their result rows (gloo
here, RCCL on the GPU node) — rank 0 checks the gathered rows are in global pair order.

`--dry-run` skips the registration (no GPU in this container): each rank writes its rows' global
pair index, so the order check covers exactly the launcher + shard + gather code bench.py runs."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 prints ONE JSON line
    return json.loads(lines[0])


def test_launcher_two_ranks_gather_order():
    line = _run("--gpus", "2", "--dry-run", "--pairs", "5")
    assert line["n_gpus"] == 2
    assert line["gathered_pairs"] == 10
    assert line["gather_order_ok"] is True


def test_launcher_single_rank_no_spawn():
    line = _run("--gpus", "1", "--dry-run", "--pairs", "4")
    assert line["n_gpus"] == 1 and line["gather_order_ok"] is True
