"""bench.py --gpus N forms a world of N ranks by itself (torch.distributed.run as a child, no HIP in
the parent), on the CPU mock path: gloo ranks shard one query, gather every response to rank 0 and
rank 0 prints n_gpus from the real world size.  A torchrun world that disagrees with --gpus is an
error, not a silently smaller measurement."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_gpus_2_launches_two_ranks():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--mock", "--steps", "1", "--warmup", "0",
                          "--query", "1500"], capture_output=True, text=True, timeout=300, env=_env())
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # one JSON line, from rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["config"]["query_samples"] == 3000 and rec["config"]["gathered"] == 3000


def test_world_disagreeing_with_gpus_fails():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--mock", "--steps", "1", "--warmup", "0"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode != 0 and "--gpus 2" in out.stderr
