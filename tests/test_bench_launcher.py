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
    assert rec["control_plane"] == "gloo"  # the ranks' default group is gloo, not RCCL


def test_control_plane_defaults_to_gloo():
    """The GPU path's control plane (barriers, max-over-ranks timing, claims) is gloo unless
    --control-backend nccl asks for RCCL (the backend the hardware rehearsal ran);
    --share-device and --mock are always gloo."""
    import argparse
    sys.path.insert(0, REPO)
    import bench
    ns = argparse.Namespace(share_device=False, mock=False, control_backend="gloo")
    assert bench.control_backend(ns) == "gloo"
    ns.control_backend = "nccl"
    assert bench.control_backend(ns) == "nccl"
    ns.share_device = True
    assert bench.control_backend(ns) == "gloo"
    old = sys.argv
    try:
        sys.argv = ["bench.py", "--gpus", "2"]
        assert bench.control_backend(bench.parse()) == "gloo"
    finally:
        sys.argv = old


def test_world_disagreeing_with_gpus_fails():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--mock", "--steps", "1", "--warmup", "0"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode != 0 and "--gpus 2" in out.stderr


def test_dumped_responses_equal_across_rank_counts(tmp_path):
    """--dump-responses + tools/compare_responses.py (the GPU rehearsal's check,
    tools/gpu.sh multirank) on the mock path: the query served by 2 ranks with dynamic claims and by
    3 ranks with the static deal gathers the same rows as 1 rank; a changed row is reported."""
    import numpy as np

    def run(ranks, query, name, *extra):
        p = str(tmp_path / f"{name}.npz")
        out = subprocess.run([sys.executable, BENCH, "--gpus", str(ranks), "--mock", "--steps", "1", "--warmup", "0",
                              "--query", str(query), "--batch", "256", "--dump-responses", p, *extra],
                             capture_output=True, text=True, timeout=300, env=_env())
        assert out.returncode == 0, out.stderr[-2000:]
        return p

    one = run(1, 1536, "one")
    cmp = os.path.join(REPO, "tools", "compare_responses.py")
    for p in (run(2, 768, "dyn2"), run(3, 512, "static3", "--deal", "static")):
        out = subprocess.run([sys.executable, cmp, p, one], capture_output=True, text=True, timeout=60)
        assert out.returncode == 0, out.stdout + out.stderr
        assert json.loads(out.stdout)["identical"]
    z = dict(np.load(one))
    z["toks"] = z["toks"].copy()
    z["toks"][0] ^= 1
    bad = str(tmp_path / "bad.npz")
    np.savez(bad, **z)
    out = subprocess.run([sys.executable, cmp, bad, one], capture_output=True, text=True, timeout=60)
    assert out.returncode == 1 and json.loads(out.stdout)["mismatched_rows"] == 1


def test_eight_ranks_gather_keeps_up_at_full_volume():
    """bench.py's 8-rank data path at the default query (300000 samples per rank,
    6144-row batches, dynamic claims) with stand-in responses of the timed workload's volume (~64
    tokens per sample): rank 0's ResponseStream receives all 2.4M rows, and the whole step -- sort,
    claims, the stand-ins and the streamed gather -- runs faster than 8 GPUs produce rows
    (8 x 121k samples/s, BENCH_r05), so the gather cannot bound an 8-GPU step."""
    out = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--mock", "--steps", "2", "--warmup", "1"],
                         capture_output=True, text=True, timeout=600, env=_env())
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["config"]["query_samples"] == 8 * 300000 and rec["config"]["gathered"] == 8 * 300000
    assert 50 * 8 * 300000 < rec["tokens_per_query"] < 80 * 8 * 300000
    assert rec["rows_per_s_gathered"] > 8 * 121000, rec
