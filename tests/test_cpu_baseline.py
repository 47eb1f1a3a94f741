"""bench.py's cpu_baseline leg runs the C restatement on the CPUs this process may actually use:
the affinity set capped by the cgroup CPU quota, one OpenMP thread pinned per CPU (VERDICT r04
item 6; the reference pins each instance's team to its cores, csrc/torch_sut.cpp:100-121,
kmp_launcher.cpp:14-29).  CPU only."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))

import bench  # noqa: E402
from oracle import oracle  # noqa: E402


def test_budget_is_capped_by_the_cgroup_quota(monkeypatch):
    aff = sorted(os.sched_getaffinity(0))
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: None)
    cpus, meta = bench.host_cpu_budget()
    assert len(cpus) == len(aff) == meta["threads"] and sorted(cpus) == aff
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: 2.5)
    cpus, meta = bench.host_cpu_budget()
    assert len(cpus) == min(2, len(aff)) and meta["cgroup_cpu_quota"] == 2.5
    assert set(cpus) <= set(aff)


def test_cgroup_quota_parses_v1_and_v2(tmp_path, monkeypatch):
    v2 = tmp_path / "v2"
    v2.mkdir()
    (v2 / "cpu.max").write_text("1600000 100000\n")
    v1 = tmp_path / "v1"
    v1.mkdir()
    (v1 / "cpu.cfs_quota_us").write_text("800000\n")
    (v1 / "cpu.cfs_period_us").write_text("100000\n")
    real = bench._read

    def fake(path, root):
        for name in ("cpu.max", "cpu.cfs_quota_us", "cpu.cfs_period_us"):
            if path.endswith(name):
                p = os.path.join(root, name)
                return open(p).read().strip() if os.path.exists(p) else None
        return real(path) if path == "/proc/self/cgroup" else None

    monkeypatch.setattr(bench, "_read", lambda p: fake(p, str(v2)))
    assert bench.cgroup_cpu_quota() == 16.0
    monkeypatch.setattr(bench, "_read", lambda p: fake(p, str(v1)))
    assert bench.cgroup_cpu_quota() == 8.0
    (v1 / "cpu.cfs_quota_us").write_text("-1\n")
    assert bench.cgroup_cpu_quota() is None


def test_pinned_team_gives_the_same_answer():
    """The pinned team computes what the unpinned one does (the restatement's OpenMP loops are over
    independent rows) and the caller's own CPU mask is restored afterwards."""
    lib = oracle.lib()
    before = os.sched_getaffinity(0)
    cpus = sorted(before)[:2]
    lib.oracle_pin_threads.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    x = np.random.default_rng(0).standard_normal((4, 1000)).astype(np.float32)
    ref = oracle.quantize(x, 20.0)
    n = lib.oracle_pin_threads(len(cpus), (ctypes.c_int * len(cpus))(*cpus))
    assert n == len(cpus)
    assert lib.oracle_bind_master(cpus[0]) == 0
    assert os.sched_getaffinity(0) == {cpus[0]}
    got = oracle.quantize(x, 20.0)
    assert lib.oracle_bind_master(-1) == 0
    assert os.sched_getaffinity(0) == before
    assert np.array_equal(got, ref)
    allc = sorted(before)  # leave the process's team at full width for the other tests
    assert lib.oracle_pin_threads(len(allc), (ctypes.c_int * len(allc))(*allc)) == len(allc)
