"""CPU check of the compiled TorchModel replacement's harness (csrc/sut/): it is built, loads with ONE
HIP runtime (torch's: its self-check exits 3 otherwise) even with LD_LIBRARY_PATH pointing at the
system ROCm, and rejects a bad command line without touching the GPU.  The GPU run is
tests/test_sut_harness_gpu.py."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(REPO, "rnnt-inference_amd", "rnnt_amd", "rnnt_sut_harness")


def test_harness_loads_one_hip_runtime():
    if not os.path.exists(HARNESS):
        pytest.skip("harness not built (no ROCm libtorch here)")
    for ld in (None, "/opt/rocm/lib"):
        env = dict(os.environ)
        env.pop("LD_LIBRARY_PATH", None)
        if ld:
            env["LD_LIBRARY_PATH"] = ld
        r = subprocess.run([HARNESS], capture_output=True, text=True, timeout=60, env=env)
        assert r.returncode == 2 and "usage" in r.stderr, (ld, r.returncode, r.stderr[-500:])
