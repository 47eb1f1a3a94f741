"""The featurizer's kernels (featurizer.hip: plan, logmel, norm through the real
rnnt_featurizer_create / run) executed on the CPU by the host emulation of the wave model
(tools/emu/fz_emu.cpp), with every logmel workgroup's LDS poisoned at start: four poisons (NaN,
1e38, zero, random bits) give bit-identical features, every output element is written, and the
features match the float64 restatement.  Lanes of a wave meet only at explicit barriers in the
emulation, so this also rules out intra-wave hand-offs that lean on lockstep.  It is the software
side of the round-3 featurizer corruption beside decode kernels: no read of LDS the
workgroup did not write, no missing wave sync, no out-of-bounds access."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    if not os.path.exists(CLANG):
        pytest.skip("no ROCm clang++")
    out = tmp_path_factory.mktemp("emu_fz")
    env = dict(os.environ, EMU_ASAN="1", EMU_OUT=str(out))
    subprocess.run(["bash", os.path.join(REPO, "tools", "emu", "build_fz.sh")], check=True, env=env,
                   capture_output=True, timeout=600)
    return str(out / "fz_emu")


def test_featurizer_kernels_on_emulator_with_poisoned_lds(emu):
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "emu", "fz_emu_check.py"), "--n", "7", "--exe", emu],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout[-3000:] + r.stderr[-3000:]
