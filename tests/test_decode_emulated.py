"""The engine's greedy-decode kernels (decoder.hip: label table, prediction, G, joint, the host
step loop) executed on the CPU by the host emulation of the wave model (tools/emu: one fiber per
lane, workgroup / wave barriers, MFMA through the oracle's pinned accumulation model, bounds
checks on every list-entry access), compared token for token with the oracle's greedy decode --
Offline (one call) and Server continuous batching (two calls over the halves of the frames,
state carried).  No GPU: this checks the kernels' indexing and control logic; compiler effects
are covered by tests/test_isa_lint.py and the -m gpu parity tests."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    if not os.path.exists(CLANG) or not shutil.which("python3"):
        pytest.skip("no ROCm clang++")
    out = tmp_path_factory.mktemp("emu")
    env = dict(os.environ, EMU_ASAN="0", EMU_OUT=str(out), EMU_CFLAGS="-DRNNT_DEV_KNOBS")  # RNNT_DEC_SLIM below
    subprocess.run(["bash", os.path.join(REPO, "tools", "emu", "build.sh")], check=True, env=env,
                   capture_output=True, timeout=600)
    return str(out / "dec_emu")


@pytest.mark.parametrize("server", [0, 1])
@pytest.mark.parametrize("slim", ["15", "0"])
def test_decode_kernels_match_oracle_on_the_emulator(emu, server, slim):
    # 6 rows (two with the same length ratio as a real batch's tail), 4 frames, blank-biased joint;
    # slim 15: the co-resident step kernels (the default), 0: the big-tile step kernels
    r = subprocess.run([emu, "6", "4", "5", str(server), "12"], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, RNNT_DEC_SLIM=slim))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bounds checks: ok" in r.stdout, r.stdout
    assert "tokens identical" in r.stdout, r.stdout
