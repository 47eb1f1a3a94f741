"""The compiled TorchModel replacement (rnnt-inference_amd/csrc/sut/rnnt_model_mi355x.hpp, INTEGRATION.md
section 1) run as the reference's OfflineSUT runs TorchModel.

The harness (csrc/sut/sut_harness.cpp, built by the Makefile against include/rnnt_mi355x.h and libtorch)
loads the engine file tools/export_model.py writes, sorts the samples longest first, assembles batches,
and per batch calls state.update -> model.encode -> model.decode and completes every sample the way
QuerySamplesComplete does (csrc/torch_sut.cpp:221-236): (state.res_[i].data_ptr(), (res_idx_[i] + 1) * 4
bytes).  Checked here: every sample answered once; each payload equals the CPU restatement's tokens,
so res_idx_ = length - 1 (metadata.cpp:59-60); and the harness itself checks the -1 (SOS) fill of
res_ past each row's tokens."""
import json
import os
import subprocess

import numpy as np
import pytest

from rnnt_amd import synthetic, weights

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(REPO, "rnnt-inference_amd", "rnnt_amd", "rnnt_sut_harness")


def _responses(path):
    b = open(path, "rb").read()
    out, off = {}, 0
    while off < len(b):
        sid, size = np.frombuffer(b, np.int32, 2, off)
        off += 8
        assert int(sid) not in out, f"sample {sid} answered twice"
        out[int(sid)] = np.frombuffer(b, np.int32, int(size) // 4, off).copy()
        off += int(size)
    return out


def test_cpp_torch_model_state_contract(tmp_path, oracle):
    assert os.path.exists(HARNESS), "harness not built (make -C rnnt-inference_amd/csrc)"
    pm, _ = weights.build_model()
    eng_file = weights.save_engine_file(pm, str(tmp_path / "rnnt.engine"))
    lens = np.array([57, 0, 31, 12, 44, 3, 50, 29, 38, 9, 61, 22, 47, 17, 5, 33, 26, 1, 40, 60], np.int32)
    N, T = len(lens), int(lens.max())
    x = synthetic.make_features(T, N, seed=24, lens=lens)[:, :, :240]  # [T][N][240]
    np.ascontiguousarray(x.transpose(1, 0, 2)).tofile(tmp_path / "feats.bin")  # [N][T][240]
    lens.tofile(tmp_path / "lens.bin")
    out = tmp_path / "responses.bin"
    env = dict(os.environ)
    r = subprocess.run([HARNESS, eng_file, str(tmp_path / "feats.bin"), str(tmp_path / "lens.bin"), str(N), str(T),
                        "8", str(out)], capture_output=True, text=True, timeout=90, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert summary == {"batches": 3, "responses": N, "bad_sos_fill_rows": 0, "bad_res_idx_rows": 0}, summary
    got = _responses(out)
    assert sorted(got) == list(range(N))
    fo = oracle.encoder_i8(pm, np.pad(x, ((0, 0), (0, 0), (0, 16))), lens)
    ro, rlo, _ = oracle.greedy_decode(pm, fo, (lens + 1) // 2, max_res=(500 // 2) * 30)
    assert rlo.max() > 3 and rlo[1] == 0
    for i in range(N):
        np.testing.assert_array_equal(got[i], ro[i, : rlo[i]], err_msg=f"sample {i}")
