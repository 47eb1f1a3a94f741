"""Packed model export (tools/export_model.py, rnnt_amd.weights.save_prepared / load_prepared):
checkpoint file -> calibration -> quantisation -> .npz, equal to the in-memory build."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from rnnt_amd import synthetic, weights

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def built():
    return weights.build_model()


def test_roundtrip_and_digest(built, tmp_path):
    pm, _ = built
    p = str(tmp_path / "m.npz")
    meta = weights.save_prepared(pm, p)
    pm2, meta2 = weights.load_prepared(p)
    assert meta2["sha256"] == meta["sha256"] == weights.prepared_digest(pm)
    for i in range(5):
        np.testing.assert_array_equal(pm2.enc_w[i], pm.enc_w[i])
        np.testing.assert_array_equal(pm2.enc_bq[i], pm.enc_bq[i])
    np.testing.assert_array_equal(pm2.enc_in_s, pm.enc_in_s)
    assert pm2.bf16 == pm.bf16 and len(pm2.pred_wih) == 2
    # a corrupted array is caught by the digest
    with np.load(p, allow_pickle=False) as z:
        arrs = {k: z[k].copy() for k in z.files}
    arrs["enc_w_3"][0, 0] ^= 1
    bad = str(tmp_path / "bad.npz")
    np.savez(bad, **arrs)
    with pytest.raises(ValueError):
        weights.load_prepared(bad)


def test_export_tool_from_checkpoint_file(built, tmp_path):
    pm, ckpt = built
    pt = str(tmp_path / "rnnt.pt")
    torch.save({"state_dict": {k: torch.from_numpy(np.asarray(v)) for k, v in ckpt.items()}}, pt)
    out = str(tmp_path / "rnnt_quant.npz")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "export_model.py"), "--checkpoint", pt, "--out", out],
                   check=True, capture_output=True)
    pm2, meta = weights.load_prepared(out)
    assert meta["sha256"] == weights.prepared_digest(pm)  # same calibration batch -> identical model
    np.testing.assert_array_equal(pm2.amax, pm.amax)


def test_export_with_calibration_file(built, tmp_path):
    _, ckpt = built
    lens = np.array([30, 17], np.int32)
    feats = synthetic.make_features(30, 2, seed=5, lens=lens)
    cal = str(tmp_path / "calib.npz")
    np.savez(cal, feats=feats, lens=lens)
    out = str(tmp_path / "m.npz")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "export_model.py"), "--synthetic",
                    "--calib-features", cal, "--out", out], check=True, capture_output=True)
    pm2, _ = weights.load_prepared(out)
    np.testing.assert_array_equal(pm2.amax, weights.calibrate_amax(weights.migrate_state_dict(ckpt), feats, lens))
