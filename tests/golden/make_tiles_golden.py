"""Generate tests/golden/tiles.npz: digests of the REFERENCE's prepacked weight tiles.

Build-container only (imports /root/reference/models/quant_modules.py, which never travels to the
GPU box):  python -B tests/golden/make_tiles_golden.py
For the golden model (the seeded checkpoint quantised with the reference's calibrated amax of
golden.npz) it packs every weight the reference graph hands its ops with the reference's own
transpose_tile_weight / transpose_tile_weight_bf16 (quant_modules.py:158-193), exactly as
iLSTMLayer._quant_parameters (quant_lstm.py:193-215), Prediction.prepack_weights
(modeling_rnnt.py:161-181) and Joint.prepack_weights (:223-257) call them, and stores sha256 of
the packed bytes (data only).  rnnt_amd.ops.amx_tiles_* must reproduce them (tests/test_ops_lib.py).
"""
import hashlib
import os
import sys

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference
import numpy as np  # noqa: E402
import torch  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "rnnt-inference_amd"))
import types  # noqa: E402

sys.modules["_C"] = types.ModuleType("_C")  # the absent plugin; packing needs none of its ops
sys.path.insert(0, "/root/reference/models")
import quant_modules as ref_qm  # noqa: E402

from rnnt_amd import synthetic, weights  # noqa: E402


def sha(t):
    return np.frombuffer(hashlib.sha256(t.contiguous().view(torch.uint8).numpy().tobytes()).hexdigest().encode(), np.uint8)


def main():
    golden = np.load(os.path.join(REPO, "tests", "golden", "golden.npz"))
    pm = weights.prepare_model(synthetic.make_checkpoint(synthetic.DEFAULT_SEED), golden["calib_amax"], bf16=True)
    out = {}
    H = 1024
    for l in range(5):
        w = torch.from_numpy(pm.enc_w[l])
        I = w.shape[1] - H
        wih = w[:, :240] if l == 0 else w[:, :I]
        out[f"enc{l}_ih"] = sha(ref_qm.transpose_tile_weight(wih.t().contiguous(), l == 0))
        out[f"enc{l}_hh"] = sha(ref_qm.transpose_tile_weight(w[:, I:].t().contiguous()))
    bf = lambda a: torch.from_numpy(np.asarray(a, np.float32)).to(torch.bfloat16)  # noqa: E731
    for l in range(2):
        out[f"pred{l}_ih"] = sha(ref_qm.transpose_tile_weight_bf16(bf(pm.pred_wih[l]).t().contiguous()))
        out[f"pred{l}_hh"] = sha(ref_qm.transpose_tile_weight_bf16(bf(pm.pred_whh[l]).t().contiguous()))
    out["w1t"] = sha(ref_qm.transpose_tile_weight_bf16(bf(pm.w1t).t().contiguous()))
    out["w1p"] = sha(ref_qm.transpose_tile_weight_bf16(bf(pm.w1p).t().contiguous()))
    out["w2"] = sha(ref_qm.transpose_tile_weight_bf16(bf(pm.w2).t().contiguous(), True))
    assert not os.path.exists("/root/reference/models/__pycache__")
    np.savez(os.path.join(REPO, "tests", "golden", "tiles.npz"), **out)
    print({k: bytes(v).decode()[:12] for k, v in out.items()})


if __name__ == "__main__":
    main()
