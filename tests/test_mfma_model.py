"""Pin the oracle's bf16-MFMA accumulation model (oracle/rnnt_oracle.c mfma_group) to gfx950
hardware outputs: tests/golden/mfma_bf16_probe.npz holds v_mfma_f32_16x16x32_bf16 results
recorded on an MI355X by tools/probe/probe_bf16 (targeted alignment / tie / cancellation
tiles + random tiles of four operand distributions).  The decoder's bf16 dot products are
defined by this model, so the GPU decode can run on bf16 MFMA and stay bit-exact."""
import os

import numpy as np

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mfma_bf16_probe.npz")


def _bf2f(b):
    return (np.asarray(b, np.uint32) << 16).view(np.float32)


def test_oracle_mfma_model_matches_hardware(oracle):
    z = np.load(FIX, allow_pickle=False)
    A, Bt, C, D = _bf2f(z["A"]), _bf2f(z["Bt"]), z["C"], z["D"]
    nt = A.shape[0]
    a = np.repeat(A[:, :, None, :], 16, axis=2).reshape(-1, 32)  # output (t, m, n): A[t, m], Bt[t, n]
    b = np.repeat(Bt[:, None, :, :], 16, axis=1).reshape(-1, 32)
    out = oracle.mfma_bf16_dot(C.reshape(-1), a, b)
    bad = np.flatnonzero(out.view(np.int32) != D.reshape(-1).view(np.int32))
    assert bad.size == 0, f"{bad.size} of {out.size} outputs differ, first {bad[:5]}"
    assert nt > 1000


def test_mfma_model_is_not_a_plain_fma_chain(oracle):
    """1 + half an ulp + 2^-29 in one group: the MFMA sums the group before rounding (-> 1 + ulp);
    a k-ordered fmaf chain rounds the tie to even first (-> 1)."""
    acc = np.array([1.0], np.float32)
    a = np.zeros((1, 32), np.float32)
    a[0, 1], a[0, 2] = 2.0 ** -24, 2.0 ** -29
    b = np.ones((1, 32), np.float32)
    assert oracle.mfma_bf16_dot(acc, a, b)[0] == np.float32(1.0 + 2.0 ** -23)
    chain = np.float32(1.0)
    for k in range(32):
        chain = np.float32(np.float64(chain) + np.float64(a[0, k]) * np.float64(b[0, k]))
    assert chain == np.float32(1.0)
