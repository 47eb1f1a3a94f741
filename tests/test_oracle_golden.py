"""Pin the oracle (CPU restatement) and the host-side model build against fixtures generated
from the reference's own Python modules (tests/golden/make_golden.py)."""
import hashlib
import math

import numpy as np
import pytest

from rnnt_amd import synthetic, weights


def test_checkpoint_regenerates_bit_exactly(ckpt, golden):
    assert synthetic.checkpoint_digest(ckpt) == bytes(golden["digest"]).decode()


def test_quantised_params_match_reference(pm_golden, golden):
    """iLSTMLayer._quant_parameters + _propagate_quantizers (quant_lstm.py:66-78, 193-215),
    bit-exact: int8 weights (sha256 of the unpacked reference tiles), fused biases, scales."""
    pm = pm_golden
    for l in range(5):
        w = pm.enc_w[l]
        assert hashlib.sha256(w.tobytes()).hexdigest() == bytes(golden[f"q_w{l}_sha"]).decode(), f"layer {l}"
        np.testing.assert_array_equal(w[::257], golden[f"q_w{l}_rows"])
        np.testing.assert_array_equal(pm.enc_bq[l].view(np.uint32), golden[f"q_bq{l}"].view(np.uint32))
    np.testing.assert_array_equal(pm.enc_in_s[:2], golden["q_pre_rnn_in"])
    np.testing.assert_array_equal(pm.enc_in_s[2:], golden["q_post_rnn_in"])
    np.testing.assert_array_equal(pm.enc_out_s[:2], golden["q_pre_rnn_out"])
    np.testing.assert_array_equal(pm.enc_out_s[2:], golden["q_post_rnn_out"])  # last = inf
    np.testing.assert_array_equal(pm.enc_rb[:2], golden["q_pre_rnn_rb"])
    np.testing.assert_array_equal(pm.enc_rb[2:], golden["q_post_rnn_rb"])
    np.testing.assert_array_equal(pm.bt + pm.bp, golden["q_joint_b1"])
    np.testing.assert_array_equal(np.pad(pm.b2, (0, 3)), golden["q_joint_b2"])


def test_calibration_matches_reference(ckpt, golden):
    """TensorQuantizer calib_amax over cat([x_t, h_{t-1}]) (quant_modules.py:110-115)."""
    cl = np.full(2, 120, np.int32)
    xc = synthetic.make_features(120, 2, seed=synthetic.DEFAULT_SEED ^ 0xCA1B, lens=cl)
    amax = weights.calibrate_amax(weights.migrate_state_dict(ckpt), xc, cl)
    np.testing.assert_allclose(amax, golden["calib_amax"], rtol=2e-6)


def _valid(f, lens):
    fl = (np.asarray(lens) + 1) // 2
    return [(t, n) for n in range(f.shape[1]) for t in range(fl[n])]


@pytest.fixture(scope="module")
def f32_out(oracle, ckpt, golden):
    sd = weights.migrate_state_dict(ckpt)
    layers = [weights.enc_layer_params(sd, l) for l in range(5)]
    return oracle.encoder_f32(layers, golden["a_x"], golden["a_lens"])


def test_f32_transcription_matches_reference(f32_out, golden):
    """QuantLSTMLayer fp32 x5 + StackTime.forward_f32 (modeling_rnnt.py:116-144, 314-324).
    Dot-product order differs (fmaf chain vs MKL sgemm) -> tolerance on valid frames."""
    ref = golden["a_f32_f"]
    idx = _valid(ref, golden["a_lens"])
    a = np.stack([f32_out[t, n] for t, n in idx])
    b = np.stack([ref[t, n] for t, n in idx])
    assert np.max(np.abs(a - b)) < 2e-4, np.max(np.abs(a - b))


def test_f32_decode_matches_reference(oracle, pm_f32, f32_out, golden):
    """greedy_decode_f32 (decoder.py:102-169) on the oracle's fp32 encoder output."""
    fl = (golden["a_lens"] + 1) // 2
    res, rl, steps = oracle.greedy_decode(pm_f32, f32_out, fl)
    np.testing.assert_array_equal(rl, golden["a_f32_len"])
    for n in range(len(rl)):
        np.testing.assert_array_equal(res[n, :rl[n]], golden["a_f32_res"][n, :rl[n]])
    np.testing.assert_array_equal(steps, golden["a_f32_steps"])


def test_split_len_chunking_is_invariant(golden):
    """decoder.py:80-91 split_len=2 chunked decode == unsplit (reference-level fact the
    engine relies on: its encoder runs the whole time axis in one pass)."""
    np.testing.assert_array_equal(golden["a_f32_split2_len"], golden["a_f32_len"])
    np.testing.assert_array_equal(golden["a_f32_split2_res"], golden["a_f32_res"])


def test_single_utterance_config1(oracle, ckpt, pm_f32, golden):
    sd = weights.migrate_state_dict(ckpt)
    layers = [weights.enc_layer_params(sd, l) for l in range(5)]
    x1 = golden["c1_x"]
    f = oracle.encoder_f32(layers, x1, np.array([x1.shape[0]], np.int32))
    res, rl, _ = oracle.greedy_decode(pm_f32, f, np.array([(x1.shape[0] + 1) // 2], np.int32))
    assert rl[0] == golden["c1_len"][0]
    np.testing.assert_array_equal(res[0, :rl[0]], golden["c1_res"][0, :rl[0]])


def test_int8_encoder_tracks_reference_fake_quant(oracle, pm_golden, golden):
    """The int8 restatement (exact int32 GEMM, fp16 cell) vs the reference's own float
    restatement of the same quantised model (run_mode fake_quant): same quantisation grid,
    so outputs agree to a few int8 LSBs of the last layer's input scale."""
    x = np.pad(golden["a_x"], ((0, 0), (0, 0), (0, 16)))
    f = oracle.encoder_i8(pm_golden, x, golden["a_lens"])
    ref = golden["a_fq_f"]
    lsb = 1.0 / pm_golden.enc_in_s[4]
    # first stacked frames: the two restatements differ only by fp32 rounding inside the
    # quantisation grid (sub-LSB); later frames accumulate occasional 1-LSB flips through
    # the recurrence, so the bound is looser there.
    early = np.abs(f[:3, :3] - ref[:3, :3]) / lsb
    assert early.mean() < 0.5 and early.max() < 4, (early.mean(), early.max())
    idx = _valid(ref, golden["a_lens"])
    err = np.abs(np.stack([f[t, n] for t, n in idx]) - np.stack([ref[t, n] for t, n in idx])) / lsb
    assert err.mean() < 4, err.mean()


def test_numerics_primitives(oracle):
    lib = oracle.lib()
    xs = np.linspace(-30, 30, 20001).astype(np.float32)
    e = np.array([lib.oracle_exp(float(v)) for v in xs[::7]], np.float64)
    ref = np.exp(xs[::7].astype(np.float64))
    assert np.max(np.abs(e / ref - 1)) < 3e-7
    s = np.array([lib.oracle_sigmoid(float(v)) for v in xs[::3]])
    assert np.max(np.abs(s - 1 / (1 + np.exp(-xs[::3].astype(np.float64))))) < 2e-7
    t = np.array([lib.oracle_tanh(float(v)) for v in xs[::3]])
    assert np.max(np.abs(t - np.tanh(xs[::3].astype(np.float64)))) < 3e-7
    # fp16 / bf16 conversions vs numpy / the torch formula
    v = (np.random.default_rng(0).standard_normal(20000) * 300).astype(np.float32)
    v[:6] = [0.0, -0.0, 65504.0, 65520.0, 6e-8, 3e-5]
    h = np.array([lib.oracle_f2h(C_float(x)) for x in v], np.uint16)
    np.testing.assert_array_equal(h, v.astype(np.float16).view(np.uint16))
    bf = np.array([lib.oracle_f2bf(C_float(x)) for x in v], np.uint16)
    np.testing.assert_array_equal(bf, weights.f32_to_bf16_bits(v))
    q = oracle.quantize(np.array([0.5, 1.5, 2.5, -0.5, -127.6, 127.5, 200, -200], np.float32), 1.0)
    np.testing.assert_array_equal(q, [0, 2, 2, 0, -128, 127, 127, -128])
    assert math.isclose(lib.oracle_h2f(0x3C00), 1.0)


def C_float(x):
    import ctypes
    return ctypes.c_float(float(x))


# ---- the 30-symbols-per-frame cap (decoder.py:131-136, 153-167)
@pytest.fixture(scope="module")
def cap_ckpt(golden):
    ck = synthetic.make_checkpoint(synthetic.DEFAULT_SEED, synthetic.CAP_RECIPE)
    assert synthetic.checkpoint_digest(ck) == bytes(golden["cap_digest"]).decode()
    return ck


def test_cap_f32_decode_matches_reference(oracle, cap_ckpt, golden):
    """The reference's greedy_decode_f32 on the cap checkpoint (make_golden.py asserts it hits
    max_symbols_per_step on most rows): the restatement reproduces its tokens, its (advance, emit)
    counters and its count of cap-forced advances per row."""
    sd = weights.migrate_state_dict(cap_ckpt)
    layers = [weights.enc_layer_params(sd, l) for l in range(5)]
    x, lens = golden["cap_x"], golden["cap_lens"]
    f = oracle.encoder_f32(layers, x, lens)
    fl = (lens + 1) // 2
    ref = golden["cap_f32_f"]
    for n in range(len(lens)):
        assert np.abs(f[: fl[n], n] - ref[: fl[n], n]).max() < 2e-4
    pm = weights.prepare_model(cap_ckpt, np.ones(5, np.float32), bf16=False)
    res, rl, steps, caps = oracle.greedy_decode_caps(pm, f, fl)
    assert caps.max() > 0
    np.testing.assert_array_equal(caps, golden["cap_f32_caps"])
    np.testing.assert_array_equal(steps, golden["cap_f32_steps"])
    np.testing.assert_array_equal(rl, golden["cap_f32_len"])
    for n in range(len(rl)):
        np.testing.assert_array_equal(res[n, : rl[n]], golden["cap_f32_res"][n, : rl[n]])


def test_cap_int8_bf16_restatement_hits_the_cap(oracle, cap_ckpt, golden):
    """The int8 encoder + bf16 decoder restatement on the cap model reaches the cap branch too
    (the case tests/test_cap_gpu.py runs the GPU paths on)."""
    from rnnt_amd.config import RNNTParam as R
    x, lens = golden["cap_x"], golden["cap_lens"]
    amax = weights.calibrate_amax(weights.migrate_state_dict(cap_ckpt), np.pad(x, ((0, 0), (0, 0), (0, 16))), lens)
    pm = weights.prepare_model(cap_ckpt, amax, bf16=True)
    f = oracle.encoder_i8(pm, np.pad(x, ((0, 0), (0, 0), (0, 16))), lens)
    res, rl, steps, caps = oracle.greedy_decode_caps(pm, f, (lens + 1) // 2)
    assert (caps > 0).sum() >= 3, caps
    assert (steps[:, 1] >= R.max_symbols_per_step * caps).all()
