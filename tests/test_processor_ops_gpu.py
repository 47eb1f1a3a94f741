"""The operators the reference's f32 prediction network and its audio processor graph bind
(torch.ops.intel_mlperf.lstm, preemphasis, power_spectrum, frame_splicing, i_layernorm_pad) on the
GPU, through the op library as the TorchScript graphs call them.

* lstm (modeling_rnnt.py:204): bit-identical to the CPU restatement's fp32 prediction
  (oracle_prediction, k-ordered fp32 chains -- the contract the fused fp32 decoder already meets).
* The processor graph (FilterbankFeatures.forward, features.py:185-252) run op by op with torch's
  own stft / baddbmm / log between the plugin ops: within FEAT_TOL of the float64 restatement
  (oracle/featurizer.py), the same bound the fused featurizer meets; lengths and padding exact.
* Each plugin op alone: preemphasis, power_spectrum and frame_splicing bit-exact against a numpy
  float32 restatement of the same operations; i_layernorm_pad within 1e-5 of float64.  The plugin's
  own source is absent: these semantics are restated from the call sites (parity unpinned).
"""
import numpy as np
import pytest
import torch

from oracle import featurizer as OF
from rnnt_amd import ops, synthetic, weights
from rnnt_amd.featurizer import make_window, mel_filterbank

pytestmark = pytest.mark.gpu
FEAT_TOL = 2e-3


@pytest.fixture(scope="module")
def lib():
    return ops.load_library()


def test_lstm_f32_op_matches_restatement(lib, oracle):
    pm32, _ = weights.build_model(bf16=False)
    N = 70  # two 64-row tiles, the second partly padding
    rng = np.random.default_rng(7)
    pre_g = rng.integers(-1, 28, N).astype(np.int32)
    pre_g[:3] = -1  # SOS rows
    h = (rng.standard_normal((2, N, 320)) * 0.5).astype(np.float32)
    c = rng.standard_normal((2, N, 320)).astype(np.float32)
    emb = np.asarray(pm32.embed, np.float32)
    x = np.where(pre_g[:, None] < 0, 0.0, emb[np.maximum(pre_g, 0)]).astype(np.float32)
    wl = [[torch.from_numpy(np.ascontiguousarray(a, np.float32)) for a in
           (pm32.pred_wih[l], pm32.pred_whh[l], pm32.pred_bih[l], pm32.pred_bhh[l])] for l in range(2)]
    g, hg, cg = lib.lstm(torch.from_numpy(x)[None].cuda(), [torch.from_numpy(h[l]).cuda() for l in range(2)],
                         [torch.from_numpy(c[l]).cuda() for l in range(2)], wl)
    torch.cuda.synchronize()
    go, ho, co = oracle.prediction(pm32, pre_g, h, c)
    assert tuple(g.shape) == (1, N, 320)
    np.testing.assert_array_equal(g[0].cpu().numpy().view(np.uint32), go.view(np.uint32))
    for l in range(2):
        np.testing.assert_array_equal(hg[l].cpu().numpy().view(np.uint32), ho[l].view(np.uint32))
        np.testing.assert_array_equal(cg[l].cpu().numpy().view(np.uint32), co[l].view(np.uint32))


def _processor(lib, x, x_lens, window, fb, n_pad):
    """FilterbankFeatures.forward (features.py:185-252) with the rnnt.toml [input_eval] geometry,
    deterministic dithering (x += dither^2 after the power spectrum, :218-220)."""
    N = x.shape[0]
    x = lib.preemphasis(x, x_lens, coeff=0.97, pad_size=256)
    x = torch.stft(x, n_fft=512, hop_length=160, win_length=320, center=False, window=window,
                   return_complex=False).permute(0, 2, 1, 3)
    x_lens = torch.floor(x_lens / 160 + 1).to(dtype=torch.int32)
    x = lib.power_spectrum(x, x_lens).permute(0, 2, 1)
    x = x + 1e-5 ** 2
    fbt = torch.from_numpy(fb).cuda()[None]
    x = torch.log(torch.baddbmm(torch.full((1, 80, 1), 1e-20, device="cuda").expand(N, -1, -1),
                                fbt.expand(N, -1, -1), x))
    x = lib.frame_splicing(x, x_lens, 3)
    x_lens = torch.ceil(x_lens / 3).to(dtype=torch.int32)
    max_len = 1680
    shape = torch.tensor((n_pad, 256, max_len), dtype=torch.int32)
    return lib.i_layernorm_pad(x, torch.ones((1, 256, max_len)), torch.zeros((1, 256, max_len)), x_lens, 1e-12,
                               unbiased=1, output_shape=shape)


def test_processor_graph_on_the_ops(lib):
    L = [16000, 8000, 4001, 480, 1]
    wavs = synthetic.make_wavs(L, seed=31)
    x = torch.zeros((len(L), max(L)), dtype=torch.float32)
    for i, w in enumerate(wavs):
        x[i, : len(w)] = w
    window = torch.from_numpy(make_window("hann", 320)).cuda()
    fb = mel_filterbank(16000, 512, 80)
    y, yl = _processor(lib, x.cuda(), torch.tensor(L, dtype=torch.int32).cuda(), window, fb, n_pad=32)
    torch.cuda.synchronize()
    T = y.shape[2]
    ref, rlen = OF.featurize([w.double().numpy() for w in wavs], make_window("hann", 320), fb, n_pad=32, T_out=T)
    assert tuple(y.shape) == (32, 256, T)
    np.testing.assert_array_equal(yl.cpu().numpy(), rlen)
    got = y.permute(2, 0, 1).cpu().numpy()
    assert np.all(got[ref == 0.0] == 0.0)
    err = np.abs(got.astype(np.float64) - ref).max()
    assert err <= FEAT_TOL, err


def _mirror(p, L):
    return OF.mirror_index(np.asarray(p), L)


def test_preemphasis_op_exact(lib):
    rng = np.random.default_rng(3)
    lens = np.array([5, 300, 1, 0, 257], np.int32)
    Lmax, pad = 300, 256
    x = (rng.standard_normal((len(lens), Lmax)) * 0.1).astype(np.float32)
    y = lib.preemphasis(torch.from_numpy(x).cuda(), torch.from_numpy(lens).cuda(), coeff=0.97, pad_size=pad)
    torch.cuda.synchronize()
    y = y.cpu().numpy()
    assert y.shape == (len(lens), Lmax + 2 * pad)
    for n, Ln in enumerate(lens):
        want = np.zeros(Lmax + 2 * pad, np.float32)
        if Ln > 0:
            z = x[n, :Ln].copy()
            z[1:] = x[n, 1:Ln] - np.float32(0.97) * x[n, : Ln - 1]
            want[: Ln + 2 * pad] = z[_mirror(np.arange(-pad, Ln + pad), Ln)]
        np.testing.assert_array_equal(y[n].view(np.uint32), want.view(np.uint32), err_msg=f"row {n}")


def test_power_spectrum_and_frame_splicing_ops_exact(lib):
    rng = np.random.default_rng(4)
    N, T = 3, 11
    frames = np.array([11, 4, 0], np.int32)
    z = rng.standard_normal((N, T, 257, 2)).astype(np.float32)
    p = lib.power_spectrum(torch.from_numpy(z).cuda(), torch.from_numpy(frames).cuda()).cpu().numpy()
    want = z[..., 0] * z[..., 0] + z[..., 1] * z[..., 1]
    want[np.arange(T)[None, :] >= frames[:, None]] = 0.0
    np.testing.assert_array_equal(p.view(np.uint32), want.view(np.uint32))
    m = rng.standard_normal((N, 80, T)).astype(np.float32)
    s = lib.frame_splicing(torch.from_numpy(m).cuda(), torch.from_numpy(frames).cuda(), 3).cpu().numpy()
    To = -(-T // 3)
    assert s.shape == (N, 240, To)
    want = np.zeros((N, 240, To), np.float32)
    for n in range(N):
        for t in range(To):
            for q in range(3):
                if 3 * t + q < frames[n]:
                    want[n, 80 * q:80 * q + 80, t] = m[n, :, 3 * t + q]
    np.testing.assert_array_equal(s, want)


def test_layernorm_pad_op(lib):
    rng = np.random.default_rng(5)
    N, C, T = 3, 240, 9
    lens = np.array([9, 1, 4], np.int32)
    x = rng.standard_normal((N, C, T)).astype(np.float32) * 3 + 1
    w = torch.from_numpy(rng.uniform(0.5, 1.5, (1, 256, 16)).astype(np.float32))
    b = torch.from_numpy(rng.uniform(-0.1, 0.1, (1, 256, 16)).astype(np.float32))
    y, yl = lib.i_layernorm_pad(torch.from_numpy(x).cuda(), w, b, torch.from_numpy(lens).cuda(), 1e-12, unbiased=1,
                                output_shape=torch.tensor((8, 256, 16), dtype=torch.int32))
    y = y.cpu().numpy()
    assert y.shape == (8, 256, T) and yl.cpu().tolist() == [9, 1, 4, 0, 0, 0, 0, 0]
    want = np.zeros((8, 256, T))
    for n in range(N):
        Tn = lens[n]
        v = x[n, :, :Tn].astype(np.float64)
        mu = v.mean(axis=1, keepdims=True)
        var = ((v - mu) ** 2).sum(axis=1, keepdims=True) / (Tn - 1) if Tn > 1 else np.zeros((C, 1))
        want[n, :C, :Tn] = (v - mu) / np.sqrt(var + 1e-12) * w.numpy()[0, :C, :Tn] + b.numpy()[0, :C, :Tn]
    assert np.abs(y - want).max() < 1e-5
    assert np.all(y[:, C:] == 0) and np.all(y[N:] == 0)
