"""CPU checks of the featurizer restatement (oracle/featurizer.py) against torch itself.

The reference's torch stages -- torch.stft(n_fft=512, hop_length=160, win_length=320,
center=False, window=hann(320, periodic=False)) on the pre-emphasised, n_fft/2-padded rows
(features.py:196-210), baddbmm with the filterbank + 1e-20 bias and log (:224-230) -- are run here
in float64 with the same arguments and compared with the oracle, pinning the framing, window
placement and stage order.  The plugin stages (preemphasis padding, frame_splicing,
i_layernorm_pad) are compared with torch restatements of their readable counterparts
(torch.stft center=True reflect padding, splice_frames :80-93, normalize_batch :52-78 with the
plugin's eps), since the plugin itself is absent.
"""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rnnt-inference_amd"))
sys.path.insert(0, ROOT)

from oracle import featurizer as OF  # noqa: E402
from rnnt_amd import featurizer as Fz  # noqa: E402
from rnnt_amd import synthetic as S  # noqa: E402

WIN = torch.hann_window(320, periodic=False, dtype=torch.float64)


def _rows():
    L = [16000, 3001, 480 * 7, 300, 257, 96000]  # torch reflect needs L > 256
    return [w.double().numpy() for w in S.make_wavs(L, seed=11)]


@pytest.mark.parametrize("i", range(6))
def test_stft_power_matches_torch(i):
    x = _rows()[i]
    F, _ = OF.frames(len(x))
    ours = OF.power_spectrum(OF.preemphasis_padded(x, 0.97), F, WIN.numpy())
    y = x.copy()
    y[1:] = x[1:] - 0.97 * x[:-1]
    yt = torch.from_numpy(y)[None]
    # the reference's call (features.py:202-210) on the plugin-padded row ...
    padded = torch.nn.functional.pad(yt[None], (256, 256), mode="reflect")[0]
    s = torch.stft(padded, n_fft=512, hop_length=160, win_length=320, center=False, window=WIN, return_complex=True)
    ref = (s.abs() ** 2)[0].T.numpy()
    assert ref.shape == ours.shape == (F, 257)
    np.testing.assert_allclose(ours, ref, rtol=1e-9, atol=1e-12 * ref.max())
    # ... which is torch.stft(center=True)'s own reflect padding for a single row
    s2 = torch.stft(yt, n_fft=512, hop_length=160, win_length=320, center=True, pad_mode="reflect", window=WIN,
                    return_complex=True)
    np.testing.assert_allclose((s2.abs() ** 2)[0].T.numpy(), ref, rtol=1e-12, atol=1e-15 * ref.max())


def test_logmel_matches_baddbmm():
    x = _rows()[0]
    F, _ = OF.frames(len(x))
    fb = Fz.mel_filterbank()
    p = OF.power_spectrum(OF.preemphasis_padded(x), F, WIN.numpy())
    ours = OF.log_mel(p, fb)
    pt = torch.from_numpy(p.T)[None] + 1e-5 ** 2
    ref = torch.log(torch.baddbmm(torch.full((1, 80, 1), 1e-20, dtype=torch.float64),
                                  torch.from_numpy(fb.astype(np.float64))[None], pt))[0].T.numpy()
    np.testing.assert_allclose(ours, ref, rtol=1e-12, atol=1e-12)


def _splice_frames_torch(x, k):
    # [1, C, F] -> [1, C*k, ceil(F/k)]: channel block q of output frame j = input frame k*j + q
    # (zero past the end), the behaviour of splice_frames (features.py:80-93)
    seq = [x]
    for n in range(1, k):
        shifted = torch.zeros_like(x)
        shifted[:, :, : x.shape[2] - n] = x[:, :, n:]
        seq.append(shifted)
    return torch.cat(seq, 1)[:, :, ::k]


@pytest.mark.parametrize("F", [1, 2, 3, 4, 5, 47, 48, 49, 100])
def test_splice_matches_splice_frames(F):
    mel = np.random.default_rng(F).standard_normal((F, 80))
    T = -(-F // 3)
    ref = _splice_frames_torch(torch.from_numpy(mel.T)[None], 3)[0].T.numpy()
    assert ref.shape == (T, 240)
    np.testing.assert_array_equal(OF.splice(mel, T), ref)


@pytest.mark.parametrize("T", [1, 2, 7, 160])
def test_normalize_matches_layernorm(T):
    x = np.random.default_rng(T).standard_normal((T, 240)) * 3 + 1
    xt = torch.from_numpy(x)
    if T > 1:
        ref = ((xt - xt.mean(0)) / torch.sqrt(xt.var(0, unbiased=True) + 1e-12)).numpy()
    else:
        ref = np.zeros_like(x)
    np.testing.assert_allclose(OF.normalize(x), ref, rtol=1e-12, atol=1e-12)


def test_frames_and_lengths():
    for L, (F, T) in {0: (0, 0), 1: (1, 1), 159: (1, 1), 160: (2, 1), 479: (3, 1), 480: (4, 2),
                      240000: (1501, 501), 239999: (1500, 500)}.items():
        assert OF.frames(L) == (F, T)
    frames = np.array([1, 2, 47, 500])
    L = S.wav_lengths_for_frames(frames, seed=3)
    assert [OF.frames(int(v))[1] for v in L] == frames.tolist()


def test_short_rows_mirror():
    # rows shorter than the 256-sample pad: periodic mirror; one-sample rows repeat the sample
    assert OF.preemphasis_padded(np.array([2.0]), 0.97).tolist() == [2.0] * 513
    p = OF.preemphasis_padded(np.arange(5.0), 0.0, pad=6)
    assert p.tolist() == [2, 3, 4, 3, 2, 1, 0, 1, 2, 3, 4, 3, 2, 1, 0, 1, 2]


def test_mel_filterbank_slaney():
    fb = Fz.mel_filterbank()
    assert fb.shape == (80, 257) and fb.dtype == np.float32 and (fb >= 0).all()
    # slaney area normalisation: the wide (upper) triangles integrate to ~1 over Hz
    area = fb.sum(1) * (8000.0 / 256)
    assert np.all(np.abs(area[35:] - 1.0) < 0.03) and np.all(np.abs(area - 1.0) < 0.15)
    # filters peak in increasing bins; each filter's non-zero weights are one contiguous span
    peaks = fb.argmax(1)
    assert np.all(np.diff(peaks) >= 0)
    for row in fb:
        nz = np.nonzero(row)[0]
        assert len(nz) and nz[-1] - nz[0] + 1 == len(nz)
    assert (fb > 0).sum() <= 2048  # the kernel's LDS span budget


def test_oracle_layout():
    wavs = _rows()[:3]
    feats, lens = OF.featurize(wavs, WIN.numpy(), Fz.mel_filterbank(), n_pad=8, T_out=40)
    assert feats.shape == (40, 8, 256) and lens.tolist()[:3] == [OF.frames(len(w))[1] for w in wavs]
    assert np.all(feats[:, :, 240:] == 0) and np.all(feats[:, 3:] == 0)
    for n in range(3):
        t = lens[n]
        assert np.all(feats[t:, n] == 0)
        np.testing.assert_allclose(feats[:t, n, :240].mean(0), 0, atol=1e-9)
