"""Audio front end on the HIP featurizer: the reference's FilterbankFeatures / AudioProcessing.

Mirrors ``FilterbankFeatures`` (reference datasets/parts/features.py:98-270),
``FeatureFactory`` (:273-286) and ``AudioProcessing`` (datasets/process_librispeech.py:100-111):
same constructor arguments and defaults, same ``forward(x, x_lens, pad_batch_size) -> (x, x_lens)``
with x [N_pad][C][T] (C = 256 with pad_out_feat, else 240) and N_pad = ceil(N/32)*32 when
pad_batch_size (features.py:239-241).  Every batch runs through ``rnnt_featurizer_run``
(csrc/featurizer.hip); there is no CPU path.  ``featurize`` is the native entry point that
writes the engine's input layout [T][n_pad][256] directly (no permute copy) and reads ragged
sample storage through per-row offsets.

Module buffers are built like the reference's __init__ (features.py:134-160): the window with
torch's window functions (periodic=False) and the filterbank with a restatement of
``librosa.filters.mel`` (slaney mel scale and area normalisation, the default of the
unpinned librosa that prepare_conda_env.sh:7 installs -- librosa is absent here, so the
filterbank values are "parity unpinned"; callers holding librosa's matrix can pass it as ``fb``).
"""
import ctypes as C
import math
from contextlib import nullcontext as _nullctx

import numpy as np

from . import _lib
from .engine import _ptr, _stream_handle

SUPPORTED = dict(sample_rate=16000, n_fft=512, win_length=320, hop_length=160, nfilt=80, frame_splicing=3)


def _hz_to_mel(f):
    f = np.asarray(f, np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    lin = f / f_sp
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-30) / min_log_hz) / logstep, lin)


def _mel_to_hz(m):
    m = np.asarray(m, np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filterbank(sr=16000, n_fft=512, n_mels=80, fmin=0.0, fmax=None):
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax) with htk=False, norm='slaney',
    dtype float32: triangular filters between consecutive slaney-mel points, scaled to unit area
    (2 / bandwidth).  Returns float32 [n_mels][n_fft//2 + 1]."""
    fmax = float(sr) / 2 if fmax is None else fmax
    fftfreqs = np.linspace(0.0, float(sr) / 2, 1 + n_fft // 2)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    w = np.zeros((n_mels, 1 + n_fft // 2), np.float32)
    for i in range(n_mels):
        w[i] = np.maximum(0.0, np.minimum(-ramps[i] / fdiff[i], ramps[i + 2] / fdiff[i + 1]))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w


def make_window(kind, win_length):
    import torch
    fns = {"hann": torch.hann_window, "hamming": torch.hamming_window, "blackman": torch.blackman_window,
           "bartlett": torch.bartlett_window}
    if kind not in fns:
        raise ValueError(f"window {kind!r}: the featurizer needs a window function (features.py:121-127)")
    return fns[kind](win_length, periodic=False).float().numpy()


def feature_frames(wav_len):
    """ceil((floor(wav_len/160) + 1) / 3) spliced frames (features.py:212, :237); 0 for no samples."""
    return int(_lib.lib().rnnt_featurizer_frames(int(wav_len)))


def write_processor_file(path, config=None, window=None, fb=None):
    """The processor file the C++ AudioProcessor drop-in loads (rnnt_featurizer_create_from_file,
    csrc/sut/rnnt_processor_mi355x.hpp) in place of the reference's TorchScript processor
    (rnnt_processor.hpp:17-22): the RNNTMI01 container with fz_config (the rnnt_featurizer_config
    fields in order), fz_window and fz_fb.  Defaults: configs/rnnt.toml [input_eval] (16 kHz, 20 ms
    hann window, 10 ms stride, n_fft 512, 80 filters, splicing 3, padded to 256 features)."""
    from .weights import write_pack_file
    if config is None:
        config = [16000, 512, 320, 160, 80, 3, 256, 0.97, 1e-5, 1e-20, 1e-12]
    if window is None:
        window = make_window("hann", int(config[2]))
    if fb is None:
        fb = mel_filterbank(int(config[0]), int(config[1]), int(config[4]), 0.0, config[0] / 2)
    return write_pack_file(path, {"fz_config": (1, np.asarray(config, np.float32)),
                                  "fz_window": (1, np.asarray(window, np.float32)),
                                  "fz_fb": (1, np.asarray(fb, np.float32))})


class FilterbankFeatures:
    """features.py:98-270 on the GPU (one native featurizer per instance and device)."""

    def __init__(self, sample_rate=8000, window_size=0.02, window_stride=0.01, window="hamming",
                 normalize="per_feature", n_fft=None, preemph=0.97, nfilt=64, lowfreq=0, highfreq=None,
                 log=True, dither=1e-5, pad_to=8, max_duration=16.7, frame_splicing=1, pad_out_feat=False,
                 device=0, fb=None):
        self.win_length = int(sample_rate * window_size)
        self.hop_length = int(sample_rate * window_stride)
        self.n_fft = n_fft or 2 ** math.ceil(math.log2(self.win_length))
        geo = dict(sample_rate=sample_rate, n_fft=self.n_fft, win_length=self.win_length,
                   hop_length=self.hop_length, nfilt=nfilt, frame_splicing=frame_splicing)
        if geo != SUPPORTED:
            raise ValueError(f"featurizer geometry {geo}: the HIP featurizer implements {SUPPORTED} "
                             "(configs/rnnt.toml [input_eval])")
        if normalize != "per_feature" or not log:
            raise ValueError("the HIP featurizer implements log filterbanks with per_feature normalisation")
        self.frame_splicing = frame_splicing
        self.normalize, self.log, self.dither, self.preemph = normalize, log, dither, preemph
        self.window = make_window(window, self.win_length)
        self.fb = (np.ascontiguousarray(fb, np.float32) if fb is not None else
                   mel_filterbank(sample_rate, self.n_fft, nfilt, lowfreq, highfreq or sample_rate / 2))
        self.out_feat = 256 if pad_out_feat else nfilt * frame_splicing
        max_length = 1 + math.ceil((max_duration * sample_rate - self.win_length) / self.hop_length)
        self.max_length = max_length + 16 - (max_length % 16)  # features.py:163-167 (STFT frames)
        self.device = device
        cfg = _lib.RnntFeaturizerConfig(sample_rate, self.n_fft, self.win_length, self.hop_length, nfilt,
                                        frame_splicing, 256, float(preemph or 0.0), float(dither), 1e-20, 1e-12)
        self.config = cfg
        L = _lib.lib()
        h = C.c_void_p()
        _lib.check(L.rnnt_featurizer_create(C.byref(cfg), self.window.ctypes.data_as(C.c_void_p),
                                            self.fb.ctypes.data_as(C.c_void_p), device, C.byref(h)),
                   "rnnt_featurizer_create")
        self._h = h

    def save_processor_file(self, path):
        """This featurizer's processor file (write_processor_file)."""
        c = self.config
        return write_processor_file(path, [c.sample_rate, c.n_fft, c.win_length, c.hop_length, c.nfilt,
                                           c.frame_splicing, c.pad_out_feat, c.preemph, c.dither, c.log_guard,
                                           c.norm_eps], self.window, self.fb)

    @classmethod
    def from_config(cls, cfg, log=False):
        """features.py:253-270."""
        return cls(sample_rate=cfg["sample_rate"], window_size=cfg["window_size"],
                   window_stride=cfg["window_stride"], n_fft=cfg["n_fft"], nfilt=cfg["features"],
                   window=cfg["window"], normalize=cfg["normalize"], max_duration=cfg.get("max_duration", 16.7),
                   dither=cfg["dither"], pad_to=cfg.get("pad_to", 0), frame_splicing=cfg.get("frame_splicing", 1),
                   log=log, pad_out_feat=cfg.get("pad_out_feat"))

    def featurize(self, wav, wav_lens, wav_lens_host=None, n=None, n_pad=None, T_out=None, offsets=None,
                  out=None, feat_lens=None, stream=None):
        """Native entry: wav cuda fp32 [N][stride] (zero-padded batch) or 1-D ragged storage with
        offsets (cuda int64 [n]); wav_lens cuda int32 [n].  Returns (feats [T_out][n_pad][256],
        feat_lens [n_pad] int32) on the device -- the engine's encode input."""
        import torch
        if wav_lens_host is None:
            wav_lens_host = wav_lens.cpu()
        lh = np.ascontiguousarray(np.asarray(wav_lens_host, dtype=np.int32))
        n = len(lh) if n is None else n
        n_pad = n if n_pad is None else n_pad
        if T_out is None:
            T_out = max([feature_frames(v) for v in lh[:n]] + [1])
        dev = wav.device
        if out is None:
            out = torch.empty((T_out, n_pad, 256), dtype=torch.float32, device=dev)
        if feat_lens is None:
            feat_lens = torch.empty(n_pad, dtype=torch.int32, device=dev)
        assert out.is_contiguous() and out.shape == (T_out, n_pad, 256) and out.dtype == torch.float32
        assert wav.dtype == torch.float32 and wav_lens.dtype == torch.int32 and wav.is_contiguous()
        if offsets is not None:
            assert offsets.dtype == torch.int64 and offsets.numel() >= n
            stride = 0
        else:
            assert wav.dim() == 2 and wav.shape[0] >= n
            stride = wav.shape[1]
        _lib.check(_lib.lib().rnnt_featurizer_run(self._h, _ptr(wav), _ptr(offsets), stride, _ptr(wav_lens),
                                                  lh.ctypes.data_as(C.c_void_p), n, n_pad, _ptr(out),
                                                  _ptr(feat_lens), T_out, _stream_handle(stream)),
                   "rnnt_featurizer_run")
        return out, feat_lens

    def featurize_rows(self, wav, wav_lens, wav_lens_host, out, row_off, max_frames, offsets=None, feat_lens=None,
                       stream=None):
        """Ragged entry for a feature store (rnnt_featurizer_run_rows): sample i's frames written as
        240-channel rows out[row_off[i] + t] (out cuda fp32 [rows][240]; row_off host int64 [n],
        bounds-checked against out here, then uploaded), nothing else touched; each sample's frames
        <= max_frames.  Returns feat_lens cuda int32 [n]."""
        import torch
        lh = np.ascontiguousarray(np.asarray(wav_lens_host, dtype=np.int32))
        n = len(lh)
        dev = wav.device
        if feat_lens is None:
            feat_lens = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        assert out.is_contiguous() and out.dim() == 2 and out.shape[1] == 240 and out.dtype == torch.float32
        assert wav.dtype == torch.float32 and wav.is_contiguous() and wav_lens.dtype == torch.int32
        ro = np.ascontiguousarray(np.asarray(row_off, dtype=np.int64))
        if ro.shape != (n,):
            raise ValueError("row_off must hold one row offset per sample")
        fr = np.array([feature_frames(int(v)) for v in lh], np.int64)
        if n and fr.max() > max_frames:
            raise ValueError("a sample's feature frames exceed max_frames")
        if n and (ro.min() < 0 or (ro + fr).max() > out.shape[0]):
            raise ValueError("row_off places a sample outside the store")
        with torch.cuda.stream(stream) if stream is not None else _nullctx():  # ordered before the kernels
            row_off = torch.from_numpy(ro).to(dev)
        if offsets is not None:
            assert offsets.dtype == torch.int64 and offsets.numel() >= n
            stride = 0
        else:
            assert wav.dim() == 2 and wav.shape[0] >= n
            stride = wav.shape[1]
        _lib.check(_lib.lib().rnnt_featurizer_run_rows(self._h, _ptr(wav), _ptr(offsets), stride, _ptr(wav_lens),
                                                       lh.ctypes.data_as(C.c_void_p), n, _ptr(out), _ptr(row_off),
                                                       _ptr(feat_lens), int(max_frames), _stream_handle(stream)),
                   "rnnt_featurizer_run_rows")
        return feat_lens

    def forward(self, x, x_lens, pad_batch_size):
        """features.py:185-252: x cuda fp32 [N][max_len] (zero-padded), x_lens int32 [N] ->
        (x [N_pad][C][T], x_lens [N_pad])."""
        n = x.shape[0]
        n_pad = (n + 31) // 32 * 32 if pad_batch_size else n
        import torch
        feats, lens = self.featurize(x.contiguous(), x_lens.to(device=x.device, dtype=torch.int32), n=n, n_pad=n_pad)
        return feats[:, :, :self.out_feat].permute(1, 2, 0), lens

    __call__ = forward

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().rnnt_featurizer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FeatureFactory:
    """features.py:273-286."""
    featurizers = {"logfbank": FilterbankFeatures, "fbank": FilterbankFeatures}

    @classmethod
    def from_config(cls, cfg):
        feat_type = cfg.get("feat_type", "logspect")
        return cls.featurizers[feat_type].from_config(cfg, log="log" in feat_type)


class AudioProcessing:
    """datasets/process_librispeech.py:100-111 (the processor_jit.pt module the C++ SUT runs)."""

    def __init__(self, run_mode, **kwargs):
        kwargs["pad_out_feat"] = run_mode == "quant"
        self.featurizer = FeatureFactory.from_config(kwargs)

    def forward(self, wavs, wav_lens, pad_batch_size):
        return self.featurizer(wavs, wav_lens, pad_batch_size)

    __call__ = forward


def load_toml(path, section="input_eval"):
    """The [input_eval] table of configs/rnnt.toml (the featurizer's kwargs)."""
    import tomli
    with open(path, "rb") as f:
        return dict(tomli.load(f)[section])
