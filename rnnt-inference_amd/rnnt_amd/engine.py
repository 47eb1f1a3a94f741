"""Engine: the per-GPU RNN-T worker object over the C ABI.

One ``Engine`` per GPU replaces the reference's per-socket ``TorchModel`` clones
(csrc/rnnt_model.hpp:39-137): ``encode``/``decode`` are TorchModel::encode / decode, with the
same result contract (res [N][max_res] int32 filled with SOS=-1, res_len = res_idx+1).
Device memory and streams come from PyTorch (plumbing only); all compute is in the HIP
library.
"""
import ctypes as C

import numpy as np

from . import _lib
from .config import RNNTParam as R
from .weights import PreparedModel, f32_to_bf16_bits

BATCH_TILE = 256


def pad_batch(n):
    return (n + BATCH_TILE - 1) // BATCH_TILE * BATCH_TILE


def _stream_handle(stream):
    import torch
    if stream is None:
        stream = torch.cuda.current_stream()
    return C.c_void_p(stream.cuda_stream)


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


class Engine:
    def __init__(self, pm: PreparedModel, device=0, max_batch=1024, max_frames=R.MAX_FEA_LEN, max_res=None,
                 _path=None):
        if pm is not None and not pm.bf16:
            raise ValueError("the engine is created from the int8 + bf16 model (enable_bf16); the fp32 path is "
                             "loaded on top with load_f32_encoder / load_f32_decoder")
        lib = _lib.lib()
        self.device = device
        self.max_frames = max_frames
        self.max_res = max_res or (max_frames // 2) * R.max_symbols_per_step
        self.max_batch = pad_batch(max_batch)
        keep = []

        def arr(a, dt):
            a = np.ascontiguousarray(a, dtype=dt)
            keep.append(a)
            return a.ctypes.data

        def bf(a):
            return arr(f32_to_bf16_bits(np.asarray(a, np.float32)), np.uint16)

        opts = _lib.RnntOpts(self.max_batch, max_frames, self.max_res)
        h = C.c_void_p()
        self._lib = lib
        if _path is not None:  # C-side loader (rnnt_engine_create_from_file)
            _lib.check(lib.rnnt_engine_create_from_file(str(_path).encode(), device, C.byref(opts), C.byref(h)),
                       "rnnt_engine_create_from_file")
            self._h = h
            return
        d = _lib.RnntModelDesc()
        for l in range(5):
            d.enc_w[l] = arr(pm.enc_w[l], np.int8)
            d.enc_bq[l] = arr(pm.enc_bq[l], np.float32)
            d.enc_rb[l] = float(pm.enc_rb[l])
            d.enc_in_s[l] = float(pm.enc_in_s[l])
            d.enc_out_s[l] = float(pm.enc_out_s[l])
        d.embed = bf(pm.embed)
        for l in range(2):
            d.pred_w_ih[l] = bf(pm.pred_wih[l])
            d.pred_w_hh[l] = bf(pm.pred_whh[l])
            d.pred_b_ih[l] = arr(pm.pred_bih[l], np.float32)
            d.pred_b_hh[l] = arr(pm.pred_bhh[l], np.float32)
        d.joint_w1t = bf(pm.w1t)
        d.joint_w1p = bf(pm.w1p)
        d.joint_bt = arr(pm.bt, np.float32)
        d.joint_bp = arr(pm.bp, np.float32)
        d.joint_w2 = bf(pm.w2)
        d.joint_b2 = arr(pm.b2, np.float32)
        _lib.check(lib.rnnt_engine_create(C.byref(d), device, C.byref(opts), C.byref(h)), "rnnt_engine_create")
        self._h = h

    @classmethod
    def from_file(cls, path, device=0, max_batch=1024, max_frames=R.MAX_FEA_LEN, max_res=None):
        """An engine loaded by the C ABI from an engine model file (weights.save_engine_file /
        tools/export_model.py --engine-file): the path a C++ SUT takes."""
        return cls(None, device=device, max_batch=max_batch, max_frames=max_frames, max_res=max_res, _path=path)

    # ---------------------------------------------------------------- batch API
    def encode(self, feats, lens, lens_host=None, n=None, f_out=None, stream=None):
        """feats: cuda fp32 [T, n_pad, 256]; lens: cuda int32 [n_pad]; lens_host: numpy [n]."""
        T, n_pad, ch = feats.shape
        assert ch == R.PADDED_INPUT_SIZE and feats.is_contiguous() and lens.is_contiguous()
        n = n if n is not None else (len(lens_host) if lens_host is not None else n_pad)
        lh = None
        if lens_host is not None:
            lh = np.ascontiguousarray(lens_host, np.int32)
        rc = self._lib.rnnt_engine_encode(self._h, _ptr(feats), _ptr(lens), lh.ctypes.data if lh is not None else None,
                                          T, n, n_pad, _ptr(f_out), _stream_handle(stream))
        _lib.check(rc, "rnnt_engine_encode")

    def encode_gather(self, store, offsets, lens, lens_host, T, n, n_pad, f_out=None, stream=None):
        """encode with AssembleSamples fused into the quantizer: store cuda fp32 [rows, 240] (the
        QSL's ragged samples), offsets cuda int64 [n], lens cuda int32 [n_pad], lens_host [n]."""
        assert store.is_contiguous() and store.shape[1] == R.trans_input_size and offsets.dtype.itemsize == 8
        lh = np.ascontiguousarray(lens_host, np.int32)
        rc = self._lib.rnnt_engine_encode_gather(self._h, _ptr(store), _ptr(offsets), _ptr(lens), lh.ctypes.data, T, n,
                                                 n_pad, _ptr(f_out), _stream_handle(stream))
        _lib.check(rc, "rnnt_engine_encode_gather")

    def encode_stream(self, store, offsets, lens, lens_host, reset, T, n, n_pad, stream=None):
        """One chunk of Server continuous batching (PipelineState, metadata.cpp:97-194): slot i's
        chunk is lens_host[i] frames from store row offsets[i]; reset cuda int32 [n_pad] flags the
        slots that start a new utterance (their LSTM state restarts at zero), the others carry
        their state from the previous chunk."""
        assert store.is_contiguous() and store.shape[1] == R.trans_input_size and offsets.dtype.itemsize == 8
        assert reset.dtype.itemsize == 4 and reset.numel() >= n_pad
        lh = np.ascontiguousarray(lens_host, np.int32)
        rc = self._lib.rnnt_engine_encode_stream(self._h, _ptr(store), _ptr(offsets), _ptr(lens), lh.ctypes.data,
                                                 _ptr(reset), T, n, n_pad, _stream_handle(stream))
        _lib.check(rc, "rnnt_engine_encode_stream")

    def decode_stream(self, res, res_len, reset, stream=None):
        """Greedy decode of the last stream chunk, carrying each slot's prediction state and result
        row (res cuda int32 [n, max_res], the same buffer every call); reset as for encode_stream."""
        rc = self._lib.rnnt_engine_decode_stream(self._h, _ptr(res), _ptr(res_len), res.shape[1], _ptr(reset),
                                                 _stream_handle(stream))
        _lib.check(rc, "rnnt_engine_decode_stream")

    def encode_stream_pl(self, store, offsets, lens, lens_host, reset, T, n, n_pad, stream=None):
        """Pipelined encode_stream (rnnt_engine_encode_stream_pl): chunk k+1's encode runs while
        chunk k decodes (decode_stream_pl from another thread).  Returns after chunk k-1's decode
        has taken its inputs; reset must stay unchanged until this chunk's decode completed."""
        assert store.is_contiguous() and store.shape[1] == R.trans_input_size and offsets.dtype.itemsize == 8
        assert reset.dtype.itemsize == 4 and reset.numel() >= n_pad
        lh = np.ascontiguousarray(lens_host, np.int32)
        rc = self._lib.rnnt_engine_encode_stream_pl(self._h, _ptr(store), _ptr(offsets), _ptr(lens),
                                                    lh.ctypes.data, _ptr(reset), T, n, n_pad,
                                                    _stream_handle(stream))
        _lib.check(rc, "rnnt_engine_encode_stream_pl")

    def decode_stream_pl(self, res, res_len, reset, stream=None):
        """Pipelined decode_stream: decodes the oldest chunk whose encode_stream_pl returned."""
        rc = self._lib.rnnt_engine_decode_stream_pl(self._h, _ptr(res), _ptr(res_len), res.shape[1], _ptr(reset),
                                                    _stream_handle(stream))
        _lib.check(rc, "rnnt_engine_decode_stream_pl")

    def decode(self, res, res_len, stream=None):
        """res: cuda int32 [n, max_res]; res_len: cuda int32 [n]."""
        rc = self._lib.rnnt_engine_decode(self._h, _ptr(res), _ptr(res_len), res.shape[1], _stream_handle(stream))
        _lib.check(rc, "rnnt_engine_decode")

    def infer(self, feats, lens, lens_host, res, res_len, n=None, stream=None):
        T, n_pad, _ = feats.shape
        n = n if n is not None else len(lens_host)
        lh = np.ascontiguousarray(lens_host, np.int32)
        rc = self._lib.rnnt_engine_infer(self._h, _ptr(feats), _ptr(lens), lh.ctypes.data, T, n, n_pad,
                                         _ptr(res), _ptr(res_len), res.shape[1], _stream_handle(stream))
        _lib.check(rc, "rnnt_engine_infer")

    # ---------------------------------------------------------------- fp32 transcription
    def load_f32_encoder(self, layers):
        """layers: 5 x (W_ih [4096, I], W_hh [4096, 1024], b_ih, b_hh) fp32 in the checkpoint's
        natural layout (weights.enc_layer_params), I = 240, 1024, 2048, 1024, 1024."""
        keep = [[np.ascontiguousarray(l[i], np.float32) for l in layers] for i in range(4)]
        arrs = [(C.c_void_p * 5)(*[a.ctypes.data for a in col]) for col in keep]
        _lib.check(self._lib.rnnt_engine_load_f32_encoder(self._h, *arrs), "rnnt_engine_load_f32_encoder")

    def load_f32_decoder(self, pm32):
        """fp32 prediction / joint weights (a PreparedModel built with bf16=False, natural
        layouts) for decode_f32 -- the run_mode="f32" decoder without enable_bf16."""
        if pm32.bf16:
            raise ValueError("load_f32_decoder takes the fp32 PreparedModel (prepare_model(..., bf16=False))")
        keep = []

        def arr(a):
            a = np.ascontiguousarray(a, dtype=np.float32)
            keep.append(a)
            return a.ctypes.data

        d = _lib.RnntF32DecoderDesc()
        d.embed = arr(pm32.embed)
        for l in range(2):
            d.pred_w_ih[l] = arr(pm32.pred_wih[l])
            d.pred_w_hh[l] = arr(pm32.pred_whh[l])
            d.pred_b_ih[l] = arr(pm32.pred_bih[l])
            d.pred_b_hh[l] = arr(pm32.pred_bhh[l])
        d.joint_w1t, d.joint_w1p = arr(pm32.w1t), arr(pm32.w1p)
        d.joint_bt, d.joint_bp = arr(pm32.bt), arr(pm32.bp)
        d.joint_w2, d.joint_b2 = arr(pm32.w2), arr(pm32.b2)
        _lib.check(self._lib.rnnt_engine_load_f32_decoder(self._h, C.byref(d)), "rnnt_engine_load_f32_decoder")

    def decode_f32(self, res, res_len, stream=None):
        """fp32 greedy decode of the last encode_f32 output: res cuda int32 [n, max_res], res_len [n]."""
        rc = self._lib.rnnt_engine_decode_f32(self._h, _ptr(res), _ptr(res_len), res.shape[1], _stream_handle(stream))
        _lib.check(rc, "rnnt_engine_decode_f32")

    def encode_f32(self, feats, lens, n, f_out=None, stream=None):
        """Transcription in fp32 (config 2): feats cuda fp32 [T, n_pad, 256], lens cuda int32
        [n_pad] -> f_out cuda fp32 [ceil(T/2), n_pad, 1024] (optional).  The engine keeps f for
        decode_f32 and, when n_pad fits the int8 workspace, a bf16 copy for decode (the
        f32 + enable_bf16 decoder)."""
        T, n_pad, ch = feats.shape
        assert ch == R.PADDED_INPUT_SIZE and feats.is_contiguous() and (f_out is None or f_out.is_contiguous())
        rc = self._lib.rnnt_engine_encode_f32(self._h, _ptr(feats), _ptr(lens), T, n, n_pad, _ptr(f_out),
                                              _stream_handle(stream))
        _lib.check(rc, "rnnt_engine_encode_f32")

    # ---------------------------------------------------------------- measurement
    def set_profiling(self, on=True):
        _lib.check(self._lib.rnnt_engine_set_profiling(self._h, int(bool(on))), "rnnt_engine_set_profiling")

    def set_tile(self, tile="auto"):
        """Pin the int8 encoder's tick tile ("big" / "small" / "tiny" / "mini"), restore the
        per-tick choice ("auto" = "ticks"), or run whole-call encodes of small batches (n_pad <= 256)
        as one persistent dataflow launch ("flow"); results are bit-identical
        either way (rnnt_engine_set_tile)."""
        _lib.check(self._lib.rnnt_engine_set_tile(self._h, str(tile).encode()), "rnnt_engine_set_tile")

    def set_decode_persist(self, rows):
        """Run a decode call's last steps, once at most `rows` (1..512; 0 = off) rows are live, as one
        persistent launch (rnnt_engine_set_decode_persist); tokens are identical.  The launch needs all
        its 48 + (joint row groups) workgroups resident at once: beside other engines' kernels a wait can
        time out, and the call then fails with "persistent decode timed out"."""
        _lib.check(self._lib.rnnt_engine_set_decode_persist(self._h, int(rows)), "rnnt_engine_set_decode_persist")

    def stats(self, reset=True):
        st = _lib.RnntStats()
        _lib.check(self._lib.rnnt_engine_get_stats(self._h, C.byref(st), int(bool(reset))), "rnnt_engine_get_stats")
        return {k: getattr(st, k) for k, _ in st._fields_}

    # ---------------------------------------------------------------- op-level API
    def lstm_int8(self, first, count, x, hx, cx, y, stream=None):
        T, n_pad = x.shape[0], x.shape[1]
        rc = self._lib.rnnt_op_lstm_int8(self._h, first, count, _ptr(x), T, n_pad, _ptr(hx), _ptr(cx), _ptr(y),
                                         _stream_handle(stream))
        _lib.check(rc, "rnnt_op_lstm_int8")

    def stack_time(self, x, x_lens, y, stream=None):
        T, n_pad, Cc = x.shape
        rc = self._lib.rnnt_op_stack_time(self._h, _ptr(x), _ptr(x_lens), T, n_pad, Cc, _ptr(y), _stream_handle(stream))
        _lib.check(rc, "rnnt_op_stack_time")

    # ---------------------------------------------------------------- op-level decode
    def op_lstm_bf16(self, x, hx, cx, hy, cy, stream=None):
        """x bf16-bits int16 [n_pad, 320]; hx/hy int16 [2, n_pad, 320]; cx/cy f32 [2, n_pad, 320]."""
        rc = self._lib.rnnt_op_lstm_bf16(self._h, _ptr(x), _ptr(hx), _ptr(cx), _ptr(hy), _ptr(cy), x.shape[0],
                                         _stream_handle(stream))
        _lib.check(rc, "rnnt_op_lstm_bf16")

    def op_joint_hidden(self, f, g, y1, stream=None):
        rc = self._lib.rnnt_op_joint_hidden(self._h, _ptr(f), _ptr(g), _ptr(y1), f.shape[0], _stream_handle(stream))
        _lib.check(rc, "rnnt_op_joint_hidden")

    def op_joint_logits(self, y1, logits, stream=None):
        rc = self._lib.rnnt_op_joint_logits(self._h, _ptr(y1), _ptr(logits), y1.shape[0], _stream_handle(stream))
        _lib.check(rc, "rnnt_op_joint_logits")

    def op_greedy_update(self, symbols, symbols_added, res, res_idx, f, f_lens, time_idx, fi, pre_g, pre_hg, pre_cg,
                         hg, cg, stream=None):
        """greedy_decode_update on the reference's operands (rnnt_op_greedy_update): symbols int64
        or int32 [n]; pre_hg / hg lists of 2 bf16 [n, 320]; pre_cg / cg lists of 2 fp32 [n, 320];
        f [Tp, f_batch, 1024].  Returns all(finished)."""
        import torch
        n = symbols.shape[0]

        def arr2(ts):
            return (C.c_void_p * 2)(*[t.data_ptr() for t in ts])

        rc = self._lib.rnnt_op_greedy_update(self._h, _ptr(symbols), int(symbols.dtype == torch.int64),
                                             _ptr(symbols_added), _ptr(res), _ptr(res_idx), _ptr(f), f.shape[1],
                                             _ptr(f_lens), _ptr(time_idx), _ptr(fi), _ptr(pre_g), arr2(pre_hg),
                                             arr2(pre_cg), arr2(hg), arr2(cg), n, res.shape[1], _stream_handle(stream))
        if rc < 0:
            _lib.check(rc, "rnnt_op_greedy_update")
        return rc == 1

    def close(self):
        if getattr(self, "_h", None):
            self._lib.rnnt_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def cu_mask_words(reserve_per_xcd, reserved=False, n_cu=256):
    """32-bit mask words over the MI355X's CUs: bit b = CU slot b // 8 of XCD b % 8.
    reserved=False: every CU except the first `reserve_per_xcd` slots of each XCD (the encoder's
    share); reserved=True: only those slots."""
    words = [0] * ((n_cu + 31) // 32)
    for b in range(n_cu):
        if (b // 8 < reserve_per_xcd) == reserved:
            words[b // 32] |= 1 << (b % 32)
    return words


class PartitionedStream:
    """A HIP stream restricted to a CU set (rnnt_stream_create), usable as a torch stream.
    cu_mask=None gives a plain non-blocking stream."""

    def __init__(self, device=0, cu_mask=None):
        import torch
        lib = _lib.lib()
        h = C.c_void_p()
        if cu_mask is None:
            rc = lib.rnnt_stream_create(device, None, 0, C.byref(h))
        else:
            arr = (C.c_uint32 * len(cu_mask))(*cu_mask)
            rc = lib.rnnt_stream_create(device, C.cast(arr, C.c_void_p), len(cu_mask), C.byref(h))
        _lib.check(rc, "rnnt_stream_create")
        self._h = h
        self.stream = torch.cuda.ExternalStream(h.value, device=torch.device("cuda", device))

    def close(self):
        if self._h:
            self.stream.synchronize()
            _lib.check(_lib.lib().rnnt_stream_destroy(self._h), "rnnt_stream_destroy")
            self._h = None
