"""The ``torch.ops.intel_mlperf`` operator surface of the hot path.

The reference's graph binds its ops from a loaded library (models/_C.py:9-51); this package
builds the MI355X one, ``libintel_mlperf_mi355x.so`` (csrc/torch_ops.cpp), which registers the
same namespace and the schemas the call sites imply (quant_lstm.py:92-101, modeling_rnnt.py:202,
269-283, 326-328, 351-365).  ``load_library()`` makes ``torch.ops.intel_mlperf.*`` available to
Python and TorchScript (torch.jit.script / torch.jit.load graphs bind to it unchanged); the
module-level functions below are those ops, so ``from rnnt_amd import ops as P`` can stand in
for the reference's ``import _C as P``.

The ops compute with the weights they are passed, in the reference's prepacked layouts
(``reference_weights`` builds them from a PreparedModel exactly as the reference's model build
does) or natural layouts.  ``transcription`` / ``greedy_decode`` are the fused engine paths
behind TorchModel::encode / decode (bound with ``bind``), used by GreedyDecoder.

Errors follow the reference's TORCH_CHECK convention: invalid arguments raise RuntimeError.
"""
import os

import numpy as np

from .config import RNNTParam as R
from .engine import pad_batch

_HERE = os.path.dirname(os.path.abspath(__file__))
OPS_LIB = os.path.join(_HERE, "libintel_mlperf_mi355x.so")
_loaded = False
_bound = {"engine": None, "model": None}


def load_library(path=OPS_LIB):
    """torch.ops.load_library of the operator library (no fallback: a missing library raises)."""
    global _loaded
    if not _loaded:
        import torch
        from . import _lib
        if not os.path.exists(path):
            raise RuntimeError(f"operator library missing: {path} (build with `make -C {_lib.CSRC}`)")
        _lib.lib()  # the engine first: torch's HIP runtime, one per process
        torch.ops.load_library(path)
        _loaded = True
    import torch
    return torch.ops.intel_mlperf


def op_weight_loads():
    """Weight-set loads the operator library has done for the calling thread (an engine loads a
    weight set the first time it sees it; a changed weight tensor reloads).  Diagnostics, not a
    reference op."""
    import ctypes
    load_library()
    f = ctypes.CDLL(OPS_LIB).intel_mlperf_mi355x_weight_loads
    f.restype = ctypes.c_int64
    return int(f())


def op_engine_count(device=0):
    """Engines in the operator library's pool of `device`: the peak number of concurrent op calls
    seen there (calls lease an engine each; threads own none)."""
    import ctypes
    load_library()
    f = ctypes.CDLL(OPS_LIB).intel_mlperf_mi355x_engine_count
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int]
    return int(f(int(device)))


def release_engines():
    """Free the operator library's idle engines on every device (device memory); the next op call
    creates and loads a new one.  -> engines freed."""
    import ctypes
    load_library()
    f = ctypes.CDLL(OPS_LIB).intel_mlperf_mi355x_release_engines
    f.restype = ctypes.c_int
    return int(f())


def release_thread_engines():
    """Round-4 name of release_engines (engines are no longer owned by threads)."""
    release_engines()


def lstm_amx_int8(x, hx, cx, weights, rb_scale, in_scale, out_scale, skip_quant_y):
    """quant_lstm.py:92-101: one iLSTM stack (pre_rnn 2 layers on fp32 x, post_rnn 3 on int8)."""
    return load_library().lstm_amx_int8(x, hx, cx, weights, rb_scale, in_scale, out_scale, skip_quant_y)


def stack_time(x, x_lens, factor):
    """modeling_rnnt.py:326-328."""
    return load_library().stack_time(x, x_lens, factor)


def lstm_amx_bf16(x, hx, cx, weights):
    """modeling_rnnt.py:202."""
    return load_library().lstm_amx_bf16(x, hx, cx, weights)


def amx_linear_bf16_accum_relu(f, w1_trans, g, w1_pred, bias):
    """modeling_rnnt.py:269-275."""
    return load_library().amx_linear_bf16_accum_relu(f, w1_trans, g, w1_pred, bias)


def amx_linear_i16o32(y, w2, b2):
    """modeling_rnnt.py:280-283: logits fp32 [N, 32] (29 labels + zero padding)."""
    return load_library().amx_linear_i16o32(y, w2, b2)


def greedy_decode_update(symbols, symbols_added, res, res_idx, f, f_lens, time_idx, fi, pre_g, pre_hg, pre_cg, hg, cg):
    """modeling_rnnt.py:331-365, in place; returns all(finished)."""
    return load_library().greedy_decode_update(symbols, symbols_added, res, res_idx, f, f_lens, time_idx, fi, pre_g,
                                               pre_hg, pre_cg, hg, cg)


# ---------------------------------------------------------------- reference-format weights
def amx_tiles_int8(wt):
    """transpose_tile_weight (quant_modules.py:175-191, padding=True) of W^T [K, O] int8:
    tiles [O/64][4][ceil(K/64)][16][64], element (k, o) at [o/64][(o%64)/16][k/64][(k%64)/4][4(o%16)+k%4]."""
    wt = np.asarray(wt, np.int8)
    K, O = wt.shape
    ct, cs = (K + 63) // 64, (O + 63) // 64
    w = np.zeros((ct * 64, cs * 64), np.int8)
    w[:K, :O] = wt
    # k = 64 kt + 4 r + kk, o = 64 s + 16 j + oo  ->  [s][j][kt][r][4 oo + kk]
    return np.ascontiguousarray(w.reshape(ct, 16, 4, cs, 4, 16).transpose(3, 4, 0, 1, 5, 2).reshape(cs, 4, ct, 16, 64))


def amx_tiles_bf16(wt_bits):
    """transpose_tile_weight_bf16 (quant_modules.py:158-172, padding=True) of W^T [K, O] (bf16 bits):
    tiles [ceil(O/32)][2][K/32][16][32], element (k, o) at [o/32][(o%32)/16][k/32][(k%32)/2][2(o%16)+k%2]."""
    wt = np.asarray(wt_bits, np.uint16)
    K, O = wt.shape
    ct, cs = (K + 31) // 32, (O + 31) // 32
    w = np.zeros((ct * 32, cs * 32), np.uint16)
    w[:K, :O] = wt
    # k = 32 kt + 2 r + kk, o = 32 s + 16 j + oo  ->  [s][j][kt][r][2 oo + kk]
    return np.ascontiguousarray(w.reshape(ct, 16, 2, cs, 2, 16).transpose(3, 4, 0, 1, 5, 2).reshape(cs, 2, ct, 16, 32))


def reference_weights(pm, device="cpu"):
    """The weight tensors the reference graph hands the ops, built from a PreparedModel the way
    the reference's model build lays them out: iLSTM.weights = [[tiles(W_ih_q^T), tiles(W_hh_q^T),
    b_ih, b_q]] + rb/in/out scale tensors (quant_lstm.py:193-215), Prediction weights =
    [[tiles(W_ih^T), tiles(W_hh^T), b_ih, b_hh + b_ih]] (modeling_rnnt.py:161-181), joint
    tiles + linear1 bias = b_trans + b_pred + zero-padded linear2 (:223-257)."""
    import torch
    from .weights import f32_to_bf16_bits
    H = R.trans_hidden_size

    def bft(a_bits):
        return torch.from_numpy(a_bits.view(np.int16)).view(torch.bfloat16).to(device)

    def f32(a):
        return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(device)

    enc = []
    for l in range(5):
        w = pm.enc_w[l]
        I = w.shape[1] - H
        wih = w[:, :I] if l else w[:, :R.trans_input_size]  # first layer: 240 real columns, padded by the tiling
        enc.append([torch.from_numpy(amx_tiles_int8(wih.T)).to(device), torch.from_numpy(amx_tiles_int8(w[:, I:].T)).to(device),
                    f32(np.zeros(4 * H)), f32(pm.enc_bq[l])])
    scales = {k: f32(getattr(pm, "enc_" + k)) for k in ("rb", "in_s", "out_s")}
    pred = []
    for l in range(R.pred_num_layers):
        pred.append([bft(amx_tiles_bf16(f32_to_bf16_bits(pm.pred_wih[l]).T)),
                     bft(amx_tiles_bf16(f32_to_bf16_bits(pm.pred_whh[l]).T)),
                     f32(pm.pred_bih[l]), f32(np.asarray(pm.pred_bhh[l], np.float32) + np.asarray(pm.pred_bih[l], np.float32))])
    joint = dict(w1_trans=bft(amx_tiles_bf16(f32_to_bf16_bits(pm.w1t).T)),
                 w1_pred=bft(amx_tiles_bf16(f32_to_bf16_bits(pm.w1p).T)),
                 bias=f32(np.asarray(pm.bt, np.float32) + np.asarray(pm.bp, np.float32)),
                 w2=bft(amx_tiles_bf16(f32_to_bf16_bits(pm.w2).T)), b2=f32(np.pad(pm.b2, (0, 3))))
    embed = bft(f32_to_bf16_bits(pm.embed))
    return dict(pre=enc[:2], post=enc[2:], pre_scales=[scales[k][:2] for k in ("rb", "in_s", "out_s")],
                post_scales=[scales[k][2:] for k in ("rb", "in_s", "out_s")], pred=pred, embed=embed, **joint)


def op_model(pm):
    """The PreparedModel the op path is numerically equivalent to: prediction b_hh recovered from
    the reference's fused slot as fp32((b_hh + b_ih) - b_ih) (csrc/torch_ops.cpp lstm_amx_bf16)."""
    import copy
    m = copy.copy(pm)
    m.pred_bhh = [((np.asarray(bh, np.float32) + np.asarray(bi, np.float32)) - np.asarray(bi, np.float32)).astype(np.float32)
                  for bh, bi in zip(pm.pred_bhh, pm.pred_bih)]
    return m


# ---------------------------------------------------------------- fused engine paths
def bind(engine, model):
    """Register the engine (and its PreparedModel) the fused transcription / greedy_decode use."""
    _bound["engine"], _bound["model"] = engine, model


def _engine():
    e = _bound["engine"]
    if e is None:
        raise RuntimeError("rnnt_amd.ops: no engine bound (call ops.bind(engine, model))")
    return e


def transcription(x, x_lens, f_out=True):
    """Transcription.forward for the whole batch (modeling_rnnt.py:116-144) on the engine:
    x fp32 [T, N, 240|256], x_lens [N] -> f fp32 [ceil(T/2), N, 1024].  The engine keeps the
    encoder state for a following ``greedy_decode`` (TorchModel::encode)."""
    import torch
    e = _engine()
    T, N = x.shape[0], x.shape[1]
    n_pad = pad_batch(N)
    xin = torch.zeros((T, n_pad, R.PADDED_INPUT_SIZE), dtype=torch.float32, device=x.device)
    xin[:, :N, : x.shape[2]] = x
    lens_host = np.asarray(x_lens.cpu(), np.int32)
    lens = torch.zeros(n_pad, dtype=torch.int32, device=x.device)
    lens[:N] = torch.from_numpy(lens_host).to(x.device)
    f = torch.empty(((T + 1) // 2, n_pad, R.trans_hidden_size), dtype=torch.float32, device=x.device) if f_out else None
    e.encode(xin, lens, lens_host, n=N, f_out=f)
    return f[:, :N] if f_out else None


def greedy_decode(n, max_res=None):
    """Prediction + joint + greedy_decode_update loop over the last transcription
    (TorchModel::decode, rnnt_model.hpp:92-124): -> (res int32 [n, max_res] filled with -1,
    res_len int32 [n])."""
    import torch
    e = _engine()
    max_res = max_res or e.max_res
    res = torch.empty((n, max_res), dtype=torch.int32, device="cuda")
    rl = torch.empty(n, dtype=torch.int32, device="cuda")
    e.decode(res, rl)
    return res, rl
