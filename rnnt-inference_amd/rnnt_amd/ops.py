"""The ``torch.ops.intel_mlperf`` operator surface of the hot path, backed by the HIP engine.

Mirrors reference ``models/_C.py:15-51`` for the ops the RNN-T graph calls on its quantised
path, with the argument meaning the reference call sites give them:

  lstm_amx_int8(x, hx, cx, weights, rb_scale, in_scale, out_scale, skip_quant_y)
        quant_lstm.py:92-101 -- one whole iLSTM stack (pre_rnn: 2 layers, post_rnn: 3)
  stack_time(x, x_lens, factor)           modeling_rnnt.py:327
  greedy_decode(...) / transcription      the fused hot loop behind TorchModel::encode/decode

Weight layout: the reference pre-packs int8 weights into AMX tiles
(quant_modules.transpose_tile_weight); the engine packs its own MFMA layout from the
*natural* int8 matrices iLSTMLayer._quant_parameters computes (quant_lstm.py:193-215), so the
``weights`` argument here is [[W_ih_q, W_hh_q, b_ih, b_q], ...] in natural [4H, I] layout.
The kernels run on the weights bound at ``bind(engine, model)`` (the engine is the device-side
owner of the packed model, like the TorchScript module owns the reference's packed tensors);
the passed tensors are checked for shape and against the bound model.

Errors follow the reference's TORCH_CHECK convention: invalid arguments raise RuntimeError.
"""
import numpy as np

from .config import ENC_INPUT_SIZES, RNNTParam as R
from .engine import pad_batch

_bound = {"engine": None, "model": None}


def bind(engine, model):
    """Register the engine (and its PreparedModel) the ops dispatch to."""
    _bound["engine"], _bound["model"] = engine, model


def _engine():
    e = _bound["engine"]
    if e is None:
        raise RuntimeError("rnnt_amd.ops: no engine bound (call ops.bind(engine, model))")
    return e


def _check(cond, msg):
    if not cond:
        raise RuntimeError(msg)


def _pad_rows(t, n_pad, dim=1):
    import torch
    n = t.shape[dim]
    if n == n_pad:
        return t.contiguous()
    shape = list(t.shape)
    shape[dim] = n_pad
    out = torch.zeros(shape, dtype=t.dtype, device=t.device)
    out.narrow(dim, 0, n).copy_(t)
    return out


def lstm_amx_int8(x, hx, cx, weights, rb_scale, in_scale, out_scale, skip_quant_y):
    """quant_lstm.py:80-102.  pre_rnn: x fp32 [T, N, 240|256] (quantised with in_scale[0]),
    post_rnn: x int8 [T, N, 2048]; hx: list of int8 [N, 1024]; cx: list of fp16 [N, 1024].
    Returns (y, hx', cx'): y int8 [T, N, 1024], or fp32 when skip_quant_y (post_rnn)."""
    import torch
    e = _engine()
    pm = _bound["model"]
    L = len(weights)
    _check(L in (R.pre_num_layers, R.post_num_layers), "lstm_amx_int8: expected 2 (pre_rnn) or 3 (post_rnn) layers")
    first = 0 if L == R.pre_num_layers and x.dtype == torch.float32 else R.pre_num_layers
    _check(len(hx) == L and len(cx) == L, "lstm_amx_int8: hx/cx must have one tensor per layer")
    _check(bool(skip_quant_y) == (first + L == 5), "lstm_amx_int8: skip_quant_y is set exactly for post_rnn")
    for i, w in enumerate(weights):
        l = first + i
        K = ENC_INPUT_SIZES[l] + R.trans_hidden_size
        wih, whh = w[0], w[1]
        _check(tuple(wih.shape)[0] == 4 * R.trans_hidden_size and wih.shape[1] + whh.shape[1] in (K, K - 16),
               f"lstm_amx_int8: layer {i} weight shape {tuple(wih.shape)} / {tuple(whh.shape)}")
        if pm is not None:
            _check(float(rb_scale[i]) == float(pm.enc_rb[l]) and float(in_scale[i]) == float(pm.enc_in_s[l]),
                   "lstm_amx_int8: scales differ from the bound model")
    T, N = x.shape[0], x.shape[1]
    n_pad = pad_batch(N)
    if first == 0:
        xin = torch.zeros((T, n_pad, R.PADDED_INPUT_SIZE), dtype=torch.float32, device=x.device)
        xin[:, :N, : x.shape[2]] = x
    else:
        _check(x.dtype == torch.int8 and x.shape[2] == 2 * R.trans_hidden_size, "lstm_amx_int8: post_rnn x int8 [T,N,2048]")
        xin = _pad_rows(x, n_pad)
    h = torch.stack([_pad_rows(t, n_pad, 0) for t in hx]).contiguous()
    c = torch.stack([_pad_rows(t.view(torch.int16), n_pad, 0) for t in cx]).contiguous()
    ydt = torch.float32 if skip_quant_y else torch.int8
    y = torch.empty((T, n_pad, R.trans_hidden_size), dtype=ydt, device=x.device)
    e.lstm_int8(first, L, xin, h, c, y)
    return (y[:, :N], [h[i, :N] for i in range(L)], [c[i, :N].view(torch.float16) for i in range(L)])


def stack_time(x, x_lens, factor):
    """modeling_rnnt.py:326-328: int8 [T, N, C] -> [ceil(T/2), N, 2C], frames >= x_lens zeroed."""
    import torch
    _check(factor == R.stack_time_factor, "stack_time: factor must be 2")
    _check(x.dtype == torch.int8, "stack_time: int8 input")
    T, N, C = x.shape
    n_pad = pad_batch(N)
    xin = _pad_rows(x, n_pad)
    lens = torch.zeros(n_pad, dtype=torch.int32, device=x.device)
    lens[:N] = x_lens.to(torch.int32)
    y = torch.empty(((T + 1) // 2, n_pad, 2 * C), dtype=torch.int8, device=x.device)
    _engine().stack_time(xin, lens, y)
    return y[:, :N]


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
