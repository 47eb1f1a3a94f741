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


# ---------------------------------------------------------------- decode operators
# The reference's op-by-op greedy loop (models/decoder.py:171-212) calls these four; tensors use
# torch's bfloat16 / float32 / int32 dtypes and the reference's shapes.  Weight arguments are
# accepted for signature compatibility and checked against the bound model's shapes; the
# engine computes with its own packed copy (as for lstm_amx_int8).

def _bits(t):
    import torch
    return t.contiguous().view(torch.int16)


def lstm_amx_bf16(x, hx, cx, weights=None):
    """modeling_rnnt.py:202: x bf16 [1, N, 320]; hx: 2 x bf16 [N, 320]; cx: 2 x fp32 [N, 320]
    -> (g bf16 [1, N, 320], hy, cy)."""
    import torch
    e = _engine()
    N = x.shape[-2]
    _check(x.shape[-1] == R.pred_hidden_size and len(hx) == 2 and len(cx) == 2, "lstm_amx_bf16: bad shapes")
    n_pad = (N + 15) // 16 * 16
    xb = torch.zeros((n_pad, R.pred_hidden_size), dtype=torch.bfloat16, device=x.device)
    xb[:N] = x.reshape(N, -1)
    h = torch.zeros((2, n_pad, R.pred_hidden_size), dtype=torch.bfloat16, device=x.device)
    c = torch.zeros((2, n_pad, R.pred_hidden_size), dtype=torch.float32, device=x.device)
    for l in range(2):
        h[l, :N] = hx[l]
        c[l, :N] = cx[l]
    hy, cy = torch.empty_like(h), torch.empty_like(c)
    e.op_lstm_bf16(_bits(xb), _bits(h), c, _bits(hy).view(torch.int16), cy)
    return hy[1, :N].unsqueeze(0), [hy[0, :N], hy[1, :N]], [cy[0, :N], cy[1, :N]]


def amx_linear_bf16_accum_relu(f, w1_trans=None, g=None, w1_pred=None, bias=None):
    """modeling_rnnt.py:269-275: f [N, 1024] (fp32 or bf16), g bf16 [N, 320] -> y1 bf16 [N, 512]."""
    import torch
    e = _engine()
    N = f.shape[0]
    n_pad = (N + 15) // 16 * 16
    fp = torch.zeros((n_pad, R.trans_hidden_size), dtype=torch.float32, device=f.device)
    fp[:N] = f.float()
    gp = torch.zeros((n_pad, R.pred_hidden_size), dtype=torch.bfloat16, device=f.device)
    gp[:N] = g.reshape(N, -1)
    y1 = torch.empty((n_pad, R.joint_hidden_size), dtype=torch.bfloat16, device=f.device)
    e.op_joint_hidden(fp, _bits(gp), y1.view(torch.int16))
    return y1[:N]


def amx_linear_i16o32(y, w2=None, b2=None):
    """modeling_rnnt.py:280-283: y1 bf16 [N, 512] -> logits fp32 [N, 32] (29 labels + zero pad)."""
    import torch
    e = _engine()
    N = y.shape[0]
    n_pad = (N + 15) // 16 * 16
    yp = torch.zeros((n_pad, R.joint_hidden_size), dtype=torch.bfloat16, device=y.device)
    yp[:N] = y
    logits = torch.empty((n_pad, 32), dtype=torch.float32, device=y.device)
    e.op_joint_logits(yp.view(torch.int16), logits)
    return logits[:N]


def greedy_decode_update(symbols, symbols_added, res, res_idx, f, f_lens, time_idx, fi, pre_g, pre_hg, pre_cg, hg, cg,
                         finish):
    """modeling_rnnt.py:331-365 (spec decoder.py:125-167), in place.  Device tensors: symbols,
    symbols_added, res_idx, f_lens, time_idx, finish int32 [N]; res int32 [N, max_res]; f fp32
    [T', n_pad, 1024]; fi fp32 [n_pad, 1024]; pre_g int32 [N]; pre_hg / hg bf16 [2, n_pad, 320];
    pre_cg / cg fp32 [2, n_pad, 320].  Returns all(finish)."""
    import torch
    e = _engine()
    N = symbols.shape[0]
    return e.op_greedy_update(symbols.to(torch.int32).contiguous(), symbols_added, res, res_idx, f, f_lens, time_idx, fi,
                              pre_g, pre_hg.view(torch.int16), pre_cg, hg.view(torch.int16), cg, finish, N)
