"""ctypes wrapper of the C restatement (oracle/rnnt_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product package.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "librnnt_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        _lib = C.CDLL(_LIB)
        for name in ("oracle_exp", "oracle_sigmoid", "oracle_tanh"):
            f = getattr(_lib, name)
            f.restype = C.c_float
            f.argtypes = [C.c_float]
        _lib.oracle_num_threads.restype = C.c_int
        for name in ("oracle_f2h", "oracle_f2bf"):
            f = getattr(_lib, name)
            f.restype = C.c_uint16
            f.argtypes = [C.c_float]
        for name in ("oracle_h2f", "oracle_bf2f"):
            f = getattr(_lib, name)
            f.restype = C.c_float
            f.argtypes = [C.c_uint16]
        _lib.oracle_q8.restype = C.c_int8
        _lib.oracle_q8.argtypes = [C.c_float]
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _ptrs(arrs):
    return (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def quantize(x, scale):
    x = _c(x, np.float32)
    out = np.empty(x.shape, np.int8)
    lib().oracle_quantize(_p(x), C.c_int64(x.size), C.c_float(scale), _p(out))
    return out


def lstm_i8_layer(x, W, bq, rb, in_s, out_s, skip_quant_y, h, c):
    """x [T,N,I] int8; W [4H, I+H] int8; h [N,H] int8; c [N,H] uint16 (fp16 bits).
    Returns (y, h', c')."""
    x = _c(x, np.int8); W = _c(W, np.int8); bq = _c(bq, np.float32)
    T, N, I = x.shape
    H = W.shape[0] // 4
    h = _c(h, np.int8).copy(); c = _c(c, np.uint16).copy()
    y8 = np.zeros((T, N, H), np.int8) if not skip_quant_y else np.zeros(1, np.int8)
    y32 = np.zeros((T, N, H), np.float32) if skip_quant_y else np.zeros(1, np.float32)
    lib().oracle_lstm_i8_layer(T, N, I, H, _p(x), _p(W), _p(bq), C.c_float(rb), C.c_float(in_s),
                               C.c_float(out_s), int(bool(skip_quant_y)), _p(h), _p(c), _p(y8), _p(y32))
    return (y32 if skip_quant_y else y8), h, c


def stack_time_i8(x, lens):
    x = _c(x, np.int8); lens = _c(lens, np.int32)
    T, N, Cc = x.shape
    y = np.empty(((T + 1) // 2, N, 2 * Cc), np.int8)
    lib().oracle_stack_time_i8(T, N, Cc, _p(x), _p(lens), _p(y))
    return y


def encoder_i8(pm, feat, lens, h_state=None, c_state=None):
    """feat [T,N,256] f32 -> f [ceil(T/2), N, 1024] f32 (PreparedModel pm)."""
    feat = _c(feat, np.float32); lens = _c(lens, np.int32)
    T, N, _ = feat.shape
    f = np.empty(((T + 1) // 2, N, 1024), np.float32)
    W = [_c(w, np.int8) for w in pm.enc_w]
    bq = [_c(b, np.float32) for b in pm.enc_bq]
    rb = _c(pm.enc_rb, np.float32); ins = _c(pm.enc_in_s, np.float32); outs = _c(pm.enc_out_s, np.float32)
    hp = _p(h_state) if h_state is not None else None
    cp = _p(c_state) if c_state is not None else None
    lib().oracle_encoder_i8(T, N, _p(feat), _p(lens), _ptrs(W), _ptrs(bq), _p(rb), _p(ins), _p(outs), _p(f), hp, cp)
    return f


def encoder_f32(layers, feat, lens):
    """layers: list of 5 (W_ih, W_hh, b_ih, b_hh) fp32; feat [T,N,I0]."""
    feat = _c(feat, np.float32); lens = _c(lens, np.int32)
    T, N, I0 = feat.shape
    f = np.empty(((T + 1) // 2, N, 1024), np.float32)
    cols = [[_c(l[i], np.float32) for l in layers] for i in range(4)]
    lib().oracle_encoder_f32(T, N, I0, _p(feat), _p(lens), _ptrs(cols[0]), _ptrs(cols[1]), _ptrs(cols[2]),
                             _ptrs(cols[3]), _p(f))
    return f


def _dec_args(pm):
    keep = dict(embed=_c(pm.embed, np.float32), wih=[_c(w, np.float32) for w in pm.pred_wih],
                whh=[_c(w, np.float32) for w in pm.pred_whh], bih=[_c(b, np.float32) for b in pm.pred_bih],
                bhh=[_c(b, np.float32) for b in pm.pred_bhh], w1t=_c(pm.w1t, np.float32),
                w1p=_c(pm.w1p, np.float32), bt=_c(pm.bt, np.float32), bp=_c(pm.bp, np.float32),
                w2=_c(pm.w2, np.float32), b2=_c(pm.b2, np.float32))
    return keep


def greedy_decode(pm, f, f_lens, max_res=None):
    """f [Tp,N,1024] f32, f_lens [N] -> (res [N,max_res] int32, res_len [N], steps [N,2])."""
    return greedy_decode_caps(pm, f, f_lens, max_res)[:3]


def greedy_decode_caps(pm, f, f_lens, max_res=None):
    """greedy_decode + caps [N]: advances forced by the 30-symbols-per-frame cap (decoder.py:131-136)."""
    return greedy_decode_walks(pm, f, f_lens, max_res)[:4]


def greedy_decode_walks(pm, f, f_lens, max_res=None):
    """greedy_decode_caps + walks [N,5]: lock-step steps per row when one joint launch may walk up to
    1, 2, 3, 4, 8 frames (diagnostics for the engine's walk cap)."""
    f = _c(f, np.float32); f_lens = _c(f_lens, np.int32)
    Tp, N, _ = f.shape
    max_res = max_res or max(1, Tp * 30)
    res = np.empty((N, max_res), np.int32); res_len = np.empty(N, np.int32); steps = np.empty((N, 2), np.int32)
    caps = np.empty(N, np.int32)
    walks = np.empty((N, 5), np.int32)
    k = _dec_args(pm)
    lib().oracle_greedy_decode_walks(Tp, N, _p(f), _p(f_lens), int(bool(pm.bf16)), _p(k["embed"]), _ptrs(k["wih"]),
                                    _ptrs(k["whh"]), _ptrs(k["bih"]), _ptrs(k["bhh"]), _p(k["w1t"]), _p(k["w1p"]),
                                    _p(k["bt"]), _p(k["bp"]), _p(k["w2"]), _p(k["b2"]), _p(res), _p(res_len),
                                    max_res, _p(steps), _p(caps), _p(walks))
    return res, res_len, steps, caps, walks


def joint(pm, f, g):
    f = _c(f, np.float32); g = _c(g, np.float32)
    N = f.shape[0]
    out = np.empty((N, 29), np.float32)
    k = _dec_args(pm)
    lib().oracle_joint(N, _p(f), _p(g), int(bool(pm.bf16)), _p(k["w1t"]), _p(k["w1p"]), _p(k["bt"]),
                       _p(k["bp"]), _p(k["w2"]), _p(k["b2"]), _p(out))
    return out


def prediction(pm, pre_g, h, c):
    """pre_g [N] int32; h, c [2,N,320] f32 -> (g [N,320], h' [2,N,320], c' [2,N,320])."""
    pre_g = _c(pre_g, np.int32); h = _c(h, np.float32); c = _c(c, np.float32)
    N = pre_g.shape[0]
    g = np.empty((N, 320), np.float32); ho = np.empty_like(h); co = np.empty_like(c)
    k = _dec_args(pm)
    lib().oracle_prediction(N, _p(pre_g), _p(h), _p(c), int(bool(pm.bf16)), _p(k["embed"]), _ptrs(k["wih"]),
                            _ptrs(k["whh"]), _ptrs(k["bih"]), _ptrs(k["bhh"]), _p(g), _p(ho), _p(co))
    return g, ho, co


def infer_i8(pm, feat, lens):
    """Whole int8 pipeline: encoder_i8 + greedy decode; returns (res, res_len, f, steps)."""
    f = encoder_i8(pm, feat, lens)
    f_lens = (np.asarray(lens, np.int32) + 1) // 2
    res, res_len, steps = greedy_decode(pm, f, f_lens)
    return res, res_len, f, steps


def mfma_bf16_dot(acc, a, b):
    """acc [N] f32, a/b [N][K] bf16-exact f32 -> [N] f32 under the bf16-MFMA accumulation model."""
    acc = _c(acc, np.float32)
    a = _c(a, np.float32)
    b = _c(b, np.float32)
    N, K = a.shape
    out = np.empty(N, np.float32)
    lib().oracle_mfma_bf16_dot(C.c_int(N), C.c_int(K), _p(acc), _p(a), _p(b), _p(out))
    return out
