"""Model build: checkpoint migration, calibration and quantisation (host side, numpy).

Restates the reference's model-build path:
  * ``migrate_state_dict``           reference models/utils.py:60-81
  * calibration (running amax of the LSTM input quantizers on cat([x_t, h_{t-1}]))
                                     quant_lstm.py:166-171, quant_modules.py:110-115
  * weight / bias quantisation       quant_lstm.py:193-215 (iLSTMLayer._quant_parameters)
  * scale propagation                quant_lstm.py:66-78, modeling_rnnt.py:62-77
  * bf16 prediction / joint prepack  modeling_rnnt.py:161-181, 223-257
The output ``PreparedModel`` keeps the reference's natural layouts; the engine packs its own
device layouts from them (rnnt_engine_create / rnnt_engine_load_*).
"""
from dataclasses import dataclass, field
from typing import List

import numpy as np

from .config import ENC_INPUT_SIZES, RNNTParam as R


def migrate_state_dict(model, split_fc1=True):
    """reference models/utils.py:60-81 (key renames + joint fc1 split into trans/pred)."""
    state_dict = model["state_dict"] if "state_dict" in model else model
    out = {}
    for key, value in state_dict.items():
        if key == "joint_net.0.weight" and split_fc1:
            out["joint.linear1_trans.weight"] = value[:, :1024]
            out["joint.linear1_pred.weight"] = value[:, 1024:]
            continue
        if key == "joint_net.0.bias" and split_fc1:
            out["joint.linear1_trans.bias"] = np.zeros(512, dtype=np.float32)
            out["joint.linear1_pred.bias"] = value
        key = key.replace("encoder.pre_rnn.lstm", "transcription.pre_rnn")
        key = key.replace("encoder.post_rnn.lstm", "transcription.post_rnn")
        key = key.replace("dec_rnn.lstm", "pred_rnn")
        key = key.replace("joint_net.0", "joint.linear1")
        key = key.replace("joint_net.3", "joint.linear2")
        out[key] = value
    out.pop("audio_preprocessor.featurizer.fb", None)
    out.pop("audio_preprocessor.featurizer.window", None)
    return out


def enc_layer_params(sd, layer):
    """(W_ih, W_hh, b_ih, b_hh) of encoder layer 0..4 from a migrated state dict."""
    stack, l = ("pre_rnn", layer) if layer < R.pre_num_layers else ("post_rnn", layer - R.pre_num_layers)
    p = f"transcription.{stack}."
    return (np.asarray(sd[p + f"weight_ih_l{l}"], np.float32), np.asarray(sd[p + f"weight_hh_l{l}"], np.float32),
            np.asarray(sd[p + f"bias_ih_l{l}"], np.float32), np.asarray(sd[p + f"bias_hh_l{l}"], np.float32))


def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def calibrate_amax(sd, feats, lens):
    """Calibration pass of the fp32 transcription (run_mode "calib").

    Returns amax[5]: running max |cat([x_t, h_{t-1}])| of each encoder layer's input quantizer
    over every frame and batch row, exactly what ``TensorQuantizer.calib_amax`` accumulates
    (quant_modules.py:110-115) from ``QuantLSTMLayer.forward`` (quant_lstm.py:166-171).
    feats: [T, N, >=240] fp32 (only the first 240 channels are used); lens: [N].
    """
    H = R.trans_hidden_size
    x = np.asarray(feats, np.float32)[:, :, : R.trans_input_size]
    amax = np.zeros(5, np.float32)
    for layer in range(5):
        wih, whh, bih, bhh = enc_layer_params(sd, layer)
        if layer == 2:  # StackTime f32 (modeling_rnnt.py:314-324)
            T, N, C = x.shape
            x = x.copy()
            for n in range(N):
                x[int(lens[n]):, n, :] = 0
            if T % 2:
                x = np.concatenate([x, np.zeros((1, N, C), np.float32)], 0)
            x = x.reshape(x.shape[0] // 2, 2, N, C).transpose(0, 2, 1, 3).reshape(x.shape[0] // 2, N, 2 * C)
        T, N, _ = x.shape
        h = np.zeros((N, H), np.float32)
        c = np.zeros((N, H), np.float32)
        ys = np.empty((T, N, H), np.float32)
        m = np.float32(0)
        for t in range(T):
            m = max(m, np.abs(x[t]).max(initial=0), np.abs(h).max(initial=0))
            g = x[t] @ wih.T + bih + h @ whh.T + bhh
            i, f, gg, o = np.split(g, 4, axis=1)
            c = _sigmoid(f) * c + _sigmoid(i) * np.tanh(gg)
            h = (_sigmoid(o) * np.tanh(c)).astype(np.float32)
            ys[t] = h
        amax[layer] = m
        x = ys
    return amax


def q8(v):
    """round_and_clamp (quant_modules.py:8-9): clamp(round_half_even(v), -128, 127)."""
    return np.clip(np.rint(v), -128, 127).astype(np.int8)


def f32_to_bf16_bits(x):
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def bf16_round(x):
    """f32 -> bf16 (round-half-even) -> f32, as torch's .to(torch.bfloat16)."""
    return (f32_to_bf16_bits(x).astype(np.uint32) << 16).view(np.float32)


@dataclass
class PreparedModel:
    """Quantised / bf16 model in the reference's natural layouts (row = gate*H + unit)."""
    enc_w: List[np.ndarray] = field(default_factory=list)   # int8 [4096, I_l + 1024]
    enc_bq: List[np.ndarray] = field(default_factory=list)  # f32 [4096]
    enc_rb: np.ndarray = None      # f32 [5]
    enc_in_s: np.ndarray = None    # f32 [5]
    enc_out_s: np.ndarray = None   # f32 [5] (last = inf, unused: skip_quant_y)
    amax: np.ndarray = None        # f32 [5] calibrated input amax
    bf16: bool = True
    embed: np.ndarray = None       # [28, 320]
    pred_wih: List[np.ndarray] = field(default_factory=list)  # [1280, 320]
    pred_whh: List[np.ndarray] = field(default_factory=list)
    pred_bih: List[np.ndarray] = field(default_factory=list)  # [1280]
    pred_bhh: List[np.ndarray] = field(default_factory=list)
    w1t: np.ndarray = None         # [512, 1024]
    w1p: np.ndarray = None         # [512, 320]
    bt: np.ndarray = None          # [512]
    bp: np.ndarray = None          # [512]
    w2: np.ndarray = None          # [29, 512]
    b2: np.ndarray = None          # [29]


def quantize_encoder_layer(wih, whh, bih, bhh, in_scale, pad_to=None):
    """iLSTMLayer._quant_parameters (quant_lstm.py:193-215), fp32 tensor arithmetic:
    s_w = 127/max|[W_ih, W_hh]|; W_q = round_and_clamp(W*s_w); b_q = (b_hh+b_ih)*(s_in*s_w);
    rb = 1/(s_in*s_w) (a python-float division, then stored into an f32 tensor)."""
    amax_w = np.float32(np.max(np.abs(np.concatenate([wih, whh], 1))))
    s_w = np.float32(np.float32(127.0) / amax_w)
    w_ih_q = q8(wih * s_w)
    w_hh_q = q8(whh * s_w)
    if pad_to is not None and w_ih_q.shape[1] < pad_to:
        w_ih_q = np.pad(w_ih_q, ((0, 0), (0, pad_to - w_ih_q.shape[1])))
    b_scale = np.float32(np.float32(in_scale) * s_w)
    bq = ((bhh + bih) * b_scale).astype(np.float32)
    rb = np.float32(1.0 / float(b_scale))
    return np.ascontiguousarray(np.concatenate([w_ih_q, w_hh_q], 1)), bq, rb


def prepare_model(ckpt, amax, bf16=True):
    """Checkpoint (original keys) + calibrated amax[5] -> PreparedModel (run_mode "quant")."""
    sd = migrate_state_dict(ckpt)
    pm = PreparedModel(bf16=bf16)
    amax = np.asarray(amax, np.float32)
    pm.amax = amax
    in_s = (np.float32(127.0) / amax).astype(np.float32)
    out_s = np.empty(5, np.float32)
    out_s[:4] = in_s[1:]
    with np.errstate(divide="ignore"):
        out_s[4] = np.float32(127.0) / np.float32(0.0)  # last post layer: its own, never-calibrated quantizer
    pm.enc_in_s, pm.enc_out_s = in_s, out_s
    rbs = []
    for layer in range(5):
        wih, whh, bih, bhh = enc_layer_params(sd, layer)
        w, bq, rb = quantize_encoder_layer(wih, whh, bih, bhh, in_s[layer], pad_to=ENC_INPUT_SIZES[layer])
        pm.enc_w.append(w)
        pm.enc_bq.append(bq)
        rbs.append(rb)
    pm.enc_rb = np.array(rbs, np.float32)
    cvt = bf16_round if bf16 else (lambda a: np.asarray(a, np.float32))
    pm.embed = cvt(np.asarray(sd["prediction.embed.weight"], np.float32))
    for l in range(R.pred_num_layers):
        p = "prediction.pred_rnn."
        pm.pred_wih.append(cvt(np.asarray(sd[p + f"weight_ih_l{l}"], np.float32)))
        pm.pred_whh.append(cvt(np.asarray(sd[p + f"weight_hh_l{l}"], np.float32)))
        pm.pred_bih.append(np.asarray(sd[p + f"bias_ih_l{l}"], np.float32))
        pm.pred_bhh.append(np.asarray(sd[p + f"bias_hh_l{l}"], np.float32))
    pm.w1t = cvt(np.asarray(sd["joint.linear1_trans.weight"], np.float32))
    pm.w1p = cvt(np.asarray(sd["joint.linear1_pred.weight"], np.float32))
    pm.bt = np.asarray(sd["joint.linear1_trans.bias"], np.float32)
    pm.bp = np.asarray(sd["joint.linear1_pred.bias"], np.float32)
    pm.w2 = cvt(np.asarray(sd["joint.linear2.weight"], np.float32))
    pm.b2 = np.asarray(sd["joint.linear2.bias"], np.float32)
    return pm


def build_model(seed=None, amax=None, calib_n=2, calib_T=120, bf16=True, recipe=None):
    """Synthetic checkpoint -> calibration on seeded synthetic features -> PreparedModel."""
    from .synthetic import DEFAULT_SEED, make_checkpoint, make_features
    seed = DEFAULT_SEED if seed is None else seed
    ckpt = make_checkpoint(seed, recipe)
    if amax is None:
        lens = np.full(calib_n, calib_T, np.int32)
        feats = make_features(calib_T, calib_n, seed=seed ^ 0xCA1B, lens=lens)
        amax = calibrate_amax(migrate_state_dict(ckpt), feats, lens)
    return prepare_model(ckpt, amax, bf16=bf16), ckpt


# ---- packed model file (the export that replaces the reference's calibrated state dict +
# TorchScript jit files, models/main.py:21-58 / utils.py:97-110): the PreparedModel arrays in an
# .npz (no pickles; load with allow_pickle=False), plus a JSON header.
PACKED_FORMAT = "rnnt-mi355x-prepared/1"
_LISTS = ("enc_w", "enc_bq", "pred_wih", "pred_whh", "pred_bih", "pred_bhh")
_ARRAYS = ("enc_rb", "enc_in_s", "enc_out_s", "amax", "embed", "w1t", "w1p", "bt", "bp", "w2", "b2")


def prepared_digest(pm):
    import hashlib
    h = hashlib.sha256()
    for k in _LISTS:
        for a in getattr(pm, k):
            h.update(np.ascontiguousarray(a).tobytes())
    for k in _ARRAYS:
        h.update(np.ascontiguousarray(getattr(pm, k)).tobytes())
    return h.hexdigest()


def save_prepared(pm, path, extra=None):
    import json
    meta = {"format": PACKED_FORMAT, "bf16": bool(pm.bf16), "sha256": prepared_digest(pm)}
    meta.update(extra or {})
    arrs = {"meta": np.frombuffer(json.dumps(meta).encode(), np.uint8)}
    for k in _LISTS:
        for i, a in enumerate(getattr(pm, k)):
            arrs[f"{k}_{i}"] = np.ascontiguousarray(a)
    for k in _ARRAYS:
        arrs[k] = np.ascontiguousarray(getattr(pm, k))
    with open(path, "wb") as f:
        np.savez(f, **arrs)
    return meta


def load_prepared(path):
    """-> (PreparedModel, header); verifies the format tag and the content digest."""
    import json
    with np.load(path, allow_pickle=False) as z:
        meta = json.loads(bytes(z["meta"]).decode())
        if meta.get("format") != PACKED_FORMAT:
            raise ValueError(f"{path}: not a {PACKED_FORMAT} file")
        pm = PreparedModel(bf16=bool(meta["bf16"]))
        for k in _LISTS:
            n = sum(1 for key in z.files if key.rsplit("_", 1)[0] == k and key.rsplit("_", 1)[1].isdigit())
            setattr(pm, k, [z[f"{k}_{i}"] for i in range(n)])
        for k in _ARRAYS:
            setattr(pm, k, z[k])
    if prepared_digest(pm) != meta["sha256"]:
        raise ValueError(f"{path}: content digest mismatch")
    return pm, meta


def load_checkpoint(path):
    """A state dict of tensors (original or migrated keys) from .pt (torch.load weights_only=True),
    .safetensors or .npz (allow_pickle=False) -> {key: float32 ndarray}."""
    if path.endswith(".safetensors"):
        from safetensors.numpy import load_file
        sd = load_file(path)
    elif path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            sd = {k: z[k] for k in z.files}
    else:
        import torch
        obj = torch.load(path, map_location="cpu", weights_only=True)
        if isinstance(obj, dict) and "state_dict" in obj and isinstance(obj["state_dict"], dict):
            obj = obj["state_dict"]
        sd = {k: v.detach().float().numpy() for k, v in obj.items() if hasattr(v, "detach")}
    return {k: np.asarray(v, np.float32) for k, v in sd.items()}


# ---- engine model file (rnnt_engine_create_from_file, include/rnnt_mi355x.h): the arrays of
# rnnt_model_desc in a flat little-endian container readable from C++ without numpy or zip.
ENGINE_FILE_MAGIC = b"RNNTMI01"
_DT = {0: np.int8, 1: np.float32, 2: np.uint16}


def engine_file_arrays(pm):
    """name -> (dtype code, array) in the order save_engine_file writes them (bf16 as bit patterns)."""
    if not pm.bf16:
        raise ValueError("the engine file holds the int8 + bf16 model (prepare_model(..., bf16=True))")
    out = {}
    for l in range(5):
        out[f"enc_w.{l}"] = (0, np.ascontiguousarray(pm.enc_w[l], np.int8))
        out[f"enc_bq.{l}"] = (1, np.ascontiguousarray(pm.enc_bq[l], np.float32))
    out["enc_rb"] = (1, np.asarray(pm.enc_rb, np.float32))
    out["enc_in_s"] = (1, np.asarray(pm.enc_in_s, np.float32))
    out["enc_out_s"] = (1, np.asarray(pm.enc_out_s, np.float32))
    out["embed"] = (2, f32_to_bf16_bits(pm.embed))
    for l in range(R.pred_num_layers):
        out[f"pred_wih.{l}"] = (2, f32_to_bf16_bits(pm.pred_wih[l]))
        out[f"pred_whh.{l}"] = (2, f32_to_bf16_bits(pm.pred_whh[l]))
        out[f"pred_bih.{l}"] = (1, np.asarray(pm.pred_bih[l], np.float32))
        out[f"pred_bhh.{l}"] = (1, np.asarray(pm.pred_bhh[l], np.float32))
    out["w1t"] = (2, f32_to_bf16_bits(pm.w1t))
    out["w1p"] = (2, f32_to_bf16_bits(pm.w1p))
    out["bt"] = (1, np.asarray(pm.bt, np.float32))
    out["bp"] = (1, np.asarray(pm.bp, np.float32))
    out["w2"] = (2, f32_to_bf16_bits(pm.w2))
    out["b2"] = (1, np.asarray(pm.b2, np.float32))
    return out


def save_engine_file(pm, path):
    """Write the engine model file: magic, u32 version 1, u32 count, count x {char name[48];
    u32 dtype; u32 ndim; u64 shape[4]; u64 offset; u64 nbytes}, then 64-byte aligned data."""
    return write_pack_file(path, engine_file_arrays(pm))


def write_pack_file(path, arrs):
    """The RNNTMI01 container of save_engine_file: {name: (dtype code, array)}."""
    import struct
    head = 16 + len(arrs) * 104
    off = (head + 63) // 64 * 64
    ents, blobs = [], []
    for name, (code, a) in arrs.items():
        a = np.ascontiguousarray(a)
        shape = list(a.shape) + [0] * (4 - a.ndim)
        ents.append(struct.pack("<48sII4QQQ", name.encode(), code, a.ndim, *shape, off, a.nbytes))
        blobs.append((off, a.tobytes()))
        off = (off + a.nbytes + 63) // 64 * 64
    with open(path, "wb") as f:
        f.write(ENGINE_FILE_MAGIC + struct.pack("<II", 1, len(arrs)) + b"".join(ents))
        for o, b in blobs:
            f.seek(o)
            f.write(b)
    return path


def read_engine_file(path):
    """-> {name: array} (the C++ reader's view; for tests and tools)."""
    import struct
    raw = open(path, "rb").read()
    if raw[:8] != ENGINE_FILE_MAGIC:
        raise ValueError(f"{path}: not an engine model file")
    version, count = struct.unpack_from("<II", raw, 8)
    if version != 1:
        raise ValueError(f"{path}: version {version}")
    out = {}
    for i in range(count):
        name, code, ndim, s0, s1, s2, s3, off, nb = struct.unpack_from("<48sII4QQQ", raw, 16 + 104 * i)
        shape = (s0, s1, s2, s3)[:ndim]
        out[name.rstrip(b"\0").decode()] = np.frombuffer(raw, _DT[code], count=nb // np.dtype(_DT[code]).itemsize,
                                                        offset=off).reshape(shape)
    return out
