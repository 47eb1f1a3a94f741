"""ctypes binding of librnnt_mi355x.so (C ABI: include/rnnt_mi355x.h).

The HIP engine is the only compute path: there is no CPU or eager-PyTorch fallback, and a
missing or unloadable library raises instead of silently degrading.
"""
import ctypes as C
import os
import re
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# RNNT_MI355X_LIB: development override (kernel variants built by tools/ into build_dev/)
LIB_PATH = os.environ.get("RNNT_MI355X_LIB") or os.path.join(_HERE, "librnnt_mi355x.so")
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
HEADER = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "rnnt_mi355x.h")

RNNT_OK, RNNT_EINVAL, RNNT_ENOMEM, RNNT_EDEVICE = 0, -22, -12, -5


class RnntModelDesc(C.Structure):
    _fields_ = [
        ("enc_w", C.c_void_p * 5), ("enc_bq", C.c_void_p * 5),
        ("enc_rb", C.c_float * 5), ("enc_in_s", C.c_float * 5), ("enc_out_s", C.c_float * 5),
        ("embed", C.c_void_p),
        ("pred_w_ih", C.c_void_p * 2), ("pred_w_hh", C.c_void_p * 2),
        ("pred_b_ih", C.c_void_p * 2), ("pred_b_hh", C.c_void_p * 2),
        ("joint_w1t", C.c_void_p), ("joint_w1p", C.c_void_p),
        ("joint_bt", C.c_void_p), ("joint_bp", C.c_void_p),
        ("joint_w2", C.c_void_p), ("joint_b2", C.c_void_p),
    ]


class RnntOpts(C.Structure):
    _fields_ = [("max_batch", C.c_int), ("max_frames", C.c_int), ("max_res", C.c_int)]


class RnntStats(C.Structure):
    _fields_ = [("encode_ms", C.c_double), ("joint_trans_ms", C.c_double), ("greedy_ms", C.c_double),
                ("step_launches", C.c_int64), ("decode_steps", C.c_int64), ("encode_calls", C.c_int64), ("decode_calls", C.c_int64)]


class RnntF32DecoderDesc(C.Structure):
    _fields_ = [("embed", C.c_void_p), ("pred_w_ih", C.c_void_p * 2), ("pred_w_hh", C.c_void_p * 2),
                ("pred_b_ih", C.c_void_p * 2), ("pred_b_hh", C.c_void_p * 2), ("joint_w1t", C.c_void_p),
                ("joint_w1p", C.c_void_p), ("joint_bt", C.c_void_p), ("joint_bp", C.c_void_p),
                ("joint_w2", C.c_void_p), ("joint_b2", C.c_void_p)]


class RnntFeaturizerConfig(C.Structure):
    _fields_ = [("sample_rate", C.c_int), ("n_fft", C.c_int), ("win_length", C.c_int), ("hop_length", C.c_int),
                ("nfilt", C.c_int), ("frame_splicing", C.c_int), ("pad_out_feat", C.c_int),
                ("preemph", C.c_float), ("dither", C.c_float), ("log_guard", C.c_float), ("norm_eps", C.c_float)]


_SIGS = {
    "rnnt_featurizer_create": (C.c_int, [C.POINTER(RnntFeaturizerConfig), C.c_void_p, C.c_void_p, C.c_int,
                                         C.POINTER(C.c_void_p)]),
    "rnnt_featurizer_destroy": (None, [C.c_void_p]),
    "rnnt_featurizer_create_from_file": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]),
    "rnnt_featurizer_frames": (C.c_int64, [C.c_int64]),
    "rnnt_featurizer_own_cu_lds": (C.c_size_t, [C.c_void_p]),
    "rnnt_featurizer_run": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int,
                                      C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "rnnt_featurizer_run_rows": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                           C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "rnnt_engine_set_profiling": (C.c_int, [C.c_void_p, C.c_int]),
    "rnnt_engine_set_tile": (C.c_int, [C.c_void_p, C.c_char_p]),
    "rnnt_engine_set_decode_persist": (C.c_int, [C.c_void_p, C.c_int]),
    "rnnt_engine_get_stats": (C.c_int, [C.c_void_p, C.POINTER(RnntStats), C.c_int]),
    "rnnt_abi_version": (C.c_int, []),
    "rnnt_install_crash_report": (C.c_int, []),
    "rnnt_stream_create": (C.c_int, [C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    "rnnt_stream_destroy": (C.c_int, [C.c_void_p]),
    "rnnt_last_error": (C.c_char_p, []),
    "rnnt_engine_create": (C.c_int, [C.POINTER(RnntModelDesc), C.c_int, C.POINTER(RnntOpts), C.POINTER(C.c_void_p)]),
    "rnnt_engine_destroy": (None, [C.c_void_p]),
    "rnnt_engine_encode": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                     C.c_void_p, C.c_void_p]),
    "rnnt_engine_encode_gather": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                            C.c_int, C.c_void_p, C.c_void_p]),
    "rnnt_engine_decode": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "rnnt_engine_encode_stream": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "rnnt_engine_decode_stream": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "rnnt_engine_encode_stream_pl": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                               C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "rnnt_engine_decode_stream_pl": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                               C.c_void_p]),
    "rnnt_op_lstm_bf16": (C.c_int, [C.c_void_p] * 6 + [C.c_int, C.c_void_p]),
    "rnnt_op_joint_hidden": (C.c_int, [C.c_void_p] * 4 + [C.c_int, C.c_void_p]),
    "rnnt_op_joint_logits": (C.c_int, [C.c_void_p] * 3 + [C.c_int, C.c_void_p]),
    "rnnt_op_greedy_update": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "rnnt_engine_create_from_file": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(RnntOpts), C.POINTER(C.c_void_p)]),
    "rnnt_engine_load_encoder_layers": (C.c_int, [C.c_void_p, C.c_int, C.c_int] + [C.c_void_p] * 5),
    "rnnt_engine_load_prediction": (C.c_int, [C.c_void_p] * 6),
    "rnnt_engine_load_joint": (C.c_int, [C.c_void_p] * 5),
    "rnnt_engine_load_joint_out": (C.c_int, [C.c_void_p] * 3),
    "rnnt_engine_load_f32_encoder": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                               C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "rnnt_engine_encode_f32": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                         C.c_void_p]),
    "rnnt_engine_load_f32_decoder": (C.c_int, [C.c_void_p, C.POINTER(RnntF32DecoderDesc)]),
    "rnnt_engine_decode_f32": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "rnnt_engine_infer": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                    C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "rnnt_op_lstm_int8": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_void_p]),
    "rnnt_op_stack_time": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                     C.c_void_p]),
    "rnnt_engine_load_f32_prediction": (C.c_int, [C.c_void_p] + [C.POINTER(C.c_void_p)] * 4),
    "rnnt_op_lstm_f32": (C.c_int, [C.c_void_p] * 6 + [C.c_int, C.c_void_p]),
    "rnnt_op_preemphasis": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_int, C.c_float, C.c_int,
                                      C.c_void_p, C.c_void_p]),
    "rnnt_op_power_spectrum": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
    "rnnt_op_frame_splicing": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                         C.c_void_p]),
    "rnnt_op_layernorm_pad": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                        C.c_int, C.c_int, C.c_int, C.c_float, C.c_int, C.c_void_p, C.c_void_p,
                                        C.c_void_p]),
}

_lib = None


def build():
    """Compile the HIP engine in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-C", CSRC], check=True)


def header_functions(path=HEADER):
    """Function names declared in include/rnnt_mi355x.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rnnt_[a-z0-9_]+)\s*\(", text)))


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"HIP engine library missing: {LIB_PATH} (build it with `make -C {CSRC}`); "
                           "rnnt_amd has no CPU fallback")
    # torch ships its own libamdhip64.so.7; importing it first makes our NEEDED entry resolve to
    # the already-loaded runtime (same SONAME), so device pointers and streams are shared.  Loading
    # ours first would bring up a second HIP runtime that then sees no device.
    import torch  # noqa: F401
    _lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        f = getattr(_lib, name)
        f.restype = res
        f.argtypes = args
    return _lib


class EngineError(RuntimeError):
    pass


def check(rc, what):
    if rc != RNNT_OK:
        msg = lib().rnnt_last_error()
        raise EngineError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
