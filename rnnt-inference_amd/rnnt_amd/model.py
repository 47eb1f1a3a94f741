"""RNNT model container (mirror of reference ``models/modeling_rnnt.py:15-81`` ``RNNT``).

``RNNT(model_path, run_mode, enable_bf16)`` loads a checkpoint (original or migrated keys;
``weights.load_checkpoint`` formats, or a state dict of arrays) and holds what the engine needs
for the requested mode, the way the reference's ``_load_model`` prepares its modules:

* ``run_mode="quant"``: the int8 encoder + bf16 prediction/joint model (``iLSTMLayer.
  _quant_parameters`` + ``prepack_weights``, quant_lstm.py:193-215, modeling_rnnt.py:161-257),
  quantised with the calibrated input amax (the reference's ``rnnt_calib.pt`` quantizer buffers);
  a packed export (``weights.save_prepared``) may be given instead of a checkpoint.
* ``run_mode="f32"`` (or None): the fp32 transcription layers and the fp32 prediction/joint;
  with ``enable_bf16`` the prediction/joint run in bf16 on the fp32 encoder's output
  (decoder.py:121-122).  The engine is created from a bf16 model either way (its int8 encoder
  half is then unused and quantised with unit amax).
"""
import numpy as np

from . import weights


class RNNT:
    def __init__(self, model_path=None, run_mode=None, enable_bf16=False, load_jit=False, amax=None):
        if run_mode not in ("quant", "f32", None):
            raise ValueError(f"run_mode {run_mode!r}: the engine runs 'quant' or 'f32'")
        self.run_mode = run_mode or "f32"
        self.enable_bf16 = bool(enable_bf16)
        if self.run_mode == "quant" and not self.enable_bf16:
            raise ValueError("run_mode='quant' runs with enable_bf16 (int8 encoder, bf16 prediction/joint), as the "
                             "reference's quantised graph does")
        if isinstance(model_path, str) and model_path.endswith(".npz") and _is_packed(model_path):
            pm, meta = weights.load_prepared(model_path)
            if self.run_mode != "quant":
                raise ValueError(f"{model_path}: a packed int8 model serves run_mode='quant' only")
            self.pm, self.sd, self.pm32 = pm, None, None
            return
        ckpt = weights.load_checkpoint(model_path) if isinstance(model_path, str) else model_path
        if ckpt is None:
            raise ValueError("RNNT needs a checkpoint (path or state dict)")
        self.sd = weights.migrate_state_dict(ckpt)
        if self.run_mode == "quant":
            if amax is None:
                raise ValueError("run_mode='quant' needs the calibrated input amax of the 5 encoder layers")
            self.pm = weights.prepare_model(ckpt, amax, bf16=True)
            self.pm32 = None
        else:
            self.pm = weights.prepare_model(ckpt, np.ones(5, np.float32) if amax is None else amax, bf16=True)
            self.pm32 = weights.prepare_model(ckpt, np.ones(5, np.float32) if amax is None else amax, bf16=False)

    def f32_encoder_layers(self):
        """5 x (W_ih, W_hh, b_ih, b_hh) fp32, natural layout (rnnt_engine_load_f32_encoder)."""
        return [weights.enc_layer_params(self.sd, l) for l in range(5)]


def _is_packed(path):
    try:
        with np.load(path, allow_pickle=False) as z:
            return "meta" in z.files
    except Exception:
        return False
