"""GreedyDecoder over the HIP engine (mirror of reference models/decoder.py:11-212).

``GreedyDecoder(model, run_mode, enable_bf16, split_len, batch_size)`` and
``forward(x, x_lens) -> (res, res_len)`` keep the reference's interface and result contract:
res [N, max_symbols_per_step * max(x_lens)] filled with SOS (-1) (int32 for run_mode "quant",
int64 otherwise, decoder.py:30), res_len = res_idx + 1.

* run_mode "quant" (greedy_decode_quant, decoder.py:171-212): int8 transcription + bf16
  prediction / joint + greedy loop, all on the engine.
* run_mode "f32" (greedy_decode_f32, decoder.py:102-169): fp32 transcription, then the fp32
  decoder, or with enable_bf16 the bf16 prediction / joint on bf16(f) (decoder.py:121-122).

``model`` is an ``rnnt_amd.model.RNNT`` (or, for "quant", a ``weights.PreparedModel``).
``split_len`` is accepted for compatibility; the engine's encoder walks the whole time axis in
one pass, which is numerically identical to the chunked loop (decoder.py:80-91; pinned by
tests/test_oracle_golden.py::test_split_len_chunking_is_invariant).
"""
from .config import RNNTParam as R
from .engine import Engine, pad_batch
from .weights import PreparedModel
from . import ops


class GreedyDecoder:
    def __init__(self, model, run_mode="quant", enable_bf16=True, split_len=-1, batch_size=1, device=0,
                 max_frames=R.MAX_FEA_LEN):
        self.run_mode = run_mode or "f32"
        self.enable_bf16 = bool(enable_bf16)
        if self.run_mode not in ("quant", "f32"):
            raise RuntimeError(f"run_mode {run_mode!r} is not served by the engine (quant | f32)")
        if self.run_mode == "quant" and not self.enable_bf16:
            raise RuntimeError("run_mode='quant' runs with enable_bf16 (int8 encoder, bf16 prediction/joint)")
        pm = model if isinstance(model, PreparedModel) else model.pm
        self.model = model
        self.split_len = split_len
        self.batch_size = batch_size
        self.engine = Engine(pm, device=device, max_batch=max(batch_size, 1), max_frames=max_frames)
        if self.run_mode == "quant":
            ops.bind(self.engine, pm)
        else:
            if isinstance(model, PreparedModel) or getattr(model, "sd", None) is None:
                raise RuntimeError("run_mode='f32' needs an rnnt_amd.model.RNNT built from a checkpoint")
            self.engine.load_f32_encoder(model.f32_encoder_layers())
            if not self.enable_bf16:
                self.engine.load_f32_decoder(model.pm32)

    def __call__(self, x, x_lens):
        return self.forward(x, x_lens)

    def forward(self, x, x_lens):
        """x: fp32 [T, N, 240|256] (cuda), x_lens: [N] -> (res [N, 30*max_len], res_len [N])."""
        import numpy as np
        import torch
        N = x_lens.shape[0]
        width = R.max_symbols_per_step * int(x_lens.max().item())
        if self.run_mode == "quant":
            ops.transcription(x, x_lens, f_out=False)
            res, rl = ops.greedy_decode(N)
        else:
            T = x.shape[0]
            n_pad = pad_batch(N)
            xin = torch.zeros((T, n_pad, R.PADDED_INPUT_SIZE), dtype=torch.float32, device=x.device)
            xin[:, :N, : x.shape[2]] = x
            lens = torch.zeros(n_pad, dtype=torch.int32, device=x.device)
            lens[:N] = torch.from_numpy(np.asarray(x_lens.cpu(), np.int32)).to(x.device)
            res = torch.empty((N, self.engine.max_res), dtype=torch.int32, device=x.device)
            rl = torch.empty(N, dtype=torch.int32, device=x.device)
            self.engine.encode_f32(xin, lens, N)
            if self.enable_bf16:
                self.engine.decode(res, rl)
            else:
                self.engine.decode_f32(res, rl)
        dt = torch.int32 if self.run_mode == "quant" else torch.int64
        out = torch.full((N, width), R.SOS, dtype=dt, device=res.device)
        w = min(width, res.shape[1])
        out[:, :w] = res[:, :w].to(dt)
        return out, rl.to(dt)

    def close(self):
        self.engine.close()
