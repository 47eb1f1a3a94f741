"""GreedyDecoder over the HIP engine (mirror of reference models/decoder.py:11-94).

``GreedyDecoder(model, run_mode="quant", enable_bf16=True, split_len, batch_size)`` and
``forward(x, x_lens) -> (res, res_len)`` keep the reference's interface and result contract:
res int32 [N, max_symbols_per_step * max(x_lens)] filled with SOS (-1), res_len = res_idx + 1.
``split_len`` is accepted for compatibility; the engine's encoder walks the whole time axis
in one pass, which is numerically identical to the chunked loop (decoder.py:80-91; pinned by
tests/test_oracle_golden.py::test_split_len_chunking_is_invariant).
"""
from .config import RNNTParam as R
from .engine import Engine
from . import ops


class GreedyDecoder:
    def __init__(self, model, run_mode="quant", enable_bf16=True, split_len=-1, batch_size=1, device=0,
                 max_frames=R.MAX_FEA_LEN):
        if run_mode != "quant" or not enable_bf16:
            raise RuntimeError("the MI355X engine runs run_mode='quant' with enable_bf16 (int8 encoder, bf16 "
                               "prediction/joint); the fp32 path is the CPU restatement's (oracle/)")
        self.model = model
        self.split_len = split_len
        self.batch_size = batch_size
        self.engine = Engine(model, device=device, max_batch=max(batch_size, 1), max_frames=max_frames)
        ops.bind(self.engine, model)

    def __call__(self, x, x_lens):
        return self.forward(x, x_lens)

    def forward(self, x, x_lens):
        """x: fp32 [T, N, 240|256] (cuda), x_lens: [N] -> (res [N, 30*max_len], res_len [N])."""
        import torch
        N = x_lens.shape[0]
        ops.transcription(x, x_lens, f_out=False)
        width = R.max_symbols_per_step * int(x_lens.max().item())
        res, rl = ops.greedy_decode(N)
        out = torch.full((N, width), R.SOS, dtype=torch.int32, device=res.device)
        w = min(width, res.shape[1])
        out[:, :w] = res[:, :w]
        return out, rl

    def close(self):
        self.engine.close()
