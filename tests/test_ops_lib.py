"""The torch.ops.intel_mlperf operator library and the engine model file, host side (no GPU).

* the library loads through torch.ops.load_library and registers every op the reference graph
  binds, with the schemas its call sites imply (quant_lstm.py:92-101, modeling_rnnt.py:174,
  202, 253, 269-283, 326-328, 351-365);
* rnnt_amd.ops.reference_weights packs weights exactly as the reference's transpose_tile_weight /
  transpose_tile_weight_bf16 do (sha256 of the reference's own packed tiles, tests/golden/tiles.npz);
* TorchScript resolves the ops (torch.jit.script of graph fragments written like the reference's);
* the engine model file round-trips (the C loader's format, rnnt_engine_create_from_file).
"""
import hashlib
import os

import numpy as np
import pytest
import torch

from rnnt_amd import ops, weights

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCHEMAS = {
    "lstm_amx_int8": "(Tensor x, Tensor[] hx, Tensor[] cx, Tensor[][] weights, Tensor rb_scale, Tensor in_scale, "
                     "Tensor out_scale, bool skip_quant_y) -> (Tensor, Tensor[], Tensor[])",
    "stack_time": "(Tensor x, Tensor x_lens, int factor) -> Tensor",
    "lstm_amx_bf16": "(Tensor x, Tensor[] hx, Tensor[] cx, Tensor[][] weights) -> (Tensor, Tensor[], Tensor[])",
    "amx_linear_bf16_accum_relu": "(Tensor f, Tensor w1_trans, Tensor g, Tensor w1_pred, Tensor bias) -> Tensor",
    "amx_linear_i16o32": "(Tensor y, Tensor w2, Tensor b2) -> Tensor",
    "prepack_lstm_weights": "(Tensor w_ih, Tensor w_hh) -> (Tensor, Tensor)",
    "prepack_linear_weight": "(Tensor w) -> Tensor",
    "lstm": "(Tensor x, Tensor[] hx, Tensor[] cx, Tensor[][] weights) -> (Tensor, Tensor[], Tensor[])",
    "preemphasis": "(Tensor x, Tensor x_lens, float coeff=0.96999999999999997, int pad_size=0) -> Tensor",
    "power_spectrum": "(Tensor x, Tensor x_lens) -> Tensor",
    "frame_splicing": "(Tensor x, Tensor x_lens, int factor) -> Tensor",
    "i_layernorm_pad": "(Tensor x, Tensor weight, Tensor bias, Tensor x_lens, float eps, int unbiased, "
                       "Tensor output_shape) -> (Tensor, Tensor)",
}

# every name the reference's operator module resolves at import (models/_C.py:15-51), in its order
REFERENCE_C_NAMES = [
    "linear", "linear_gelu", "amx_linear", "amx_linear_i8o32", "amx_linear_bf16_accum_relu", "amx_linear_i16o32",
    "baddbmm_out_", "prepack_linear_weight", "matmul_out_", "reorder_test", "i_softmax", "i_softmax_u", "i_gelu",
    "i_identity", "i_identity_cin", "i_identity_", "i_layernorm", "i_layernorm_pad", "i_residual_layernorm",
    "i_residual_layernorm_", "i_residual_layernorm_cin_", "amx_mha", "amx_mha_concat", "preemphasis",
    "frame_splicing", "stack_time", "prepack_lstm_weights", "tanh", "sigmoid", "tanh_f16", "lstm_postop",
    "lstm_layer_amx_int8", "lstm_amx_int8", "lstm_layer_amx_bf16", "lstm_amx_bf16", "greedy_decode_update", "lstm"]


@pytest.fixture(scope="module")
def lib():
    return ops.load_library()


def test_library_registers_reference_schemas(lib):
    for name, sig in SCHEMAS.items():
        schema = str(getattr(lib, name).default._schema)
        assert schema == f"intel_mlperf::{name}{sig}", schema
    s = str(lib.greedy_decode_update.default._schema)
    assert s.endswith("-> bool") and s.count("Tensor") == 13, s  # 13 operands, finish kept internal


def test_reference_operator_module_binds(lib):
    """`import _C` (models/_C.py:15-51) resolves 37 names; all bind here, plus power_spectrum
    (datasets/parts/features.py:215).  The names the RNN-T graph never calls fail loudly, naming
    the op."""
    assert len(REFERENCE_C_NAMES) == 37
    for name in REFERENCE_C_NAMES + ["power_spectrum"]:
        assert hasattr(lib, name), name
        assert getattr(lib, name).default._schema.name == f"intel_mlperf::{name}"
    for name in ("amx_mha", "i_softmax", "tanh_f16"):
        with pytest.raises(RuntimeError, match=f"intel_mlperf::{name} is not served"):
            getattr(lib, name)(torch.zeros(2))
    with pytest.raises(RuntimeError, match="lstm_postop is not served"):
        z = torch.zeros(2, 4)
        lib.lstm_postop(z, z, z, z, z, 1.0, 1.0, False)


def test_reference_tile_layouts(pm_golden):
    tiles = np.load(os.path.join(REPO, "tests", "golden", "tiles.npz"))
    w = ops.reference_weights(pm_golden)

    def sha(t):
        return hashlib.sha256(t.contiguous().view(torch.uint8).numpy().tobytes()).hexdigest()

    for l in range(5):
        lw = (w["pre"] + w["post"])[l]
        assert sha(lw[0]) == bytes(tiles[f"enc{l}_ih"]).decode(), f"layer {l} W_ih tiles"
        assert sha(lw[1]) == bytes(tiles[f"enc{l}_hh"]).decode(), f"layer {l} W_hh tiles"
    for l in range(2):
        assert sha(w["pred"][l][0]) == bytes(tiles[f"pred{l}_ih"]).decode()
        assert sha(w["pred"][l][1]) == bytes(tiles[f"pred{l}_hh"]).decode()
    for k, name in (("w1_trans", "w1t"), ("w1_pred", "w1p"), ("w2", "w2")):
        assert sha(w[k]) == bytes(tiles[name]).decode(), name


def test_torchscript_binds_the_ops(lib):
    """Graph fragments written like the reference's modules script against the library (the
    C++ SUT's torch::jit::load path resolves the same schemas)."""
    from typing import List

    class Update(torch.nn.Module):  # GreedyDecoderUpdate.forward, modeling_rnnt.py:331-365
        def forward(self, symbols: torch.Tensor, symbols_added: torch.Tensor, res: torch.Tensor, res_idx: torch.Tensor,
                    f: torch.Tensor, f_lens: torch.Tensor, time_idx: torch.Tensor, fi: torch.Tensor,
                    pre_g: torch.Tensor, pre_hg: List[torch.Tensor], pre_cg: List[torch.Tensor],
                    hg: List[torch.Tensor], cg: List[torch.Tensor]) -> bool:
            return torch.ops.intel_mlperf.greedy_decode_update(symbols, symbols_added, res, res_idx, f, f_lens,
                                                               time_idx, fi, pre_g, pre_hg, pre_cg, hg, cg)

    class Stack(torch.nn.Module):  # iLSTM.forward + StackTime.forward_quant
        def forward(self, x: torch.Tensor, x_lens: torch.Tensor, hx: List[torch.Tensor], cx: List[torch.Tensor],
                    weights: List[List[torch.Tensor]], rb: torch.Tensor, ins: torch.Tensor, outs: torch.Tensor):
            y, h, c = torch.ops.intel_mlperf.lstm_amx_int8(x, hx, cx, weights, rb, ins, outs, False)
            return torch.ops.intel_mlperf.stack_time(y, x_lens, 2), h, c

    class Joint(torch.nn.Module):  # Joint.forward (enable_bf16), modeling_rnnt.py:259-283
        def forward(self, f: torch.Tensor, g: torch.Tensor, w1t: torch.Tensor, w1p: torch.Tensor, b: torch.Tensor,
                    w2: torch.Tensor, b2: torch.Tensor) -> torch.Tensor:
            y = torch.ops.intel_mlperf.amx_linear_bf16_accum_relu(f, w1t, g, w1p, b)
            return torch.ops.intel_mlperf.amx_linear_i16o32(y, w2, b2)

    class Prediction32(torch.nn.Module):  # Prediction.forward, run_mode f32 (modeling_rnnt.py:183-205)
        def forward(self, g: torch.Tensor, hg: List[torch.Tensor], cg: List[torch.Tensor],
                    weights: List[List[torch.Tensor]]):
            return torch.ops.intel_mlperf.lstm(g, hg, cg, weights)

    class Processor(torch.nn.Module):  # FilterbankFeatures.forward's plugin ops (features.py:185-252)
        def forward(self, x: torch.Tensor, x_lens: torch.Tensor, window: torch.Tensor, fb: torch.Tensor,
                    fb_bias: torch.Tensor, w: torch.Tensor, b: torch.Tensor, shape: torch.Tensor):
            x = torch.ops.intel_mlperf.preemphasis(x, x_lens, coeff=0.97, pad_size=256)
            x = torch.stft(x, n_fft=512, hop_length=160, win_length=320, center=False, window=window,
                           return_complex=False).permute(0, 2, 1, 3)
            x_lens = torch.floor(x_lens / 160 + 1).to(dtype=torch.int32)
            x = torch.ops.intel_mlperf.power_spectrum(x, x_lens).permute(0, 2, 1)
            x = torch.log(torch.baddbmm(fb_bias, fb, x))
            x = torch.ops.intel_mlperf.frame_splicing(x, x_lens, 3)
            x_lens = torch.ceil(x_lens / 3).to(dtype=torch.int32)
            return torch.ops.intel_mlperf.i_layernorm_pad(x, w, b, x_lens, 1e-12, unbiased=1, output_shape=shape)

    for m in (Update(), Stack(), Joint(), Prediction32(), Processor()):
        g = torch.jit.script(m).graph
        assert "intel_mlperf::" in str(g)


def test_ops_refuse_host_activations(lib):
    """No CPU path: CPU activations are rejected (the compute lives on the GPU only)."""
    with pytest.raises((RuntimeError, NotImplementedError)):
        lib.stack_time(torch.zeros((4, 2, 16), dtype=torch.int8), torch.tensor([4, 2], dtype=torch.int32), 2)


def test_engine_file_roundtrip(pm_golden, tmp_path):
    p = weights.save_engine_file(pm_golden, str(tmp_path / "m.rnntmi"))
    d = weights.read_engine_file(p)
    assert open(p, "rb").read(8) == b"RNNTMI01"
    for l in range(5):
        np.testing.assert_array_equal(d[f"enc_w.{l}"], pm_golden.enc_w[l])
        np.testing.assert_array_equal(d[f"enc_bq.{l}"], pm_golden.enc_bq[l])
    np.testing.assert_array_equal(d["enc_in_s"], pm_golden.enc_in_s)
    np.testing.assert_array_equal(d["w2"], weights.f32_to_bf16_bits(pm_golden.w2))
    np.testing.assert_array_equal(d["b2"], pm_golden.b2)
