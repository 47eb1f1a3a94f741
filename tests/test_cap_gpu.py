"""The 30-symbols-per-frame cap on the GPU.

The reference forces an advance when a frame has emitted max_symbols_per_step symbols
(models/decoder.py:131-136, 153-167; csrc/rnnt_model.hpp:115-121 -> greedy_decode_update).  The
throughput model's planted anti-repeat prior almost never gets there, so these tests run on the cap
checkpoint (synthetic.CAP_RECIPE), on which the reference's own greedy_decode_f32 hits the cap on
most rows (tests/golden/make_golden.py asserts it; golden cap_* keys):
* the fused int8 / bf16 decode (dec_joint_kernel's update) vs the restatement, which counts the
  cap-forced advances per row and must see them;
* the reference graph's op-by-op loop (lstm_amx_bf16 -> amx_linear_* -> argmax ->
  greedy_decode_update) on the same model;
* the fp32 decoder (decoder_f32.hip) vs the reference's own fp32 tokens of the fixture.
"""
import numpy as np
import pytest
import torch

from rnnt_amd import synthetic, weights

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cap_ckpt(golden):
    ck = synthetic.make_checkpoint(synthetic.DEFAULT_SEED, synthetic.CAP_RECIPE)
    assert synthetic.checkpoint_digest(ck) == bytes(golden["cap_digest"]).decode()
    return ck


@pytest.fixture(scope="module")
def cap_pm(cap_ckpt, golden):
    x = np.pad(golden["cap_x"], ((0, 0), (0, 0), (0, 16)))
    amax = weights.calibrate_amax(weights.migrate_state_dict(cap_ckpt), x, golden["cap_lens"])
    return weights.prepare_model(cap_ckpt, amax, bf16=True)


def _cap_input(golden, reps=3):
    """The fixture's 6 utterances, repeated so the batch spans several 16-row decode tiles."""
    x, lens = golden["cap_x"], golden["cap_lens"]
    x = np.concatenate([x] * reps, 1)
    lens = np.concatenate([lens] * reps)
    return np.pad(x, ((0, 0), (0, 0), (0, 16))), lens


def test_fused_decode_at_the_cap(cap_pm, golden, oracle):
    from rnnt_amd.engine import Engine
    x, lens = _cap_input(golden)
    n, T, n_pad = len(lens), x.shape[0], 256
    xp = np.zeros((T, n_pad, 256), np.float32)
    xp[:, :n] = x
    lp = np.zeros(n_pad, np.int32)
    lp[:n] = lens
    eng = Engine(cap_pm, device=0, max_batch=n_pad, max_frames=64)
    try:
        f = torch.zeros(((T + 1) // 2, n_pad, 1024), dtype=torch.float32, device="cuda")
        res = torch.empty((n, eng.max_res), dtype=torch.int32, device="cuda")
        rl = torch.empty(n, dtype=torch.int32, device="cuda")
        eng.encode(torch.from_numpy(xp).cuda(), torch.from_numpy(lp).cuda(), lens, n=n, f_out=f)
        eng.decode(res, rl)
        torch.cuda.synchronize()
        fo = oracle.encoder_i8(cap_pm, x, lens)
        fg = f.cpu().numpy()[:, :n]
        for i in range(n):
            fl = (lens[i] + 1) // 2
            assert np.array_equal(fg[:fl, i].view(np.uint32), fo[:fl, i].view(np.uint32)), f"encoder row {i}"
        ro, rlo, _, caps = oracle.greedy_decode_caps(cap_pm, fo, (lens + 1) // 2, max_res=eng.max_res)
        assert (caps > 0).sum() >= 3, f"the input does not reach the cap: {caps}"
        np.testing.assert_array_equal(rl.cpu().numpy(), rlo)
        np.testing.assert_array_equal(res.cpu().numpy(), ro)
    finally:
        eng.close()


def test_op_loop_at_the_cap(cap_pm, golden, oracle):
    """TorchModel::decode's op loop (rnnt_model.hpp:92-124) on torch.ops.intel_mlperf with the cap
    model's reference-layout weights: tokens, res_idx and the -1 fill equal the restatement's."""
    from rnnt_amd import ops
    from test_torch_ops_gpu import _decode, _eager_step, _encoder
    ops.load_library()
    W = ops.reference_weights(cap_pm, device="cpu")
    x, lens = _cap_input(golden, reps=2)
    xd = torch.from_numpy(x[:, :, :240].copy()).cuda()
    ld = torch.from_numpy(lens).cuda()
    f, _ = _encoder(W, xd, ld)
    torch.cuda.synchronize()
    fo = oracle.encoder_i8(cap_pm, x, lens)
    f_lens = ((ld + 1) // 2).to(torch.int32)
    st = _decode(W, f, f_lens, _eager_step(W))
    ro, rlo, _, caps = oracle.greedy_decode_caps(ops.op_model(cap_pm), fo, (lens + 1) // 2,
                                                 max_res=st["res"].shape[1])
    assert (caps > 0).sum() >= 2, caps
    np.testing.assert_array_equal((st["res_idx"] + 1).cpu().numpy(), rlo)
    np.testing.assert_array_equal(st["res"].cpu().numpy(), ro)


def test_f32_decoder_at_the_cap_matches_reference(cap_ckpt, golden):
    """The fp32 run_mode through GreedyDecoder (pytorch_sut.py's model call) on the cap fixture:
    the reference's own tokens, produced with the cap firing on most rows."""
    from rnnt_amd.decoder import GreedyDecoder
    from rnnt_amd.model import RNNT
    assert golden["cap_f32_caps"].max() > 0
    m = RNNT(cap_ckpt, "f32", enable_bf16=False)
    n = len(golden["cap_lens"])
    dec = GreedyDecoder(m, "f32", False, batch_size=n, max_frames=64)
    try:
        res, rl = dec(torch.from_numpy(golden["cap_x"]).cuda(), torch.from_numpy(golden["cap_lens"]))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(rl.cpu().numpy(), golden["cap_f32_len"])
        for i in range(n):
            L = int(golden["cap_f32_len"][i])
            np.testing.assert_array_equal(res[i, :L].cpu().numpy(), golden["cap_f32_res"][i, :L])
            assert bool((res[i, L:] == -1).all())
    finally:
        dec.close()
