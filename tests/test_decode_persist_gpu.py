"""The persistent tail decode (decoder.hip dec_persist_kernel, rnnt_engine_set_decode_persist): once
at most `rows` rows of a decode call are live, one launch runs every remaining lock-step step with the
step kernels' own bodies, weight slices kept in registers and the phases handed off through device
counters.  Tokens (res rows incl. the -1 fill, res_len) must equal the restatement's and the
four-launch loop's, also where the cap fires and in the Server's chunked calls."""
import numpy as np
import pytest

from rnnt_amd import synthetic, weights

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def model():
    return weights.build_model()[0]


def _run(pm, x, lens, persist, n_pad=256):
    from rnnt_amd.engine import Engine
    n, T = len(lens), x.shape[0]
    xp = np.zeros((T, n_pad, 256), np.float32)
    xp[:, :n] = x
    lp = np.zeros(n_pad, np.int32)
    lp[:n] = lens
    eng = Engine(pm, device=0, max_batch=n_pad, max_frames=max(64, T))
    try:
        eng.set_decode_persist(persist)
        res = torch.empty((n, eng.max_res), dtype=torch.int32, device="cuda")
        rl = torch.empty(n, dtype=torch.int32, device="cuda")
        eng.encode(torch.from_numpy(xp).cuda(), torch.from_numpy(lp).cuda(), lens, n=n)
        eng.decode(res, rl)
        torch.cuda.synchronize()
        st = eng.stats(reset=True)
        return res.cpu().numpy(), rl.cpu().numpy(), st, eng.max_res
    finally:
        eng.close()


@pytest.mark.parametrize("persist", [1, 16, 64, 512])
def test_persistent_tail_matches_oracle(model, oracle, persist):
    """40 rows of mixed lengths: the persistent launch takes over after the first 32-step chunk
    (64: nearly the whole decode; 1: only the last row), token-identical to the restatement."""
    lens = np.array([120, 7, 64, 99, 3, 0, 118, 45, 80, 31] * 4, np.int32)
    n, T = len(lens), int(lens.max())
    x = synthetic.make_features(T, n, seed=71, lens=lens)
    res, rl, st, max_res = _run(model, x, lens, persist)
    fo = oracle.encoder_i8(model, x, lens)
    ro, rlo, _ = oracle.greedy_decode(model, fo, (lens + 1) // 2, max_res=max_res)
    assert rlo.max() > 30
    np.testing.assert_array_equal(rl, rlo)
    np.testing.assert_array_equal(res, ro)


def test_persistent_tail_equals_four_launch_loop(model):
    """A 512-row batch of dev-clean-shaped lengths: the persistent tail (32, 256 and 512 rows: 2 to
    32 joint workgroups, prediction workgroups looping over up to 16 row tiles) and the four-launch
    loop give the same tokens."""
    lens = np.minimum(synthetic.devclean_lengths(512, seed=73), 160).astype(np.int32)
    T = int(lens.max())
    x = synthetic.make_features(T, len(lens), seed=74, lens=lens)
    r0, l0, _, _ = _run(model, x, lens, 0, n_pad=512)
    for persist in (32, 256, 512):
        r1, l1, _, _ = _run(model, x, lens, persist, n_pad=512)
        np.testing.assert_array_equal(l1, l0)
        np.testing.assert_array_equal(r1, r0)


def test_persistent_tail_at_the_cap(golden, oracle):
    """The cap checkpoint (the reference's own decode hits max_symbols_per_step there): the
    persistent launch runs the forced advances too."""
    ck = synthetic.make_checkpoint(synthetic.DEFAULT_SEED, synthetic.CAP_RECIPE)
    x = np.pad(np.concatenate([golden["cap_x"]] * 3, 1), ((0, 0), (0, 0), (0, 16)))
    lens = np.concatenate([golden["cap_lens"]] * 3)
    amax = weights.calibrate_amax(weights.migrate_state_dict(ck), x, lens)
    pm = weights.prepare_model(ck, amax, bf16=True)
    res, rl, _, max_res = _run(pm, x, lens, 64)
    fo = oracle.encoder_i8(pm, x, lens)
    ro, rlo, _, caps = oracle.greedy_decode_caps(pm, fo, (lens + 1) // 2, max_res=max_res)
    assert (caps > 0).sum() >= 3
    np.testing.assert_array_equal(rl, rlo)
    np.testing.assert_array_equal(res, ro)


def test_persistent_tail_in_server_chunks(model):
    """The Server's chunked calls (encode_stream / decode_stream, per-slot state carried across
    calls, slots reset between utterances): identical answers with and without the persistent
    tail."""
    from rnnt_amd.sut import GpuQSL, QuerySample, ServerSUT
    from rnnt_amd.engine import Engine
    lengths = np.minimum(synthetic.devclean_lengths(48, seed=75), 200)
    out = []
    for persist in (0, 32):
        qsl = GpuQSL(lengths, seed=76)
        eng = Engine(model, device=0, max_batch=256, max_frames=500)
        eng.set_decode_persist(persist)
        try:
            import time
            srv = ServerSUT([eng], qsl, slots=256, split_len=64)
            srv.start()
            srv.issue_query([QuerySample(id=i, index=i) for i in range(len(lengths))])
            srv.flush_queries()
            deadline = time.time() + 90
            while len(srv.latency) < len(lengths) and time.time() < deadline and not srv.errors:
                time.sleep(0.005)
            srv.stop()
            assert not srv.errors and len(srv.responses) == len(lengths), srv.errors
            out.append(dict(srv.responses))
        finally:
            eng.close()
    for k in out[0]:
        np.testing.assert_array_equal(out[1][k], out[0][k])
