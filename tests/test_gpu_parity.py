"""HIP engine vs the CPU restatement (oracle/), through the C ABI.  Bit-exact on every int8 /
fp16 / fp32 tensor and token-identical (the numerics contract makes the decode exact too)."""
import numpy as np
import pytest

from rnnt_amd import synthetic, weights
from rnnt_amd.engine import pad_batch

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def model():
    pm, _ = weights.build_model()
    return pm


@pytest.fixture(scope="module")
def engine(model):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rnnt_amd.engine import Engine
    e = Engine(model, device=0, max_batch=256, max_frames=500)
    yield e
    e.close()


@pytest.fixture(params=["big", "small", "tiny", "mini", "flow"])
def tile(request, engine):
    """Every encoder tile variant (256 x 256; 128 x 128 with a 2- and a 4-deep stage ring;
    64 x 128 with a 4-deep ring, encoder.hip) pinned in turn (rnnt_engine_set_tile); the engine
    otherwise picks one per tick."""
    engine.set_tile(request.param)
    yield request.param
    engine.set_tile("auto")


def _cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _valid(f, lens):
    fl = (np.asarray(lens) + 1) // 2
    return np.concatenate([f[: fl[n], n].reshape(-1) for n in range(len(lens))])


def test_pre_rnn_layers_bitexact(engine, model, oracle, tile):
    T, n, n_pad = 7, 5, 256
    rng = np.random.default_rng(5)
    x = synthetic.make_features(T, n_pad, seed=3)
    hx = rng.integers(-128, 128, (2, n_pad, 1024)).astype(np.int8)
    cx = (rng.standard_normal((2, n_pad, 1024)) * 3).astype(np.float16).view(np.uint16)
    y = torch.zeros((T, n_pad, 1024), dtype=torch.int8, device="cuda")
    hd, cd = _cuda(hx), _cuda(cx)
    engine.lstm_int8(0, 2, _cuda(x), hd, cd, y)
    torch.cuda.synchronize()
    xq = oracle.quantize(x, model.enc_in_s[0])
    y0, h0, c0 = oracle.lstm_i8_layer(xq, model.enc_w[0], model.enc_bq[0], model.enc_rb[0], model.enc_in_s[0],
                                      model.enc_out_s[0], False, hx[0], cx[0])
    y1, h1, c1 = oracle.lstm_i8_layer(y0, model.enc_w[1], model.enc_bq[1], model.enc_rb[1], model.enc_in_s[1],
                                      model.enc_out_s[1], False, hx[1], cx[1])
    np.testing.assert_array_equal(y.cpu().numpy(), y1)
    np.testing.assert_array_equal(hd.cpu().numpy(), np.stack([h0, h1]))
    np.testing.assert_array_equal(cd.cpu().numpy(), np.stack([c0, c1]))


def test_post_rnn_layers_bitexact(engine, model, oracle, tile):
    T, n_pad = 5, 256
    rng = np.random.default_rng(6)
    x = rng.integers(-128, 128, (T, n_pad, 2048)).astype(np.int8)
    hx = np.zeros((3, n_pad, 1024), np.int8)
    cx = np.zeros((3, n_pad, 1024), np.uint16)
    y = torch.zeros((T, n_pad, 1024), dtype=torch.float32, device="cuda")
    hd, cd = _cuda(hx), _cuda(cx)
    engine.lstm_int8(2, 3, _cuda(x), hd, cd, y)
    torch.cuda.synchronize()
    cur = x
    for i, l in enumerate((2, 3, 4)):
        cur, hh, cc = oracle.lstm_i8_layer(cur, model.enc_w[l], model.enc_bq[l], model.enc_rb[l], model.enc_in_s[l],
                                          model.enc_out_s[l], l == 4, hx[i], cx[i])
        np.testing.assert_array_equal(hd[i].cpu().numpy(), hh)
        np.testing.assert_array_equal(cd[i].cpu().numpy(), cc)
    np.testing.assert_array_equal(y.cpu().numpy().view(np.uint32), cur.view(np.uint32))


def test_stack_time_op(engine, oracle):
    T, n_pad = 9, 256
    x = np.random.default_rng(7).integers(-128, 128, (T, n_pad, 1024)).astype(np.int8)
    lens = np.zeros(n_pad, np.int32)
    lens[:4] = [9, 4, 1, 0]
    y = torch.empty(((T + 1) // 2, n_pad, 2048), dtype=torch.int8, device="cuda")
    engine.stack_time(_cuda(x), _cuda(lens), y)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(y.cpu().numpy(), oracle.stack_time_i8(x, lens))


def _run(engine, model, oracle, T, lens, seed):
    n = len(lens)
    n_pad = pad_batch(n)
    lens_pad = np.zeros(n_pad, np.int32)
    lens_pad[:n] = lens
    x = synthetic.make_features(T, n_pad, seed=seed, lens=lens_pad)
    Tp = (T + 1) // 2
    f = torch.zeros((Tp, n_pad, 1024), dtype=torch.float32, device="cuda")
    res = torch.empty((n, engine.max_res), dtype=torch.int32, device="cuda")
    rl = torch.empty(n, dtype=torch.int32, device="cuda")
    engine.encode(_cuda(x), _cuda(lens_pad), lens, n=n, f_out=f)
    engine.decode(res, rl)
    torch.cuda.synchronize()
    fo = oracle.encoder_i8(model, x, lens_pad)
    fg = f.cpu().numpy()
    np.testing.assert_array_equal(_valid(fg[:, :n], lens).view(np.uint32), _valid(fo[:, :n], lens).view(np.uint32))
    ro, rlo, steps = oracle.greedy_decode(model, fo[:, :n], (lens + 1) // 2, max_res=engine.max_res)
    rl_g, res_g = rl.cpu().numpy(), res.cpu().numpy()
    np.testing.assert_array_equal(rl_g, rlo)
    np.testing.assert_array_equal(res_g, ro)  # including the -1 fill past res_len
    return rlo, steps


def test_infer_small_batch(engine, model, oracle, tile):
    rl, steps = _run(engine, model, oracle, 60, np.array([60, 51, 33, 8, 1, 60, 17, 2], np.int32), seed=1)
    assert rl.sum() > 0


def test_infer_edge_cases(engine, model, oracle, tile):
    """odd T, a zero-length utterance (batch padding row), length-1 and unsorted lengths."""
    _run(engine, model, oracle, 31, np.array([3, 31, 0, 1, 30, 29], np.int32), seed=2)
    _run(engine, model, oracle, 2, np.array([2], np.int32), seed=4)


def test_config3_int8_full_batch128(engine, model, oracle, tile):
    """BASELINE config 3: int8 enc + bf16 pred/joint greedy, N=128, lengths U{47..500}, sorted
    descending like the QSL (rnnt_qsl.cpp:104-133)."""
    lens = np.sort(synthetic.uniform_lengths(128, seed=3))[::-1].copy()
    rl, steps = _run(engine, model, oracle, int(lens.max()), lens, seed=3)
    emit_rate = rl.sum() / ((lens + 1) // 2).sum()
    assert 0.02 < emit_rate < 5, emit_rate


def test_large_batch_rows_match_small_batch(engine, model, oracle):
    """N=4096 (16 batch tiles: several tiles per workgroup / CU, every tick schedule path) on the
    256 x 256 tile vs the same rows run as small batches on the 128 x 128 tile: the int8 encoder
    is exact and row-independent, so encoder frames must be bit-identical and tokens identical
    whatever the batch composition and tile shape; the first rows are also checked against the
    oracle directly."""
    from rnnt_amd.engine import Engine
    n, T = 4096, 20
    lens = np.sort(np.random.default_rng(11).integers(1, T + 1, n).astype(np.int32))[::-1].copy()
    x = synthetic.make_features(T, n, seed=11, lens=lens)
    Tp = (T + 1) // 2
    big = Engine(model, device=0, max_batch=n, max_frames=T)
    big.set_tile("big")
    try:
        f = torch.zeros((Tp, n, 1024), dtype=torch.float32, device="cuda")
        res = torch.empty((n, big.max_res), dtype=torch.int32, device="cuda")
        rl = torch.empty(n, dtype=torch.int32, device="cuda")
        big.encode(_cuda(x), _cuda(lens), lens, n=n, f_out=f)
        big.decode(res, rl)
        torch.cuda.synchronize()
        fg, res_g, rl_g = f.cpu().numpy(), res.cpu().numpy(), rl.cpu().numpy()
    finally:
        big.close()
    engine.set_tile("small")
    try:
        for lo in (0, 1800, 4096 - 200):
            rows = np.arange(lo, lo + 200)
            sl = lens[rows]
            xs = np.zeros((T, 256, x.shape[2]), np.float32)
            xs[:, :200] = x[:, rows]
            lp = np.zeros(256, np.int32)
            lp[:200] = sl
            fs = torch.zeros((Tp, 256, 1024), dtype=torch.float32, device="cuda")
            rs = torch.empty((200, res_g.shape[1]), dtype=torch.int32, device="cuda")
            rls = torch.empty(200, dtype=torch.int32, device="cuda")
            engine.encode(_cuda(xs), _cuda(lp), sl, n=200, f_out=fs)
            engine.decode(rs, rls)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(_valid(fs.cpu().numpy()[:, :200], sl).view(np.uint32),
                                          _valid(fg[:, rows], sl).view(np.uint32))
            np.testing.assert_array_equal(rls.cpu().numpy(), rl_g[rows])
            np.testing.assert_array_equal(rs.cpu().numpy(), res_g[rows])
            if lo == 0:
                fo = oracle.encoder_i8(model, xs[:, :8], lp[:8])
                np.testing.assert_array_equal(_valid(fg[:, :8], lens[:8]).view(np.uint32), _valid(fo, lens[:8]).view(np.uint32))
    finally:
        engine.set_tile("auto")


@pytest.mark.gpu
def test_engine_rejects_sizes_past_the_decode_entry_fields(model):
    """The decode's live-list entries hold the row in 24 bits and the frame / f_len in 16 bits
    each (decoder.hip live_entry): an engine whose frames could exceed them is refused at create."""
    from rnnt_amd._lib import EngineError
    from rnnt_amd.engine import Engine
    with pytest.raises(EngineError, match="max_batch or max_frames too large"):
        Engine(model, device=0, max_batch=256, max_frames=2 * 65536 + 2)
