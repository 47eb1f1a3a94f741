"""The intel_mlperf operator mirror (rnnt_amd.ops) and the GreedyDecoder mirror on the GPU,
against the CPU restatement, at batch sizes that are not multiples of the engine's tile."""
import numpy as np
import pytest

from rnnt_amd import synthetic, weights

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def model():
    return weights.build_model()[0]


@pytest.fixture(scope="module")
def dec(model):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rnnt_amd.decoder import GreedyDecoder
    d = GreedyDecoder(model, "quant", True, split_len=2, batch_size=64, max_frames=128)
    yield d
    d.close()


def test_lstm_amx_int8_pre_and_post(dec, model, oracle):
    from rnnt_amd import ops
    T, N = 6, 5
    x = synthetic.make_features(T, N, seed=9)[:, :, :240]
    hx = [torch.zeros((N, 1024), dtype=torch.int8, device="cuda") for _ in range(2)]
    cx = [torch.zeros((N, 1024), dtype=torch.float16, device="cuda") for _ in range(2)]
    w = [[torch.from_numpy(model.enc_w[l][:, :I]), torch.from_numpy(model.enc_w[l][:, I:]), None, None]
         for l, I in ((0, 256), (1, 1024))]
    y, h, c = ops.lstm_amx_int8(torch.from_numpy(x.copy()).cuda(), hx, cx, w, model.enc_rb[:2], model.enc_in_s[:2],
                                model.enc_out_s[:2], False)
    xq = oracle.quantize(np.pad(x, ((0, 0), (0, 0), (0, 16))), model.enc_in_s[0])
    y0, h0, c0 = oracle.lstm_i8_layer(xq, model.enc_w[0], model.enc_bq[0], model.enc_rb[0], model.enc_in_s[0],
                                      model.enc_out_s[0], False, np.zeros((N, 1024), np.int8), np.zeros((N, 1024), np.uint16))
    y1, h1, c1 = oracle.lstm_i8_layer(y0, model.enc_w[1], model.enc_bq[1], model.enc_rb[1], model.enc_in_s[1],
                                      model.enc_out_s[1], False, np.zeros((N, 1024), np.int8), np.zeros((N, 1024), np.uint16))
    np.testing.assert_array_equal(y.cpu().numpy(), y1)
    np.testing.assert_array_equal(h[1].cpu().numpy(), h1)
    np.testing.assert_array_equal(c[0].cpu().numpy().view(np.uint16), c0)
    # stack_time + post_rnn through the same surface
    lens = torch.tensor([6, 3, 6, 1, 0], dtype=torch.int32)
    xs = ops.stack_time(y, lens.cuda(), 2)
    np.testing.assert_array_equal(xs.cpu().numpy(), oracle.stack_time_i8(y1, lens.numpy()))
    hx3 = [torch.zeros((N, 1024), dtype=torch.int8, device="cuda") for _ in range(3)]
    cx3 = [torch.zeros((N, 1024), dtype=torch.float16, device="cuda") for _ in range(3)]
    w3 = [[torch.from_numpy(model.enc_w[l][:, :-1024]), torch.from_numpy(model.enc_w[l][:, -1024:]), None, None] for l in (2, 3, 4)]
    f, _, _ = ops.lstm_amx_int8(xs, hx3, cx3, w3, model.enc_rb[2:], model.enc_in_s[2:], model.enc_out_s[2:], True)
    cur = xs.cpu().numpy()
    for l in (2, 3, 4):
        cur, _, _ = oracle.lstm_i8_layer(cur, model.enc_w[l], model.enc_bq[l], model.enc_rb[l], model.enc_in_s[l],
                                         model.enc_out_s[l], l == 4, np.zeros((N, 1024), np.int8), np.zeros((N, 1024), np.uint16))
    np.testing.assert_array_equal(f.cpu().numpy().view(np.uint32), cur.view(np.uint32))


def test_greedy_decoder_mirror(dec, model, oracle):
    """GreedyDecoder.forward contract (decoder.py:21-94): res [N, 30*max_len] SOS-filled, lens."""
    lens = np.array([77, 40, 3, 60, 11], np.int32)
    T = int(lens.max())
    x = synthetic.make_features(T, len(lens), seed=12, lens=lens)[:, :, :240]
    res, rl = dec(torch.from_numpy(x.copy()).cuda(), torch.from_numpy(lens))
    assert res.shape == (5, 30 * T)
    fo = oracle.encoder_i8(model, np.pad(x, ((0, 0), (0, 0), (0, 16))), lens)
    ro, rlo, _ = oracle.greedy_decode(model, fo, (lens + 1) // 2, max_res=30 * T)
    np.testing.assert_array_equal(rl.cpu().numpy(), rlo)
    np.testing.assert_array_equal(res.cpu().numpy(), ro)


def test_offline_sut_end_to_end(dec, model, oracle):
    """OfflineSUT.issue_queries (torch_sut.cpp:140-236 semantics): sorted batches through the
    engine, each sample completed with its own token row; identical to the CPU restatement."""
    from rnnt_amd.sut import OfflineSUT, QuerySample, RNNTQSL
    lengths = synthetic.devclean_lengths(37, seed=31)
    lengths = np.minimum(lengths, 128)
    qsl = RNNTQSL.synthetic(lengths, seed=32)
    done = []
    sut = OfflineSUT(dec.engine, qsl, batch_size=16, on_complete=lambda s, row: done.append(s.id))
    samples = [QuerySample(id=1000 + i, index=i) for i in range(len(lengths))]
    sut.issue_queries(samples)
    assert sorted(done) == [s.id for s in samples]
    for s in samples[:8]:
        L = int(lengths[s.index])
        x = np.zeros((L, 1, 256), np.float32)
        x[:, 0, :240] = qsl.features[s.index]
        fo = oracle.encoder_i8(model, x, np.array([L], np.int32))
        ro, rlo, _ = oracle.greedy_decode(model, fo, np.array([(L + 1) // 2], np.int32))
        np.testing.assert_array_equal(sut.responses[s.id], ro[0, : rlo[0]])


def test_offline_sut_batches_in_flight(dec, model):
    """Two engines on one GPU (own stream + host thread each, encoders taking turns) give the
    same responses as one engine: the pipelining is pure scheduling."""
    from rnnt_amd.engine import Engine
    from rnnt_amd.sut import OfflineSUT, QuerySample, RNNTQSL
    lengths = np.minimum(synthetic.devclean_lengths(53, seed=41), 128)
    qsl = RNNTQSL.synthetic(lengths, seed=42)
    samples = [QuerySample(id=i, index=i) for i in range(len(lengths))]
    one = OfflineSUT(dec.engine, qsl, batch_size=12)
    one.issue_queries(samples)
    e2 = Engine(model, device=0, max_batch=64, max_frames=128)
    try:
        two = OfflineSUT([dec.engine, e2], qsl, batch_size=12)
        two.issue_queries(samples)
    finally:
        e2.close()
    assert sorted(two.responses) == sorted(one.responses)
    for k in one.responses:
        np.testing.assert_array_equal(two.responses[k], one.responses[k])


def test_op_by_op_greedy_loop(dec, model, oracle):
    """The reference's op-by-op decode loop (decoder.py:171-212 greedy_decode_quant) written
    with the four decode operators (lstm_amx_bf16, amx_linear_bf16_accum_relu,
    amx_linear_i16o32, greedy_decode_update) gives the same tokens as the fused device loop
    and the CPU restatement."""
    from rnnt_amd import ops
    from rnnt_amd.config import RNNTParam as R
    e = dec.engine
    lens = np.array([57, 31, 12, 44, 3], np.int32)
    N, T = len(lens), int(lens.max())
    n_pad = 256
    x = synthetic.make_features(T, n_pad, seed=21, lens=np.pad(lens, (0, n_pad - N)))
    xd = torch.from_numpy(x).cuda()
    ld = torch.from_numpy(np.pad(lens, (0, n_pad - N))).cuda()
    Tp = (T + 1) // 2
    f = torch.empty((Tp, n_pad, 1024), dtype=torch.float32, device="cuda")
    e.encode(xd, ld, lens, n=N, f_out=f)
    max_res = 30 * Tp
    # fused loop
    res_f = torch.empty((N, max_res), dtype=torch.int32, device="cuda")
    rl_f = torch.empty(N, dtype=torch.int32, device="cuda")
    e.decode(res_f, rl_f)
    # op-by-op loop
    dev = "cuda"
    f_lens = torch.from_numpy((lens + 1) // 2).to(dev)
    symbols_added = torch.zeros(N, dtype=torch.int32, device=dev)
    time_idx = torch.zeros(N, dtype=torch.int32, device=dev)
    finish = (f_lens == 0).to(torch.int32)
    res = torch.full((N, max_res), R.SOS, dtype=torch.int32, device=dev)
    res_idx = torch.full((N,), -1, dtype=torch.int32, device=dev)
    pre_g = torch.full((N,), R.SOS, dtype=torch.int32, device=dev)
    pre_hg = torch.zeros((2, n_pad, 320), dtype=torch.bfloat16, device=dev)
    pre_cg = torch.zeros((2, n_pad, 320), dtype=torch.float32, device=dev)
    fi = f[0].clone()
    embed = torch.from_numpy(np.asarray(model.embed, np.float32)).to(dev).to(torch.bfloat16)
    for _ in range(30 * Tp + Tp + 2):
        sos = pre_g.eq(R.SOS)
        xg = embed[pre_g.clamp(min=0).long()].masked_fill(sos[:, None], 0.0)  # modeling_rnnt.py:193-197
        g, hgl, cgl = ops.lstm_amx_bf16(xg.unsqueeze(0), [pre_hg[0, :N], pre_hg[1, :N]], [pre_cg[0, :N], pre_cg[1, :N]])
        hg = torch.zeros_like(pre_hg)
        cg = torch.zeros_like(pre_cg)
        for l in range(2):
            hg[l, :N] = hgl[l]
            cg[l, :N] = cgl[l]
        y1 = ops.amx_linear_bf16_accum_relu(fi[:N], None, g[0])
        logits = ops.amx_linear_i16o32(y1)
        assert torch.all(logits[:, R.num_labels:] == 0)
        symbols = torch.argmax(logits[:, : R.num_labels], dim=1).to(torch.int32)
        if ops.greedy_decode_update(symbols, symbols_added, res, res_idx, f, f_lens, time_idx, fi, pre_g, pre_hg, pre_cg,
                                    hg, cg, finish):
            break
    else:
        raise AssertionError("op-by-op loop did not finish")
    np.testing.assert_array_equal((res_idx + 1).cpu().numpy(), rl_f.cpu().numpy())
    np.testing.assert_array_equal(res.cpu().numpy(), res_f.cpu().numpy())
    fo = f.cpu().numpy()[:, :N]
    ro, rlo, _ = oracle.greedy_decode(model, fo, (lens + 1) // 2, max_res=max_res)
    np.testing.assert_array_equal(res.cpu().numpy(), ro)


def test_server_sut_dynamic_batching(dec, model):
    """ServerSUT (dynamic batching over two engines in flight) answers every sample with the
    same tokens as the Offline path, whatever batches the arrivals happened to form."""
    import time
    from rnnt_amd.engine import Engine
    from rnnt_amd.sut import GpuQSL, OfflineSUT, QuerySample, ServerSUT
    lengths = np.minimum(synthetic.devclean_lengths(40, seed=51), 128)
    qsl = GpuQSL(lengths, seed=52)
    e2 = Engine(model, device=0, max_batch=64, max_frames=128)
    try:
        srv = ServerSUT([dec.engine, e2], qsl, max_batch=16)
        srv.start()
        samples = [QuerySample(id=i, index=i) for i in range(len(lengths))]
        for k in range(0, len(samples), 7):
            srv.issue_query(samples[k:k + 7])
            time.sleep(0.002)
        deadline = time.time() + 60
        while len(srv.latency) < len(samples) and time.time() < deadline:
            time.sleep(0.01)
        srv.stop()
        assert not srv.errors and len(srv.responses) == len(samples)
        # reference answers: one Offline batch of the same samples (assembled from the same features)
        x, lens, bl = qsl.assemble(list(range(len(lengths))))
        n = len(lengths)
        res = torch.empty((n, dec.engine.max_res), dtype=torch.int32, device="cuda")
        rl = torch.empty(n, dtype=torch.int32, device="cuda")
        dec.engine.infer(x, lens, bl, res, rl, n=n)
        res, rl = res.cpu().numpy(), rl.cpu().numpy()
        for i in range(n):
            np.testing.assert_array_equal(srv.responses[i], res[i, : rl[i]])
    finally:
        e2.close()
