"""The GreedyDecoder / SUT mirrors on the GPU against the CPU restatement, at batch sizes that are
not multiples of the engine's tile (the operator library: tests/test_torch_ops_gpu.py)."""
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


def test_server_sut_dynamic_batching(dec, model):
    """DynamicBatchServerSUT (dynamic batching over two engines in flight) answers every sample with the
    same tokens as the Offline path, whatever batches the arrivals happened to form."""
    import time
    from rnnt_amd.engine import Engine
    from rnnt_amd.sut import DynamicBatchServerSUT, GpuQSL, OfflineSUT, QuerySample
    lengths = np.minimum(synthetic.devclean_lengths(40, seed=51), 128)
    qsl = GpuQSL(lengths, seed=52)
    e2 = Engine(model, device=0, max_batch=64, max_frames=128)
    try:
        srv = DynamicBatchServerSUT([dec.engine, e2], qsl, max_batch=16)
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
