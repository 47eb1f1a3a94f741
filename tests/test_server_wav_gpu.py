"""Server over WAV on the GPU (reference ServerSUT with processor=true: producers featurize
queued samples, consumers run the model, torch_sut.cpp:354-571): WAV feeds featurize arriving
samples into per-device feature stores (rnnt_featurizer_run_rows) and the continuous-batching
ServerSUT's engines encode from those stores chunk by chunk.  Two feeds, each with its own audio
copy and store, serve one Server instance -- on this one-GPU box both sit on device 0, which
exercises the same lanes as two devices would (the routing itself is covered on CPU by
test_server_feed.py).  Every response equals the Offline answer of the same audio (padded
featurizer batch, whole-utterance encode), and a spread of them equals the CPU restatement run on
the GPU's features."""
import time

import numpy as np
import pytest
import torch

from rnnt_amd import synthetic, weights
from rnnt_amd.engine import Engine
from rnnt_amd.sut import GpuWavQSL, OfflineSUT, QuerySample, ServerSUT, WavFeed, make_batches

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("pipelined", [False, True], ids=["rounds", "pipelined"])
def test_server_over_wav_feeds(oracle, pipelined):
    pm = weights.build_model()[0]
    count, n, qps, qos = 240, 600, 1500.0, 420
    frames = np.minimum(synthetic.devclean_lengths(count, seed=71), 480)
    wavs = synthetic.make_wavs(synthetic.wav_lengths_for_frames(frames, seed=71), seed=71, device="cuda")
    qsls = [GpuWavQSL(wavs) for _ in range(2)]  # one audio copy per lane, as one per device
    assert qsls[0].lengths.tolist() == frames.tolist()
    engines = [Engine(pm, device=0, max_batch=256, max_frames=500) for _ in range(2)]
    feeds = [WavFeed(q, pro_batch=32) for q in qsls]
    rng = np.random.default_rng(72)
    index = rng.integers(0, count, size=n)
    arrivals = np.cumsum(rng.exponential(1.0 / qps, size=n))
    try:
        srv = ServerSUT(engines, slots=256, split_len=32, qos_len=qos, pipelined=pipelined, feeds=feeds)
        assert srv.lanes == [0, 1]
        srv.start()
        t0 = time.perf_counter()
        i = 0
        while i < n:
            j = int(np.searchsorted(arrivals, time.perf_counter() - t0, side="right"))
            if j > i:
                for k in range(i, j):
                    srv.issue_query([QuerySample(id=k, index=int(index[k]))], now=t0 + arrivals[k])
                i = j
            else:
                time.sleep(0.0005)
        long_ids = [k for k in range(n) if frames[index[k]] > qos]
        deadline = time.time() + 60
        while len(srv.latency) < n - len(long_ids) and time.time() < deadline and not srv.errors:
            time.sleep(0.005)
        assert not any(k in srv.responses for k in long_ids)  # QoS samples wait for FlushQueries
        srv.flush_queries()
        while len(srv.latency) < n and time.time() < deadline and not srv.errors:
            time.sleep(0.005)
        srv.stop()
        assert not srv.errors, srv.errors
        assert len(srv.responses) == n and len(long_ids) > 0
        for f in feeds:  # both lanes featurized work; every store slot came back
            assert f.batches > 0 and f.store.free == f.store.slots
        if pipelined:  # an engine that ran pipelined stream calls refuses the other calls
            engines.append(Engine(pm, device=0, max_batch=256, max_frames=500))
        off = OfflineSUT(engines[-1], qsls[0], batch_size=256)
        off.issue_batches(make_batches(qsls[0], np.arange(n), index, 256))
        offline = off.responses
    finally:
        for e in engines:
            e.close()
    for k in range(n):
        np.testing.assert_array_equal(srv.responses[k], offline[k], err_msg=f"sample {k} (QSL {index[k]})")
    lat = np.array([srv.latency[k] for k in range(n) if k not in set(long_ids)])
    assert np.isfinite(lat).all() and np.percentile(lat, 99) < 1.0
    # the CPU restatement on the GPU's features of a spread of samples (shortest to longest)
    ks = np.argsort(frames[index], kind="stable")[np.linspace(0, n - 1, 8).round().astype(int)]
    idx = [int(index[k]) for k in ks]
    x, _, bl = qsls[0].assemble(idx)
    feats = np.ascontiguousarray(x.cpu().numpy()[:, : len(idx)])
    fo = oracle.encoder_i8(pm, feats, bl)
    ro, rlo, _ = oracle.greedy_decode(pm, fo, (bl + 1) // 2, max_res=250 * 30)
    for i, k in enumerate(ks):
        np.testing.assert_array_equal(srv.responses[int(k)], ro[i, : rlo[i]], err_msg=f"sample {k}")
