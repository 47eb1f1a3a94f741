"""Server scenario on the GPU: continuous batching with carried state (reference ServerSUT,
csrc/torch_sut.cpp:238-571; PipelineState, csrc/metadata.cpp:97-194).

* engine level: utterances fed in split_len chunks through rnnt_engine_encode_stream /
  rnnt_engine_decode_stream while finished slots are refilled -- every answer equals the CPU
  restatement's whole-utterance answer (chunking is exact);
* the same through the pipelined entry points (round k+1 encodes while round k decodes);
* BASELINE config 5 shape: Poisson arrivals over a 2513-sample dev-clean-shaped QSL into the
  ServerSUT (two engines in flight, slot refill, early response, QoS deferral of the longest
  samples until FlushQueries) -- every response equals the Offline answer for that sample, and a
  spread of them equals the CPU restatement."""
import time

import numpy as np
import pytest
import torch

from rnnt_amd import synthetic, weights
from rnnt_amd._lib import EngineError
from rnnt_amd.engine import Engine
from rnnt_amd.sut import GpuQSL, OfflineSUT, QuerySample, ServerSUT, make_batches

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pm():
    return weights.build_model()[0]


def _oracle_answers(oracle, pm, qsl, idx):
    sl = qsl.lengths[idx].astype(np.int32)
    x = np.zeros((int(sl.max()), len(idx), 256), np.float32)
    for i, q in enumerate(idx):
        o = int(qsl.offsets[q])
        x[: sl[i], i, :240] = qsl.feats[o: o + int(sl[i])].cpu().numpy()
    f = oracle.encoder_i8(pm, x, sl)
    ro, rlo, _ = oracle.greedy_decode(pm, f, (sl + 1) // 2, max_res=250 * 30)
    return [ro[i, : rlo[i]] for i in range(len(idx))]


@pytest.mark.parametrize("pl,slot_rows", [(False, (0, 1, 2)), (True, (0, 1, 2)), (False, (5, 300, 301))],
                         ids=["plain", "pipelined_calls", "plain_tile_holes"])
def test_stream_chunks_with_refill_equal_whole_utterances(pm, oracle, pl, slot_rows):
    """Slots keep their LSTM / prediction state across chunks; a slot that finishes is refilled
    (reset) with the next utterance while the others continue.  pl: the same rounds through the
    pipelined entry points (rnnt_engine_encode_stream_pl / decode_stream_pl) from one thread.
    slot_rows (5, 300, 301) of 512: busy rows in 128-row tiles 0 and 2 only, so every tick's
    batch-tile mask has holes (tiles 1 and 3) and, once slot 5 idles, tile 0 drops out while tile 2
    runs on."""
    lens = np.array([137, 64, 92, 161, 45, 130, 77, 104, 59], np.int32)  # odd lengths end in odd chunks
    x = synthetic.make_features(int(lens.max()), len(lens), seed=61, lens=lens)  # emits 251 symbols in all
    store = torch.from_numpy(np.concatenate([x[: lens[i], i, :240] for i in range(len(lens))])).cuda()
    qsl = GpuQSL(lens, seed=0, store=store)
    S, L, nslot = (256 if max(slot_rows) < 256 else 512), 16, len(slot_rows)
    eng = Engine(pm, device=0, max_batch=S, max_frames=200)
    try:
        res = torch.empty((S, eng.max_res), dtype=torch.int32, device="cuda")
        rl = torch.zeros(S, dtype=torch.int32, device="cuda")
        if pl:  # a pipelined decode needs its chunk's pipelined encode first
            with pytest.raises(EngineError, match="before encode_stream_pl"):
                eng.decode_stream_pl(res, rl, torch.zeros(S, dtype=torch.int32, device="cuda"))
        queue = list(range(len(lens)))
        slot = [None] * S
        pos, remain = np.zeros(S, np.int64), np.zeros(S, np.int32)
        got, rounds = {}, 0
        while queue or any(slot[i] is not None for i in slot_rows):
            reset = np.zeros(S, np.int32)
            for i in slot_rows:
                if slot[i] is None and queue:
                    slot[i] = queue.pop(0)
                    pos[i], remain[i], reset[i] = 0, lens[slot[i]], 1
            busy = np.array([s is not None for s in slot])
            cl = np.where(busy, np.minimum(remain, L), 0).astype(np.int32)
            off = np.array([qsl.offsets[s] if s is not None else 0 for s in slot], np.int64) + pos
            T = max(int(cl.max()), 1)
            rd = torch.from_numpy(reset).cuda()
            enc, dec = (eng.encode_stream_pl, eng.decode_stream_pl) if pl else (eng.encode_stream, eng.decode_stream)
            enc(qsl.feats, torch.from_numpy(np.where(busy, off, 0)).cuda(), torch.from_numpy(cl).cuda(), cl, rd, T, S, S)
            dec(res, rl, rd)
            torch.cuda.synchronize()
            pos += cl
            remain -= cl
            rlh = rl.cpu().numpy()
            for i in np.nonzero(busy & (remain == 0))[0]:
                got[slot[i]] = res[i, : rlh[i]].cpu().numpy()
                slot[i] = None
            rounds += 1
        assert rounds > len(lens) // nslot + 2  # utterances really spanned several chunks
        if pl:  # every chunk was decoded: one more decode has no chunk; round-form calls are refused
            with pytest.raises(EngineError, match="before its chunk"):
                eng.decode_stream_pl(res, rl, rd)
            with pytest.raises(EngineError, match="pipelined"):
                eng.decode_stream(res, rl, rd)
    finally:
        eng.close()
    want = _oracle_answers(oracle, pm, qsl, np.arange(len(lens)))
    assert sum(len(w) for w in want) > 200
    for q in range(len(lens)):
        np.testing.assert_array_equal(got[q], want[q], err_msg=f"utterance {q} (len {lens[q]})")


@pytest.mark.parametrize("pipelined,refill", [(False, "fcfs"), (True, "fcfs"), (False, "tile")],
                         ids=["rounds", "pipelined", "rounds_tile_refill"])
def test_config5_server_continuous_batching(pm, oracle, pipelined, refill):
    count, n, qps = 2513, 1200, 3000.0
    lengths = synthetic.devclean_lengths(count, seed=4)
    qsl = GpuQSL(lengths, seed=4, device="cuda")
    engines = [Engine(pm, device=0, max_batch=512, max_frames=500) for _ in range(2)]
    rng = np.random.default_rng(5)
    index = rng.integers(0, count, size=n)
    arrivals = np.cumsum(rng.exponential(1.0 / qps, size=n))
    qos = 460  # frames (the reference's QOS=233500 wav samples = 14.6 s)
    try:
        # refill='tile': whole 128-row tiles refilled with similar lengths, so stream chunks skip done
        # tiles wherever they sit (the tick kernel's batch-tile mask)
        srv = ServerSUT(engines, qsl, slots=512, split_len=32, qos_len=qos, pipelined=pipelined, refill=refill)
        srv.warmup(iters=1)  # ServerSUT::warmup (torch_sut.cpp:328-352): dummy rounds leave no trace in the answers
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
        deferred = len(srv._qos)
        deadline = time.time() + 60
        regular = int((lengths[index] <= qos).sum())
        while len(srv.latency) < regular and time.time() < deadline and not srv.errors:
            time.sleep(0.005)
        # deferred samples are not served before FlushQueries
        long_ids = [k for k in range(n) if lengths[index[k]] > qos]
        assert not any(k in srv.responses for k in long_ids)
        srv.flush_queries()
        while len(srv.latency) < n and time.time() < deadline and not srv.errors:
            time.sleep(0.005)
        srv.stop()
        assert not srv.errors, srv.errors
        assert len(srv.responses) == n and deferred == len(long_ids) > 0
        assert srv.rounds > 2 * 500 // 32  # chunked: the longest samples took >= 16 rounds
        # the Offline answers of the same samples (sorted batches of whole utterances)
        if pipelined:  # an engine that ran pipelined stream calls refuses the other calls
            engines.append(Engine(pm, device=0, max_batch=512, max_frames=500))
        off = OfflineSUT(engines[-1], qsl, batch_size=512)
        off.issue_batches(make_batches(qsl, np.arange(n), index, 512))
        offline = off.responses
    finally:
        for e in engines:
            e.close()
    for k in range(n):
        np.testing.assert_array_equal(srv.responses[k], offline[k], err_msg=f"sample {k} (QSL {index[k]})")
    lat = np.array([srv.latency[k] for k in range(n) if k not in set(long_ids)])
    assert np.isfinite(lat).all() and np.percentile(lat, 99) < 1.0  # the Server bound at this load
    # the CPU restatement on a spread of samples, shortest to longest (incl. deferred ones)
    ks = np.argsort(lengths[index], kind="stable")[np.linspace(0, n - 1, 12).round().astype(int)]
    want = _oracle_answers(oracle, pm, qsl, index[ks])
    for k, w in zip(ks, want):
        np.testing.assert_array_equal(srv.responses[int(k)], w, err_msg=f"sample {k}")


def test_pipelined_decode_failure_does_not_hang_the_next_encode(pm):
    """A pipelined decode that fails before its hand-off (here: no result columns, max_res 0)
    marks the engine failed and wakes the encode side: the next encode_stream_pl returns an error
    instead of waiting forever for a hand-off that will not come."""
    import threading
    S = 256
    lens = np.array([40, 33, 20], np.int32)
    qsl = GpuQSL(lens, seed=3, device="cuda")
    eng = Engine(pm, device=0, max_batch=S, max_frames=64)
    try:
        cl = np.zeros(S, np.int32)
        cl[:3] = 16
        off = np.zeros(S, np.int64)
        off[:3] = qsl.offsets[:3]
        reset = torch.zeros(S, dtype=torch.int32, device="cuda")
        reset[:3] = 1
        args = (qsl.feats, torch.from_numpy(off).cuda(), torch.from_numpy(cl).cuda(), cl, reset, 16, S, S)
        eng.encode_stream_pl(*args)
        res0 = torch.empty((S, 0), dtype=torch.int32, device="cuda")
        rl = torch.zeros(S, dtype=torch.int32, device="cuda")
        with pytest.raises(EngineError):
            eng.decode_stream_pl(res0, rl, reset)
        out = []

        def nxt():
            try:
                eng.encode_stream_pl(*args)
                out.append("returned")
            except EngineError as ex:
                out.append(str(ex))

        th = threading.Thread(target=nxt, daemon=True)
        th.start()
        th.join(timeout=30)
        assert not th.is_alive(), "encode_stream_pl still waiting for the failed decode's hand-off"
        assert out and "failed" in out[0], out
    finally:
        torch.cuda.synchronize()
        eng.close()
