"""Server over WAV, host side (CPU): the per-device feature stores and the routing of arriving
samples through WAV feeds (producers, reference ServerSUT::thProducer, torch_sut.cpp:354-468) to
the engines of their lane.  The featurize step and the engines are stand-ins here; the GPU test
(test_server_wav_gpu.py) runs the same ServerSUT with the HIP featurizer and engines."""
import threading
import time
from collections import Counter
from types import SimpleNamespace

import numpy as np
import pytest

from rnnt_amd.sut import FeatureStore, QuerySample, ServerSUT, WavFeed


def test_feature_store_slots():
    st = FeatureStore(4, 10, alloc=False)
    a = st.alloc(3)
    assert a == [0, 1, 2] and st.free == 1
    assert st.alloc(5) == [3] and st.free == 0 and st.alloc(1) == []
    st.release([1])
    assert st.alloc(1) == [1]  # the slot released last is reused first
    with pytest.raises(ValueError, match="not in use"):
        st.release([7])
    st.release([0, 1, 2, 3])
    with pytest.raises(ValueError, match="not in use"):
        st.release([0])
    assert st.free == 4 and st.row(3) == 30
    with pytest.raises(ValueError):
        FeatureStore(0, 10, alloc=False)


class _FakeQSL:
    def __init__(self, lengths, device):
        self.lengths = np.asarray(lengths, np.int32)
        self.device = device


class _FakeFeed(WavFeed):
    """featurize = record which store slot each sample went to (the HIP path writes its rows)."""

    def __init__(self, qsl, **kw):
        super().__init__(qsl, alloc=False, **kw)
        self.log = []
        self.lock = threading.Lock()

    def make_stream(self):
        return None

    def featurize(self, indices, slots, stream):
        time.sleep(0.0005)
        with self.lock:
            self.log.extend(zip(indices, slots))
        self.batches += 1
        return self.qsl.lengths[np.asarray(indices)]


def _engines(devices, max_batch=256):
    return [SimpleNamespace(device=d, max_batch=max_batch) for d in devices]


def test_lane_assignment():
    L = np.arange(1, 11)
    f0, f1 = _FakeFeed(_FakeQSL(L, "cuda:0")), _FakeFeed(_FakeQSL(L, "cuda:1"))
    srv = ServerSUT(_engines([0, 1, 0, 1]), feeds=[f0, f1], slots=256, split_len=8)
    assert srv.lanes == [0, 1, 0, 1]
    assert f0.store.slots == 2 * 256 + 256 and f0.ahead == 256  # the lane's engine slots + lookahead
    # two feeds on one device (the one-GPU rehearsal of a two-device Server): round-robin
    g0, g1 = _FakeFeed(_FakeQSL(L, "cuda:0")), _FakeFeed(_FakeQSL(L, "cuda:0"))
    assert ServerSUT(_engines([0, 0]), feeds=[g0, g1], slots=256, split_len=8).lanes == [0, 1]
    with pytest.raises(ValueError, match="no WAV feed on device 2"):
        ServerSUT(_engines([0, 2]), feeds=[_FakeFeed(_FakeQSL(L, "cuda:0"))], slots=256, split_len=8)
    with pytest.raises(ValueError, match="every feed needs"):
        ServerSUT(_engines([0]), feeds=[_FakeFeed(_FakeQSL(L, "cuda:0")), _FakeFeed(_FakeQSL(L, "cuda:1"))],
                  slots=256, split_len=8)
    with pytest.raises(ValueError, match="assigned to a feed on device"):
        ServerSUT(_engines([0, 1]), feeds=[_FakeFeed(_FakeQSL(L, "cuda:0")), _FakeFeed(_FakeQSL(L, "cuda:1"))],
                  slots=256, split_len=8, lanes=[1, 0])
    with pytest.raises(ValueError, match="same samples"):
        ServerSUT(_engines([0, 1]), feeds=[_FakeFeed(_FakeQSL(L, "cuda:0")), _FakeFeed(_FakeQSL(L + 1, "cuda:1"))],
                  slots=256, split_len=8)
    with pytest.raises(ValueError, match="feature QSL or WAV feeds"):
        ServerSUT(_engines([0]), slots=256, split_len=8)


@pytest.mark.parametrize("devices", [(0, 1), (0, 0)], ids=["two_devices", "two_feeds_one_device"])
def test_two_lane_routing(devices):
    """Bursty arrivals into two lanes: every sample is featurized once, into a slot of the store
    of the lane whose engine then serves it; a lane's featurized backlog stays within its
    lookahead; both lanes take work; QoS samples wait for FlushQueries; every slot comes back."""
    rng = np.random.default_rng(11)
    count, n, qos = 400, 900, 60
    lengths = rng.integers(5, 80, count)
    feeds = [_FakeFeed(_FakeQSL(lengths, f"cuda:{d}"), pro_batch=16) for d in devices]
    S = 256
    srv = ServerSUT(_engines(devices, max_batch=S), feeds=feeds, slots=S, split_len=8, qos_len=qos)
    served = {}  # sample id -> (lane, slot)
    max_backlog = [0, 0]
    lock = threading.Lock()

    def engine(lane):  # a stand-in consumer: S slots, one sample finishes per slot per round
        held = []
        while True:
            new = srv._take(S - len(held), busy=bool(held), lane=lane)
            if new is None:
                return
            with lock:
                max_backlog[lane] = max(max_backlog[lane], len(srv._ready[lane]))
                for t0, s, row, nfr, sl in new:
                    assert s.id not in served, "sample served twice"
                    assert row == feeds[lane].store.row(sl) and nfr == lengths[s.index]
                    served[s.id] = (lane, sl)
            held.extend(new)
            if held:
                k = max(1, len(held) // 3)
                done, held = held[:k], held[k:]
                srv._release(lane, [sl for *_, sl in done])
                with lock:
                    for t0, s, *_ in done:
                        srv.latency[s.id] = time.perf_counter() - t0
            time.sleep(0.0002)

    srv._start_producers()
    workers = [threading.Thread(target=engine, args=(f,), daemon=True) for f in range(2)]
    for w in workers:
        w.start()
    index = rng.integers(0, count, n)
    i = 0
    while i < n:  # bursts of 1..60 samples
        k = int(rng.integers(1, 61))
        srv.issue_query([QuerySample(id=j, index=int(index[j])) for j in range(i, min(n, i + k))])
        i += k
        time.sleep(0.001)
    long_ids = {j for j in range(n) if lengths[index[j]] > qos}
    deadline = time.time() + 30
    while len(srv.latency) < n - len(long_ids) and time.time() < deadline:
        time.sleep(0.002)
    assert not any(j in srv.latency for j in long_ids)  # deferred until FlushQueries
    srv.flush_queries()
    while len(srv.latency) < n and time.time() < deadline:
        time.sleep(0.002)
    srv.stop()
    for w in workers:
        w.join(timeout=10)
    assert not srv.errors, srv.errors
    assert len(served) == n and len(srv.latency) == n
    for f, fd in enumerate(feeds):  # featurized once, in the store of the lane that served it
        featurized = Counter((int(idx), int(sl)) for idx, sl in fd.log)
        consumed = Counter((int(index[j]), sl) for j, (lane, sl) in served.items() if lane == f)
        assert featurized == consumed
        assert fd.store.free == fd.store.slots and not srv._ready[f]
        assert max_backlog[f] <= fd.ahead
    by_lane = [sum(1 for v in served.values() if v[0] == f) for f in range(2)]
    assert sum(len(fd.log) for fd in feeds) == n
    assert min(by_lane) > n // 5, by_lane  # both lanes take work


class _LenQSL:
    def __init__(self, lengths):
        self.lengths = np.asarray(lengths, np.int32)
        self.offsets = np.concatenate([[0], np.cumsum(self.lengths)[:-1]]).astype(np.int64)


def test_tile_refill_groups_similar_lengths():
    """refill='tile' (DESIGN §5 Server): waiting samples are taken in groups of 128 -- the oldest
    waiting one and those closest to its length among the first refill_window -- so a refilled
    tile's rows run out together; every sample is taken exactly once, the oldest always first."""
    rng = np.random.default_rng(7)
    lengths = rng.integers(47, 501, 1000)
    srv = ServerSUT(_engines([0], max_batch=512), _LenQSL(lengths), slots=512, refill="tile", refill_window=600)
    srv.issue_query([QuerySample(id=i, index=i) for i in range(700)], now=0.0)
    got = srv._take(300, busy=True)
    assert len(got) == 300
    ids = [s.id for _, s, _, _, _ in got]
    assert len(set(ids)) == 300
    groups = [ids[0:128], ids[128:256], ids[256:300]]
    remaining = list(range(700))
    for g in groups:
        assert g[0] == min(remaining)  # the oldest waiting sample leads its group
        x0 = lengths[g[0]]
        window = remaining[:600]
        worst_in = max(abs(lengths[i] - x0) for i in g)
        outside = [abs(lengths[i] - x0) for i in window if i not in set(g)]
        assert not outside or worst_in <= min(outside)  # nobody closer was left behind
        assert g == sorted(g)  # arrival order inside the group
        remaining = [i for i in remaining if i not in set(g)]
    # the rest stays queued in arrival order
    left = [s.id for _, s in srv._pending]
    assert left == remaining
    # rows of the whole-tile refill: an fcfs SUT takes the oldest in order
    fc = ServerSUT(_engines([0], max_batch=512), _LenQSL(lengths), slots=512)
    fc.issue_query([QuerySample(id=i, index=i) for i in range(10)], now=0.0)
    assert [s.id for _, s, _, _, _ in fc._take(4, busy=True)] == [0, 1, 2, 3]
    with pytest.raises(ValueError):
        ServerSUT(_engines([0], max_batch=512), _LenQSL(lengths), slots=512, refill="tile", pipelined=True)
