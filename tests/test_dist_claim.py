"""Cross-rank dynamic batch pull (CPU, gloo): every rank claims the next length-sorted batch of
one Offline query from a shared counter (dist.BatchClaim over the rendezvous TCPStore) whenever
its encoder is free -- the reference's instances pulling from one queue, torch_sut.cpp:167-182.

The OfflineSUT here is the real one (its worker threads, encode turns and claim gates) with the
device calls stood in for by host sleeps: one rank is slowed, and it must end up with fewer
batches while every response of every query reaches rank 0 unchanged.  Several queries run back
to back without a barrier between them, each with its own payloads, so a stream that mixed two
queries' messages (untagged ResponseStream) would be caught."""
import contextlib
import os
import socket
import time

import numpy as np
import torch.multiprocessing as mp

from rnnt_amd import dist as rdist
from rnnt_amd.sut import OfflineSUT, RNNTQSL, make_batches


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tokens(sid, q):
    """stand-in response of sample `sid` in query `q` (variable length, incl. empty)"""
    return (np.arange((sid + q) % 6, dtype=np.int32) + sid * 3 + q) % 29


class _HostEngine:
    def __init__(self, device, slow):
        self.device, self.slow, self.max_res = device, slow, 8


class _HostSUT(OfflineSUT):
    """OfflineSUT with the HIP calls replaced by sleeps proportional to the batch's frames."""
    query = 0

    def _stream_for(self, eng):
        return None

    def _device_scope(self, eng, st):
        return contextlib.nullcontext()

    def _encode(self, eng, st, ids, idx, n, n_pad):
        time.sleep(2e-6 * float(self.qsl.lengths[idx].sum()) * eng.slow)
        return ids

    def _decode(self, eng, st, ids):
        time.sleep(1e-6 * float(len(ids)) * eng.slow)
        rows = [_tokens(int(i), self.query) for i in ids]
        lens = np.array([len(r) for r in rows], np.int32)
        toks = np.zeros((len(ids), max(1, int(lens.max()))), np.int32)
        for k, r in enumerate(rows):
            toks[k, : len(r)] = r
        return lens, toks


def _worker(rank, world, port, slow_rank, queries, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    r, _, w, group = rdist.setup("gloo")
    lengths = np.random.default_rng(5).integers(47, 501, 900).astype(np.int32)
    qsl = RNNTQSL([None] * len(lengths), lengths)
    ids, idx = rdist.query_arrays(len(lengths), 3000)
    slow = 20.0 if rank == slow_rank else 1.0
    sut = _HostSUT([_HostEngine(0, slow) for _ in range(2)], qsl)
    out = []
    for qn in range(queries):
        batches = make_batches(qsl, ids, idx, 100)
        sut.query = qn
        stream = rdist.ResponseStream(world, group, tag=qn)
        sut.on_batch = stream.push
        sut.issue_batches(batches, claim=rdist.claim_for_query(qn, len(batches)))
        sut.take_completed()
        got = stream.finish()
        ran = [i for i, e in enumerate(sut.batch_engine) if e is not None]
        frames = int(sum(lengths[batches[i][1]].sum() for i in ran))
        out.append((ran, frames, None if got is None else (got[0].tolist(), got[1].tolist(), got[2].tolist())))
        # no barrier: the next query starts while rank 0 may still be receiving this one
    q.put((rank, out))
    rdist.barrier(group)
    dist.destroy_process_group()


def _run(world, slow_rank, queries):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, slow_rank, queries, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return outs


def _check(outs, world, slow_rank, queries):
    for qn in range(queries):
        claimed = [outs[r][qn][0] for r in range(world)]
        flat = sorted(i for c in claimed for i in c)
        assert flat == list(range(30)), "every batch claimed exactly once"
        # longest first: each rank's claims are increasing and every fast rank takes part (the slowed
        # one may start after the others took every batch of a query)
        for r, c in enumerate(claimed):
            assert c == sorted(c) and (len(c) > 0 or r == slow_rank)
        gids, glens, gtoks = outs[0][qn][2]
        assert sorted(gids) == list(range(3000))
        off = 0
        for sid, L in zip(gids, glens):
            np.testing.assert_array_equal(gtoks[off: off + L], _tokens(sid, qn))
            off += L
        assert off == len(gtoks)
        assert all(outs[r][qn][2] is None for r in range(1, world))
    # the slowed rank (20x) sheds work to the others: a weak ordering, so a loaded runner's schedule
    # cannot break it; exactly-once and the payloads above are the strict checks
    fr = {r: sum(outs[r][qn][1] for qn in range(queries)) for r in range(world)}
    fast = [fr[r] for r in range(world) if r != slow_rank]
    assert fr[slow_rank] < min(fast), fr


def test_dynamic_claims_two_ranks_one_slow():
    outs = _run(2, slow_rank=1, queries=3)
    _check(outs, 2, 1, 3)


def test_dynamic_claims_three_ranks_one_slow():
    outs = _run(3, slow_rank=0, queries=2)
    _check(outs, 3, 0, 2)


def test_batch_claim_counter_semantics():
    """BatchClaim on a local store: indices 0..n-1 once each, then None, per key."""
    import datetime
    from torch.distributed import HashStore
    st = HashStore()
    st.set_timeout(datetime.timedelta(seconds=5))
    a, b = rdist.BatchClaim(st, "k0", 3), rdist.BatchClaim(st, "k1", 1)
    assert [a(), a(), b(), a(), a(), b()] == [0, 1, 0, 2, None, None]


def test_failing_batch_releases_the_encode_gate():
    """a worker whose batch fails before its encode starts (here: entering the device
    scope raises) must still hand the device's encode gate and its turn on, so issue_batches raises
    the error instead of the device's other workers blocking on the gate forever."""
    import datetime
    import threading
    from torch.distributed import HashStore

    class _Failing(_HostSUT):
        calls = 0

        def _device_scope(self, eng, st):
            type(self).calls += 1
            if type(self).calls == 2:
                raise RuntimeError("injected device-scope failure")
            return contextlib.nullcontext()

    lengths = np.random.default_rng(6).integers(47, 501, 300).astype(np.int32)
    qsl = RNNTQSL([None] * len(lengths), lengths)
    ids, idx = rdist.query_arrays(len(lengths), 600)
    batches = make_batches(qsl, ids, idx, 100)
    st = HashStore()
    st.set_timeout(datetime.timedelta(seconds=5))
    sut = _Failing([_HostEngine(0, 0.01) for _ in range(3)], qsl)
    err = []

    def run():
        try:
            sut.issue_batches(batches, claim=rdist.BatchClaim(st, "q", len(batches)))
        except RuntimeError as e:
            err.append(e)

    t = threading.Thread(target=run, daemon=True)
    t.start()
    t.join(timeout=60)
    assert not t.is_alive(), "issue_batches hung after a failed batch (encode gate never released)"
    assert err and "injected" in str(err[0])
