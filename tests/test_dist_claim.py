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
    slow = 6.0 if rank == slow_rank else 1.0
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
        # longest first: each rank's claims are increasing and every rank takes part
        for c in claimed:
            assert c == sorted(c) and len(c) > 0
        gids, glens, gtoks = outs[0][qn][2]
        assert sorted(gids) == list(range(3000))
        off = 0
        for sid, L in zip(gids, glens):
            np.testing.assert_array_equal(gtoks[off: off + L], _tokens(sid, qn))
            off += L
        assert off == len(gtoks)
        assert all(outs[r][qn][2] is None for r in range(1, world))
    # the slowed rank sheds work to the others
    fr = {r: sum(outs[r][qn][1] for qn in range(queries)) for r in range(world)}
    fast = [fr[r] for r in range(world) if r != slow_rank]
    assert fr[slow_rank] < 0.6 * min(fast), fr


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
