"""Host-side logic of the SUT/QSL mirror and of the multi-GPU path bench.py runs (CPU, gloo):
rnnt_amd.dist.shard_query deals one sorted query over the ranks, each rank completes its share,
rnnt_amd.dist.gather_responses brings every response to rank 0's host."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from rnnt_amd import dist as rdist
from rnnt_amd.sut import QuerySample, RNNTQSL, make_batches


def _qsl(lengths):
    return RNNTQSL([np.full((int(l), 240), i, np.float32) for i, l in enumerate(lengths)], lengths)


def test_sort_is_length_descending_bucket_sort():
    """rnnt_qsl.cpp:104-133: buckets by length, longest first, arrival order kept per bucket."""
    lengths = np.array([5, 9, 5, 47, 9, 1, 47], np.int32)
    qsl = _qsl(lengths)
    samples = [QuerySample(id=100 + i, index=i) for i in range(len(lengths))]
    out = qsl.sort(samples)
    assert [s.index for s in out] == [3, 6, 1, 4, 0, 2, 5]


def test_assemble_layout():
    """AssembleSamples (rnnt_qsl.cpp:150-188): [T_max, n_pad, 256], zero padded."""
    lengths = np.array([3, 7, 2], np.int32)
    qsl = _qsl(lengths)
    x, lens = qsl.assemble([1, 0, 2])
    assert x.shape == (7, 256, 256) and lens.shape == (256,)
    assert list(lens[:4]) == [7, 3, 2, 0]
    assert np.all(x[:7, 0, :240] == 1) and np.all(x[:3, 1, :240] == 0) and np.all(x[:2, 2, :240] == 2)
    assert np.all(x[3:, 1] == 0) and np.all(x[:, :, 240:] == 0) and np.all(x[:, 3:] == 0)


def test_make_batches_sorts_like_the_bucket_sort():
    lengths = np.random.default_rng(3).integers(47, 501, 777).astype(np.int32)
    qsl = RNNTQSL([None] * len(lengths), lengths)
    ids, idx = rdist.query_arrays(len(lengths), 2000)
    batches = make_batches(qsl, ids, idx, 256)
    flat = np.concatenate([b[1] for b in batches])
    ref = [s.index for s in qsl.sort([QuerySample(id=int(i), index=int(j)) for i, j in zip(ids, idx)])]
    assert list(flat) == ref
    assert all(len(b[0]) <= 256 for b in batches) and sorted(np.concatenate([b[0] for b in batches])) == list(ids)


def test_shard_query_covers_query_once():
    lengths = synthetic_lengths = np.random.default_rng(1).integers(47, 501, 2513).astype(np.int32)
    qsl = RNNTQSL([None] * len(lengths), synthetic_lengths)
    ids, idx = rdist.query_arrays(len(lengths), 24576)
    got = []
    for r in range(4):
        for b in rdist.shard_query(qsl, ids, idx, 2048, r, 4):
            assert len(b[0]) <= 2048
            got.extend(b[0])
    assert sorted(got) == list(ids)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tokens(sid):
    """a deterministic stand-in response per sample id (variable length, incl. empty)"""
    return (np.arange(sid % 7, dtype=np.int32) + sid) % 29


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    r, _, w, group = rdist.setup("gloo")
    assert (r, w) == (rank, world)
    lengths = np.random.default_rng(0).integers(47, 501, 1000).astype(np.int32)
    qsl = RNNTQSL([None] * len(lengths), lengths)
    ids, idx = rdist.query_arrays(len(lengths), 3000)
    mine = rdist.shard_query(qsl, ids, idx, 128, rank, world)
    # this rank "completes" its samples (bench.py: OfflineSUT.take_completed)
    my_ids = np.concatenate([b[0] for b in mine])
    rows = [_tokens(int(i)) for i in my_ids]
    lens = np.array([len(t) for t in rows], np.int32)
    toks = np.concatenate(rows).astype(np.int32)
    got = rdist.gather_responses(my_ids, lens, toks, world, group)
    frames = rdist.reduce_sum(int(lengths[np.concatenate([b[1] for b in mine])].sum()), group)
    slowest = rdist.reduce_max(float(rank + 1), group)
    rdist.barrier(group)
    out = None
    if got is not None:
        out = (got[0].tolist(), got[1].tolist(), got[2].tolist())
    q.put((rank, sorted(my_ids.tolist()), frames, slowest, out))
    dist.destroy_process_group()


def test_two_rank_query_shard_and_gather_gloo():
    """world_size-2 run of bench.py's multi-GPU path (rnnt_amd.dist): disjoint shards covering
    the query, every response gathered to rank 0 intact, sum/max reductions."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    outs.sort(key=lambda o: o[0])
    a, b = outs[0][1], outs[1][1]
    assert not set(a) & set(b) and sorted(a + b) == list(range(3000))
    lengths = np.random.default_rng(0).integers(47, 501, 1000)
    assert outs[0][2] == outs[1][2] == float(lengths[np.arange(3000) % 1000].sum())
    assert outs[0][3] == outs[1][3] == 2.0
    assert outs[1][4] is None
    gids, glens, gtoks = outs[0][4]
    assert sorted(gids) == list(range(3000))
    off = 0
    for sid, L in zip(gids, glens):
        np.testing.assert_array_equal(gtoks[off: off + L], _tokens(sid))
        off += L
    # snake dealing of sorted batches balances the shards' work
    fa, fb = lengths[np.array(a) % 1000].sum(), lengths[np.array(b) % 1000].sum()
    assert abs(fa - fb) / (fa + fb) < 0.1


def _stream_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import threading
    import torch.distributed as dist
    r, _, w, group = rdist.setup("gloo")
    lengths = np.random.default_rng(1).integers(47, 501, 700).astype(np.int32)
    qsl = RNNTQSL([None] * len(lengths), lengths)
    ids, idx = rdist.query_arrays(len(lengths), 2000)
    mine = rdist.shard_query(qsl, ids, idx, 96, rank, world)
    stream = rdist.ResponseStream(world, group)
    # batches complete on two "engine" threads in any order, like the OfflineSUT's workers
    halves = [mine[0::2], mine[1::2]]

    def engine(part):
        for b_ids, _ in part:
            rows = [_tokens(int(i)) for i in b_ids]
            stream.push(b_ids, np.array([len(t) for t in rows], np.int32),
                        np.concatenate(rows + [np.zeros(0, np.int32)]).astype(np.int32))

    ths = [threading.Thread(target=engine, args=(h,)) for h in halves]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    got = stream.finish()
    out = None
    if got is not None:
        out = (got[0].tolist(), got[1].tolist(), got[2].tolist())
    q.put((rank, out))
    rdist.barrier(group)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_response_stream_gloo(world):
    """dist.ResponseStream (bench.py): every rank's batches, completed on several threads, reach
    rank 0 intact in the compact wire form (ids int32, lens int16, tokens uint8)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stream_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(outs[r] is None for r in range(1, world))
    gids, glens, gtoks = outs[0]
    assert sorted(gids) == list(range(2000))
    off = 0
    for i, L in zip(gids, glens):
        np.testing.assert_array_equal(gtoks[off: off + L], _tokens(i))
        off += L
    assert off == len(gtoks)


def test_pack_responses_roundtrip_and_range():
    ids = np.array([0, 5, 2 ** 31 - 1], np.int64)
    lens = np.array([0, 3, 7500], np.int32)
    toks = np.arange(7503, dtype=np.int32) % 29
    back = rdist.unpack_responses(rdist.pack_responses(ids, lens, toks), 3, len(toks))
    for a, b in zip(back, (ids, lens, toks)):
        np.testing.assert_array_equal(a, b)
    with pytest.raises(ValueError):
        rdist.pack_responses(np.array([2 ** 31]), np.array([1]), np.array([0]))
    with pytest.raises(ValueError):
        rdist.pack_responses(np.array([1]), np.array([1]), np.array([256]))
