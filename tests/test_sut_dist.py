"""Host-side logic of the SUT/QSL mirror and the multi-rank sharding (CPU, gloo)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from rnnt_amd.sut import QuerySample, RNNTQSL, deal_batches


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


def test_deal_batches_covers_query_once():
    samples = list(range(2513))
    world = 4
    got = []
    for r in range(world):
        for b in deal_batches(samples, 256, r, world):
            assert len(b) <= 256
            got.extend(b)
    assert sorted(got) == samples


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from rnnt_amd import dist as rdist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lengths = np.random.default_rng(0).integers(47, 501, 1000).astype(np.int32)
    qsl = RNNTQSL([None] * len(lengths), lengths)
    samples = [QuerySample(id=i, index=i) for i in range(len(lengths))]
    mine = [s.index for b in deal_batches(qsl.sort(samples), 128, rank, world) for s in b]
    total = rdist.reduce_sum(len(mine))
    frames = rdist.reduce_sum(int(lengths[mine].sum()))
    slowest = rdist.reduce_max(float(rank + 1))
    rdist.barrier()
    q.put((rank, sorted(mine), total, frames, slowest))
    dist.destroy_process_group()


def test_two_rank_sharding_gloo():
    """world_size-2 run of the multi-GPU path's control plane: disjoint shards that cover the
    query, sum/max reductions as bench.py uses them."""
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
    outs.sort()
    a, b = outs[0][1], outs[1][1]
    assert not set(a) & set(b) and sorted(a + b) == list(range(1000))
    assert outs[0][2] == outs[1][2] == 1000
    lengths = np.random.default_rng(0).integers(47, 501, 1000)
    assert outs[0][3] == int(lengths.sum())
    assert outs[0][4] == outs[1][4] == 2.0
    # round-robin dealing of sorted chunks balances the shards' work
    fa, fb = lengths[a].sum(), lengths[b].sum()
    assert abs(fa - fb) / (fa + fb) < 0.1
