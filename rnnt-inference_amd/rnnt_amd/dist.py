"""Multi-GPU serving of one Offline query: one process per GPU, host-side gather.

SURVEY 8e / north_star: the query shards embarrassingly (utterances are independent).  Every
rank sorts the same query (rnnt_qsl.cpp:104-133), ``shard_query`` deals its length-sorted
batches to the ranks in snake order (every rank gets a similar mix of long and short
utterances), each rank runs its share through its own OfflineSUT, and
``gather_responses`` brings every rank's token rows to rank 0's host, where the one LoadGen
instance would complete them (the reference's single QuerySamplesComplete point,
torch_sut.cpp:221-236).  The gather runs over a gloo (host) group -- the responses are host
data after the per-batch D2H copy, so no device-side collective is involved (RCCL stays for the
control plane: barriers and timing reductions).
"""
import os

import numpy as np

from .sut import QuerySample, batch_bounds, make_batches


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def setup(device_backend="nccl"):
    """Initialise torch.distributed from the torchrun environment (world > 1) and a gloo group
    for the host-side response gather.  -> (rank, local_rank, world, gather_group)."""
    rank, local, world = env_rank()
    if world == 1:
        return rank, local, world, None
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        if device_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(device_backend)
    group = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else dist.group.WORLD
    return rank, local, world, group


def shard_query(qsl, ids, idx, batch_size, rank=0, world=1, sizes=None):
    """This rank's batches of one query: every rank sorts the same query and splits it into the
    same batches (sut.make_batches); batch i goes to rank i % world in snake order
    (0..w-1, w-1..0, ...), so every rank gets a similar mix of long and short utterances."""
    batches = make_batches(qsl, ids, idx, batch_size, sizes)
    mine = []
    for i, b in enumerate(batches):
        r = i % world if (i // world) % 2 == 0 else world - 1 - (i % world)
        if r == rank:
            mine.append(b)
    return mine


def query_arrays(count, query):
    """An Offline query of `query` samples over a QSL of `count` (LoadGen repeats the QSL):
    (sample ids, QSL indices)."""
    ids = np.arange(query, dtype=np.int64)
    return ids, ids % count


def gather_responses(ids, lens, toks, world, group=None):
    """Host-side gather of the completed responses to rank 0.  ids int64 [n], lens int32 [n],
    toks int32 [sum(lens)] (this rank's) -> on rank 0 the concatenation over ranks in rank
    order, elsewhere None.  gloo gathers of two tensors per rank (padded to the largest)."""
    if world == 1:
        return ids, lens, toks
    import torch
    import torch.distributed as dist
    rank = dist.get_rank()
    n, m = len(ids), len(toks)
    sizes = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([n, m], dtype=torch.int64), group=group)
    nmax = max(int(s[0]) for s in sizes)
    mmax = max(int(s[1]) for s in sizes)
    meta = torch.zeros((nmax, 2), dtype=torch.int64)
    meta[:n, 0] = torch.from_numpy(np.asarray(ids, np.int64))
    meta[:n, 1] = torch.from_numpy(np.asarray(lens, np.int64))
    tk = torch.zeros(max(mmax, 1), dtype=torch.int32)
    tk[:m] = torch.from_numpy(np.asarray(toks, np.int32))
    metas = [torch.zeros_like(meta) for _ in range(world)] if rank == 0 else None
    tks = [torch.zeros_like(tk) for _ in range(world)] if rank == 0 else None
    dist.gather(meta, metas, dst=0, group=group)
    dist.gather(tk, tks, dst=0, group=group)
    if rank != 0:
        return None
    out_ids, out_lens, out_toks = [], [], []
    for r in range(world):
        nr, mr = int(sizes[r][0]), int(sizes[r][1])
        out_ids.append(metas[r][:nr, 0].numpy())
        out_lens.append(metas[r][:nr, 1].numpy().astype(np.int32))
        out_toks.append(tks[r][:mr].numpy())
    return np.concatenate(out_ids), np.concatenate(out_lens), np.concatenate(out_toks)


def barrier(group=None):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier(group=group)


def reduce_max(x, group=None):
    """max over ranks of a host float (gloo group, or the default group)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return x
    dev = "cuda" if group is None and dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def reduce_sum(x, group=None):
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return x
    dev = "cuda" if group is None and dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return float(t.item())


__all__ = ["setup", "shard_query", "query_arrays", "QuerySample", "gather_responses", "barrier", "reduce_max", "reduce_sum",
           "batch_bounds", "env_rank"]
