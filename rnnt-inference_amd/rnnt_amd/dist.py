"""Multi-GPU serving of one Offline query: one process per GPU, host-side gather.

SURVEY 8e / north_star: the query shards embarrassingly (utterances are independent).  Every
rank sorts the same query (rnnt_qsl.cpp:104-133) into the same length-sorted batches and pulls
them from ONE shared claim counter (``BatchClaim``: ``TCPStore.add`` on the job's rendezvous
store), the cross-process form of the reference's instances pulling the next slice from one
mutex-guarded queue (torch_sut.cpp:167-182): a rank claims a batch only when its encoder is free
(OfflineSUT's per-device encode gate), so longer batches go first and a slower GPU simply takes
fewer of them.  ``shard_query`` (a static snake deal) is kept as the alternative
(``bench.py --deal static``).  Each rank runs its batches through its own OfflineSUT, and
``ResponseStream`` (bench.py; ``gather_responses`` is the one-shot form) brings every rank's
token rows to rank 0's host as its batches complete, where the one LoadGen instance would
complete them (the reference's single QuerySamplesComplete point,
torch_sut.cpp:221-236).  The gather runs over a gloo (host) group -- the responses are host
data after the per-batch D2H copy, so no device-side collective is involved.  The control plane
(barriers, timing reductions, claims) is gloo as well by default (bench.py --control-backend;
RCCL is opt-in: nothing on the data path needs a device collective).
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


class BatchClaim:
    """Shared claim counter over one query's batches: ``claim()`` -> the next batch index not yet
    taken by any rank, or None when all are taken.  ``store.add`` is atomic on the rendezvous
    store (one TCP round trip, ~0.1 ms, against tens of ms per batch encode); every query gets its
    own key, so nothing needs resetting between queries."""

    def __init__(self, store, key, n_batches):
        self.store, self.key, self.n = store, key, int(n_batches)

    def __call__(self):
        i = int(self.store.add(self.key, 1)) - 1
        return i if i < self.n else None


def claim_for_query(qno, n_batches, store=None):
    """The BatchClaim of query number `qno` (every rank must use the same numbering) on the
    default process group's store (or `store`); None on a single process (nothing to share)."""
    import torch.distributed as dist
    if store is None:
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return None
        store = dist.distributed_c10d._get_default_store()
    return BatchClaim(store, f"rnnt_offline_claim/{int(qno)}", n_batches)


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


def pack_responses(ids, lens, toks):
    """Wire form of a batch of responses: ids int32, lens int16 (<= max_res 7500), tokens uint8
    (labels 0..28) -- 7 bytes per sample + 1 per token instead of 16 + 4."""
    ids = np.asarray(ids)
    lens = np.asarray(lens)
    toks = np.asarray(toks)
    if len(ids) and (ids.min() < 0 or ids.max() >= 2 ** 31 or lens.min() < 0 or lens.max() >= 2 ** 15):
        raise ValueError("response ids / lengths out of the wire format's range")
    if len(toks) and (toks.min() < 0 or toks.max() > 255):
        raise ValueError("token values out of the wire format's range")
    return (np.ascontiguousarray(ids, np.int32).tobytes() + np.ascontiguousarray(lens, np.int16).tobytes()
            + np.ascontiguousarray(toks, np.uint8).tobytes())


def unpack_responses(buf, n, m):
    b = np.frombuffer(buf, np.uint8)
    ids = b[: 4 * n].view(np.int32).astype(np.int64)
    lens = b[4 * n: 6 * n].view(np.int16).astype(np.int32)
    toks = b[6 * n: 6 * n + m].astype(np.int32)
    return ids, lens, toks


class ResponseStream:
    """The ranks' Offline responses streamed to rank 0 while the query runs, instead of one gather
    after it: every rank but 0 hands each completed batch (``push``, from the SUT's completion
    callback) to a sender thread that ships it over the gloo group in the compact wire form
    (``pack_responses``: header (n, m) then payload); rank 0's receiver thread takes headers from
    any source and the payload from that source.  ``finish`` sends the end marker / waits for
    every rank's, so only the responses of each rank's last batches are still in flight when the
    GPUs finish.  At 8 ranks the one-shot int32 gather moved ~7 MB per rank after the query
    (≈45-55 ms over gloo on the host); this moves ~1.7 MB per rank, mostly during the query."""

    def __init__(self, world, group=None, tag=0):
        """tag: this stream's message tag (the query number): streams of back-to-back queries
        never mix even when a fast rank's next query overtakes a slow rank's end marker."""
        import queue
        import threading
        import torch.distributed as dist
        self.world, self.group, self.tag = world, group, int(tag) & 0x7FFFFFFF
        self.rank = dist.get_rank()
        self.errors = []
        self._got = []
        self._q = queue.Queue()
        if self.rank == 0:
            self._th = threading.Thread(target=self._receive, daemon=True)
        else:
            self._th = threading.Thread(target=self._send, daemon=True)
        self._th.start()

    def push(self, ids, lens, toks):
        """A completed batch of this rank's responses (rank 0 keeps its own)."""
        if self.rank == 0:
            self._got.append((np.asarray(ids, np.int64), np.asarray(lens, np.int32), np.asarray(toks, np.int32)))
        else:
            self._q.put((ids, lens, toks))

    def _send(self):
        import torch
        import torch.distributed as dist
        try:
            while True:
                item = self._q.get()
                if item is None:
                    dist.send(torch.tensor([-1, 0], dtype=torch.int64), dst=0, group=self.group, tag=self.tag)
                    return
                buf = pack_responses(*item)
                n, m = len(item[0]), len(item[2])
                dist.send(torch.tensor([n, m], dtype=torch.int64), dst=0, group=self.group, tag=self.tag)
                dist.send(torch.frombuffer(bytearray(buf), dtype=torch.uint8), dst=0, group=self.group, tag=self.tag)
        except Exception as ex:  # surfaced by finish()
            self.errors.append(ex)

    def _receive(self):
        import torch
        import torch.distributed as dist
        try:
            ended = set()  # end markers counted per source rank, never twice from one
            while len(ended) < self.world - 1:
                hdr = torch.zeros(2, dtype=torch.int64)
                src = dist.recv(hdr, src=None, group=self.group, tag=self.tag)
                n, m = int(hdr[0]), int(hdr[1])
                if n < 0:
                    if src in ended:
                        raise RuntimeError(f"ResponseStream: second end marker from rank {src} (tag {self.tag})")
                    ended.add(src)
                    continue
                if src in ended:
                    raise RuntimeError(f"ResponseStream: data from rank {src} after its end marker (tag {self.tag})")
                buf = torch.empty(6 * n + m, dtype=torch.uint8)
                dist.recv(buf, src=src, group=self.group, tag=self.tag)
                self._got.append(unpack_responses(buf.numpy().tobytes(), n, m))
        except Exception as ex:
            self.errors.append(ex)

    def finish(self):
        """-> on rank 0 every rank's responses (ids, lens, toks) concatenated, elsewhere None."""
        if self.rank != 0:
            self._q.put(None)
        self._th.join()
        if self.errors:
            raise self.errors[0]
        if self.rank != 0:
            return None
        if not self._got:
            return np.zeros(0, np.int64), np.zeros(0, np.int32), np.zeros(0, np.int32)
        return tuple(np.concatenate([g[k] for g in self._got]) for k in range(3))


def backend_name():
    """The default group's backend ("gloo" / "nccl"), or None on a single process."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return str(dist.get_backend())
    return None


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


__all__ = ["setup", "shard_query", "BatchClaim", "claim_for_query", "query_arrays", "QuerySample", "gather_responses", "ResponseStream", "pack_responses",
           "unpack_responses", "backend_name", "barrier", "reduce_max", "reduce_sum", "batch_bounds", "env_rank"]
