"""Multi-GPU plumbing: one process per GPU, sharded queries, no data-path collective.

The Offline query shards embarrassingly (utterances are independent): each rank
takes batch-sized chunks of the length-sorted query round-robin (``sut.deal_batches``) and
completes its own samples.  The only collectives are control-plane: a barrier around the
timed region and max/sum reductions of the per-rank timings and counts (RCCL on GPUs, gloo
in the CPU tests).
"""
import os


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def barrier():
    d = _dist()
    if d is not None:
        d.barrier()


def _reduce(x, op):
    d = _dist()
    if d is None:
        return x
    import torch
    dev = "cuda" if d.get_backend() == "nccl" else "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    d.all_reduce(t, op=op)
    return float(t.item())


def reduce_max(x):
    import torch.distributed as dist
    return _reduce(x, dist.ReduceOp.MAX)


def reduce_sum(x):
    import torch.distributed as dist
    return _reduce(x, dist.ReduceOp.SUM)
