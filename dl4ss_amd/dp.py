"""Data-parallel host logic: one process per GPU, the utterance
batch sharded across ranks, the flat gradient SUM-all-reduced once per step (flat, or in
buckets), the mean's 1 / world applied inside the HIP Adam (dl4ss_adam_guarded_dp_scaled).

Kept free of HIP calls so the multi-rank behaviour is testable with the ``gloo``
backend on CPU (``tests/test_dp_cpu.py``); on the GPU box the same calls run over
RCCL (backend ``nccl``) on the device buffers.
"""
import torch
import torch.distributed as dist


def world(pg=None):
    return dist.get_world_size(pg) if dist.is_available() and dist.is_initialized() else 1


def broadcast_params_(flat, pg=None, src=0):
    """Identical initial weights on every rank (rank `src`'s)."""
    if world(pg) > 1:
        dist.broadcast(flat, src, group=pg)
    return flat


def allreduce_sum_async(t, pg=None):
    """Start the SUM all-reduce of t over ranks; returns the work handle (None without a process
    group).  On RCCL the collective runs on the group's own stream, ordered after the work
    enqueued on the current stream so far, so the caller can go on enqueueing (the next graph
    replay) and make the current stream wait later with ``work.wait()``.  The trainer applies the
    1 / world of the mean inside Adam (dl4ss_adam_guarded_dp_scaled), not as a pass over t."""
    if not (dist.is_available() and dist.is_initialized()):
        return None
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=pg, async_op=True)


def allreduce_buckets_(ext, splits, pg=None):
    """The bucketed form of one SUM all-reduce of ``ext``: ``splits`` (an index, or ascending indices)
    cut it into contiguous buckets, all-reduced asynchronously from the LAST bucket to the first (the
    order the bucketed step completes them: Linear / embedding / ADDJUST, the upper layers, then the
    lower layers with the status flag), then waited for -- elementwise the same sums as the flat
    all-reduce (tests/test_dp_cpu.py)."""
    cuts = [0] + ([int(splits)] if isinstance(splits, int) else [int(x) for x in splits]) + [ext.numel()]
    works = [allreduce_sum_async(ext[a:b], pg) for a, b in reversed(list(zip(cuts[:-1], cuts[1:])))]
    for w in works:
        if w is not None:
            w.wait()
    return ext


def max_over_ranks(value, device, pg=None):
    """Max of a host float over ranks (bench timing: the slowest rank's time)."""
    if world(pg) == 1:
        return float(value)
    t = torch.tensor([float(value)], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=pg)
    return float(t.item())
