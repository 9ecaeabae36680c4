"""Round-robin sharding of independent values over the GPUs of one node
(SURVEY.md §8(e)): value i -> rank i mod N.  Each value is self-contained
(no cross-value codec state), so there is no data-path
collective; ranks only meet at a barrier and reduce their timings
(max) and counts (sum)."""
import torch
import torch.distributed as dist


def shard(rank, world):
    """(first, stride): this rank's k-th value is global value first + k*stride."""
    return rank, world


def global_indices(rank, world, count):
    first, stride = shard(rank, world)
    return [first + k * stride for k in range(count)]


def reduce_stats(maxes, sums, device="cpu"):
    """Max-reduce `maxes` (timings) and sum-reduce `sums` (bytes, counts)
    over the process group, if one is initialised; returns python lists."""
    tm = torch.tensor(maxes, dtype=torch.float64, device=device)
    ts = torch.tensor(sums, dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        dist.all_reduce(ts, op=dist.ReduceOp.SUM)
    return tm.tolist(), ts.tolist()


def spread_stats(values, device="cpu"):
    """(min, max) over the process group of each of `values` (one per rank):
    the per-rank imbalance bench.py reports beside the max it times by."""
    t = torch.tensor([float(v) for v in values] + [-float(v) for v in values], dtype=torch.float64,
                     device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    k = len(values)
    return [-x for x in t[k:].tolist()], t[:k].tolist()
