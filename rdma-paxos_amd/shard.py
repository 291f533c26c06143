"""Sharding of independent consensus groups across ranks.

Groups never interact, so the path shards by group id with no data-path
exchange: rank r owns the contiguous gid range [r*G, (r+1)*G) (weak scaling,
per-rank batch fixed), and its synthetic trace is generated with
apus_gen_cfg_t.gid_base = r*G, which makes the shard byte-identical to that
slice of the unsharded batch.  The only cross-rank step is the per-batch
statistics all-reduce: MIN over APUS_STAT_MIN_WATERMARK (the global pruning
watermark) and SUM over every other statistic.  On the GPUs that
is apus_stats_allreduce (RCCL over xGMI, inside libapus_gpu); the host-side
reduction below has the same semantics over any torch.distributed backend and
is what the gloo tests and CPU-side callers use.
"""
import numpy as np

from . import abi

SUMMED = [k for k in range(abi.STAT_COUNT) if k != abi.STAT_MIN_WATERMARK]
U64_MAX = np.uint64(0xFFFFFFFFFFFFFFFF)


def gid_range(rank, groups_per_rank):
    """(gid_base, n_groups) of this rank's shard"""
    return rank * groups_per_rank, groups_per_rank


def combine(stats_list):
    """reduce a list of uint64[STAT_COUNT] vectors exactly as apus_stats_allreduce does"""
    s = np.stack([np.asarray(x, np.uint64) for x in stats_list])
    out = np.zeros(abi.STAT_COUNT, np.uint64)
    out[SUMMED] = s[:, SUMMED].sum(axis=0, dtype=np.uint64)
    out[abi.STAT_MIN_WATERMARK] = s[:, abi.STAT_MIN_WATERMARK].min()
    return out


def allreduce_stats(stats, group=None):
    """host all-reduce (torch.distributed, e.g. gloo) of one uint64 stats vector"""
    import torch
    import torch.distributed as dist
    st = np.asarray(stats, np.uint64)
    # counts fit in int64; the watermark's "none" value UINT64_MAX maps to INT64_MAX
    sums = torch.from_numpy(st[SUMMED].astype(np.int64))
    wm = st[abi.STAT_MIN_WATERMARK]
    m = torch.tensor([np.iinfo(np.int64).max if wm >= np.uint64(2 ** 63) else int(wm)], dtype=torch.int64)
    dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(m, op=dist.ReduceOp.MIN, group=group)
    out = st.copy()
    out[SUMMED] = sums.numpy().astype(np.uint64)
    out[abi.STAT_MIN_WATERMARK] = U64_MAX if int(m[0]) == np.iinfo(np.int64).max else np.uint64(int(m[0]))
    return out
