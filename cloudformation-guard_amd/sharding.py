"""Document sharding and tally reduction for N ranks.

Documents shard with no data-path exchange: rank r owns templates [r*D, (r+1)*D) (weak scaling,
D per GPU).  The only collective is the all-reduce of the per-(rules file, rule) PASS/FAIL/SKIP/
error tallies that rule_count_kernel writes (layout in include/cfn_guard_mi355x.h).
"""

STATUSES = ("PASS", "FAIL", "SKIP", "ERROR")


def shard_range(rank, world, docs_per_rank):
    """Templates owned by `rank` under weak scaling."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return rank * docs_per_rank, docs_per_rank


def tally_index(file, rule, status, max_top):
    """Index into the tally vector: ((file * (max_top + 1) + rule) * 4) + status.
    rule == max_top is the file-level line (file status, errored tiles in status 3)."""
    return (file * (max_top + 1) + rule) * 4 + status


def tally_size(nfiles, max_top):
    return nfiles * (max_top + 1) * 4


def all_reduce_tallies(tensor, dist):
    """Sum the tally tensor across ranks (RCCL on GPU ranks, gloo in the CPU tests)."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(tensor)
    return tensor
