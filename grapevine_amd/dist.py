"""Multi-GPU plumbing for the store: one process per GPU, each owning an
independent shard.  torch.distributed is plumbing only: a
barrier around the timed region and a max-over-ranks reduction of the elapsed
time.  No collective is on the data path in this round."""
import os
from dataclasses import dataclass


@dataclass
class RankInfo:
    rank: int
    world: int
    local: int


def rank_info():
    return RankInfo(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                    int(os.environ.get("LOCAL_RANK", "0")))


def init(backend):
    """Initialise the process group when WORLD_SIZE > 1 (env:// rendezvous)."""
    import torch.distributed as dist
    ri = rank_info()
    if ri.world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend)
    return ri


def shard_seed(base, rank):
    """Per-shard seed: every shard serves its own independent request stream."""
    return base + 7919 * rank


def barrier(ri):
    if ri.world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(ri, value, device=None):
    """Max of a float over ranks (the slowest rank sets the job time)."""
    if ri.world == 1:
        return float(value)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(ri, value, device=None):
    if ri.world == 1:
        return int(value)
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def finalize(ri):
    if ri.world > 1:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
