"""Multi-GPU plumbing for the store: one process per GPU, each owning one shard
(DESIGN.md §6).  torch.distributed is plumbing only: it hands the store's
RCCL unique id from rank 0 to every rank, and gives a barrier around the timed
region and a max-over-ranks reduction of the elapsed time.  The data path's
all-to-all runs on the store's own RCCL communicator inside libgvstore.so."""
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


def gather_ints(ri, values, device=None):
    """Every rank's list of ints (same length on every rank), rank order."""
    if ri.world == 1:
        return [list(values)]
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(v) for v in values], dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(ri.world)]
    dist.all_gather(out, t)
    return [[int(x) for x in o.cpu().tolist()] for o in out]


def broadcast_bytes(ri, data, device=None):
    """rank 0's `data` (bytes) on every rank."""
    if ri.world == 1:
        return data
    import torch
    import torch.distributed as dist
    n = torch.tensor([len(data) if ri.rank == 0 else 0], dtype=torch.int64, device=device)
    dist.broadcast(n, 0)
    buf = torch.zeros(int(n.item()), dtype=torch.uint8, device=device)
    if ri.rank == 0:
        buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    dist.broadcast(buf, 0)
    return bytes(buf.cpu().numpy().tobytes())


def finalize(ri):
    if ri.world > 1:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
