"""Multi-GPU plumbing for the frame-sharded front end.

Frames are independent (a frame only needs its predecessor's keypoints, handled by a one-frame
halo per shard), so ranks never exchange data: torch.distributed (gloo) carries only the
start/stop barriers and the max-over-ranks of the timed interval.  One process per GPU
(LOCAL_RANK selects the device); no RCCL collective on the data path.
"""
import os


class Ranks:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if not dist.is_initialized():
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max(self, x):
        if self.dist is None:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x):
        if self.dist is None:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None


def shard(total, world, rank):
    """Contiguous chunk [lo, hi) of `total` frames for `rank`, plus the halo frame lo-1
    (SURVEY.md s8e): returns (halo_lo, lo, hi)."""
    per = total // world
    rem = total % world
    lo = rank * per + min(rank, rem)
    hi = lo + per + (1 if rank < rem else 0)
    return max(lo - 1, 0), lo, hi
