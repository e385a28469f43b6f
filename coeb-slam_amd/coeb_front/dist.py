"""Multi-GPU plumbing for the frame-sharded front end.

Frames are independent (a frame only needs its predecessor's keypoints, handled by a one-frame
halo per shard), so ranks never exchange data.  Two ways to run N ranks:

- `Ranks`: one process per GPU under torch.distributed.run (LOCAL_RANK selects the device);
  torch.distributed (gloo) carries only the start/stop barriers and the max-over-ranks of the
  timed interval.
- `ThreadRanks`: `bench.py --gpus N` started directly: N host threads of one process, thread r
  driving device r through its own libcoeb_front context (ctypes releases the GIL for every
  library call, so the threads issue work concurrently).  A threading.Barrier replaces gloo.

No RCCL collective on the data path in either form.
"""
import os
import threading


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


class ThreadRanks:
    """N ranks as N threads of this process (same surface as one rank's `Ranks`: call `view(r)`
    from thread r).  A rank that raises breaks the barrier, so the others fail instead of
    waiting forever."""

    def __init__(self, world, timeout=600.0):
        self.world = world
        self._bar = threading.Barrier(world, timeout=timeout)
        self._vals = [0.0] * world

    def view(self, rank):
        return _ThreadRank(self, rank)

    def abort(self):
        self._bar.abort()

    def _reduce(self, rank, x, fn):
        self._vals[rank] = float(x)
        self._bar.wait()
        r = fn(self._vals)
        self._bar.wait()          # nobody overwrites _vals before every rank has read it
        return r


class _ThreadRank:
    def __init__(self, grp, rank):
        self.grp, self.world, self.rank, self.local_rank = grp, grp.world, rank, rank

    def barrier(self):
        self.grp._bar.wait()

    def max(self, x):
        return self.grp._reduce(self.rank, x, max)

    def sum(self, x):
        return self.grp._reduce(self.rank, x, sum)

    def close(self):
        pass


def shard_frames(total, world, rank, halo=1):
    """Frames of one rank when a sequence of `total` matched frames is split over `world` ranks.

    The sequence has frames 0..total; frame 0 has no predecessor and is not counted, frame j >= 1
    is matched against frame j-1.  Rank r matches the contiguous chunk [lo+1, hi] (`shard` over
    the matched frames) and also extracts the `halo` frames before it, so every dependency is
    local: 1 for extract + match (frame lo, the LastFrame); the full GrabImageRGBD loop needs 3
    (the Frame ctor's T_M of frame lo comes from frame lo-1, and TrackLocalMap's KeyFrame f-2 of
    frame lo+1 is frame lo-1, itself built from frame lo-2).  The counted frames are the last
    nmatched of the rank's batch.  Returns (first, nextract, nmatched): the rank extracts frames
    first .. first+nextract-1."""
    if halo < 1:
        raise ValueError("halo must be >= 1")
    _, lo, hi = shard(total, world, rank)
    first = max(lo - (halo - 1), 0)
    return first, hi - first + 1, hi - lo


def shard(total, world, rank):
    """Contiguous chunk [lo, hi) of `total` frames for `rank`, plus the halo frame lo-1
    (SURVEY.md s8e): returns (halo_lo, lo, hi)."""
    per = total // world
    rem = total % world
    lo = rank * per + min(rank, rem)
    hi = lo + per + (1 if rank < rem else 0)
    return max(lo - 1, 0), lo, hi
