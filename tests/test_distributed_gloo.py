"""Multi-rank path on the CPU (gloo, world_size 2): shard arithmetic, barrier + max-over-ranks
timing, and bench.py's rank-0 JSON line under torch.distributed.run."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_covers_all_frames():
    from coeb_front.dist import shard
    for total in (1, 7, 512, 513):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                halo, lo, hi = shard(total, world, r)
                assert halo == max(lo - 1, 0) and lo <= hi
                seen.extend(range(lo, hi))
            assert seen == list(range(total))


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, os.path.join(ROOT, "coeb-slam_amd"))
    from coeb_front.dist import Ranks
    r = Ranks()
    r.barrier()
    q.put((rank, r.max(rank * 10.0 + 1), r.sum(1.0)))
    r.close()


def test_gloo_barrier_and_max():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert [x[1] for x in res] == [11.0, 11.0] and [x[2] for x in res] == [2.0, 2.0]


@pytest.mark.timeout(300)
def test_bench_two_ranks_dry_run():
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--batch", "4", "--dry-run"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout          # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["scaling"] == "weak"
    # rank 1 sleeps 4 ms per step: the max over ranks must set the time
    assert rec["ms_per_step"] >= 4.0
    assert abs(rec["value"] - 2 * 4 * 3 / (rec["ms_per_step"] * 3 / 1e3)) / rec["value"] < 1e-3


@pytest.mark.parametrize("config", ["C", "D"])
def test_bench_config_dry_run(config):
    """The other BASELINE configs keep the bench contract (one JSON line, the config's
    workload named, whole-job frames/s)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", config, "--steps", "2", "--warmup", "1",
           "--batch", "4", "--dry-run", "--no-cpu-baseline"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    want = {"C": "configs[2]", "D": "configs[4]"}[config]
    assert want in rec["config"]["workload"] and rec["n_gpus"] == 1 and rec["unit"] == "frames/s"
    assert abs(rec["value"] - 4 * 2 / (rec["ms_per_step"] * 2 / 1e3)) / rec["value"] < 1e-3
