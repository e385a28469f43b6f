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


def test_shard_frames_halo():
    """Each rank extracts its matched chunk plus the frame before it (the halo); the chunks tile
    frames 1..total of the sequence."""
    from coeb_front.dist import shard_frames
    for total in (1, 7, 256, 512, 513):
        for world in (1, 2, 3, 8):
            if total < world:
                continue
            matched = []
            for r in range(world):
                first, nex, nm = shard_frames(total, world, r)
                assert nex == nm + 1 and nm >= 1
                matched.extend(range(first + 1, first + nex))
            assert matched == list(range(1, total + 1))
            # deeper halos (the full GrabImageRGBD loop: 3): the counted frames are the last nm of
            # each rank's batch, every rank sees `halo` frames before its first counted one
            # (fewer at the sequence start), and the counted frames still tile 1..total
            for halo in (2, 3):
                matched = []
                for r in range(world):
                    first, nex, nm = shard_frames(total, world, r, halo=halo)
                    c0 = first + nex - nm
                    assert c0 - first == min(halo, c0)
                    matched.extend(range(c0, first + nex))
                assert matched == list(range(1, total + 1))


def test_thread_ranks_barrier_and_max():
    import threading
    from coeb_front.dist import ThreadRanks
    g = ThreadRanks(3, timeout=30)
    res = [None] * 3

    def body(r):
        v = g.view(r)
        v.barrier()
        res[r] = (v.max(r * 10.0 + 1), v.sum(1.0), v.max(-r))
    ths = [threading.Thread(target=body, args=(r,)) for r in range(3)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert res == [(21.0, 3.0, 0.0)] * 3


def _bench(args, env=None, timeout=280):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        e.pop(k, None)
    e.update(env or {})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                         timeout=timeout, cwd=ROOT, env=e)
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    return out, lines


@pytest.mark.timeout(300)
def test_bench_one_device_rehearsal_is_marked():
    """COEB_BENCH_ONE_DEVICE=1 (every rank on device 0, to rehearse --gpus N on a one-GPU box)
    labels its line, so a rehearsal is never read as an N-GPU measurement; the default batch of
    config A is 3072 matched frames per GPU in three pipelines of 1024."""
    out, lines = _bench(["--gpus", "2", "--steps", "2", "--warmup", "0", "--dry-run"], env={"COEB_BENCH_ONE_DEVICE": "1"})
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads(lines[0])
    assert rec["rehearsal_one_device"] is True and rec["n_gpus"] == 2
    assert rec["config"]["frames_per_rank"] == [3072, 3072]
    assert rec["config"]["pipelines_per_gpu"] == 3 and rec["config"]["frames_per_pipeline"] == [1024, 1024, 1024]
    out, lines = _bench(["--gpus", "2", "--steps", "2", "--warmup", "0", "--batch", "4", "--dry-run"])
    assert out.returncode == 0 and "rehearsal_one_device" not in json.loads(lines[0])


@pytest.mark.timeout(300)
def test_bench_gpus_without_torchrun():
    """`bench.py --gpus 2` started directly drives two ranks (threads, one device each): the line
    says n_gpus 2, the shards cover the whole weak-scaled sequence, the slower rank sets the time."""
    out, lines = _bench(["--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "4", "--dry-run"])
    assert out.returncode == 0, out.stderr[-2000:]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["scaling"] == "weak" and rec["config"]["ranks"] == "threads"
    assert rec["config"]["frames_per_rank"] == [4, 4] and rec["config"]["matched_frames_per_step"] == 8
    assert rec["ms_per_step"] >= 4.0       # rank 1 sleeps 4 ms per step
    assert abs(rec["value"] - 8 * 3 / (rec["ms_per_step"] * 3 / 1e3)) / rec["value"] < 1e-3


@pytest.mark.timeout(300)
def test_bench_fixed_batch_strong_scaling():
    """BASELINE configs[3]: a fixed 512-frame batch split over the GPUs (config B default)."""
    out, lines = _bench(["--gpus", "3", "--config", "B", "--steps", "2", "--warmup", "1", "--dry-run",
                         "--no-cpu-baseline"])
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 3 and rec["scaling"] == "strong"
    assert rec["config"]["frames_per_rank"] == [171, 171, 170] and sum(rec["config"]["frames_per_rank"]) == 512


def test_bench_refuses_world_mismatch():
    out, lines = _bench(["--gpus", "4", "--steps", "1", "--warmup", "0", "--batch", "2", "--dry-run"],
                        env=dict(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), timeout=120)
    assert out.returncode != 0 and not lines and "WORLD_SIZE" in out.stderr


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
    # config C runs its pipelines on one shared side stream, D a side stream each (bench.py CONFIGS)
    assert rec["config"]["side_stream"] == {"C": "shared", "D": "own"}[config]


def test_bench_side_stream_option():
    """--side-stream overrides the config's choice and the environment (set here to the opposite),
    and the line reports what ran."""
    for opt, want in (("off", "off"), ("shared", "shared"), ("own", "own")):
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--side-stream", opt, "--steps", "1", "--warmup", "0",
               "--batch", "2", "--dry-run", "--no-cpu-baseline"]
        env = dict(os.environ, COEB_SIDE_STREAM="0" if opt != "off" else "1", COEB_SIDE_SHARED="1" if opt == "own" else "0")
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
        assert out.returncode == 0, out.stderr[-2000:]
        rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
        assert rec["config"]["side_stream"] == want
