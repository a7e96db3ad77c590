"""Multi-rank path on CPU with gloo (world_size 2): bench.py's launch and
max-over-ranks timing, and world sharding = unsharded results."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module", autouse=True)
def _libs(native_lib, oracle_lib):
    pass


def test_bench_two_ranks_gloo():
    port = free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1", BB_CPU_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--exec", "cpu", "--worlds", "512", "--steps", "20", "--warmup", "2", "--cpu-seconds", "0.5", "--cpu-procs", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["total_worlds"] == 1024 and out["value"] > 0
    assert out["scaling"] == "weak" and out["steps"] == 20
    # the CPU baselines are timed at N = 1 only (the bench contract)
    assert out["cpu_baseline"] is None and out["cpu_executor"] is None
    assert out["e2e"]["value"] > 0  # the env.py loop, max over ranks


def test_bench_starts_its_own_ranks():
    """`bench.py --gpus 2` with no launcher starts two ranks itself (one
    process per device, RANK / WORLD_SIZE set by the parent) and rank 0 prints
    one line with the whole job's n_gpus."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", BB_CPU_THREADS="2")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--exec", "cpu", "--worlds", "256",
           "--steps", "10", "--warmup", "2", "--no-cpu-baseline", "--no-e2e"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["total_worlds"] == 512 and out["value"] > 0
    assert "world-sharded x2" in out["config"]["parallelism"]


def test_bench_rejects_gpus_other_than_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(free_port()))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--exec", "cpu", "--worlds", "64",
           "--steps", "2", "--warmup", "0", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode != 0 and "--gpus 3" in r.stderr and "WORLD_SIZE" in r.stderr


def _worker(rank, world, port, W, steps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.helpers import make_sim
    from madrona_basketball_amd import ExecMode
    shard = W // world
    sim = make_sim(ExecMode.CPU, shard, per_world_rng=True, world_offset=rank * shard)
    sim.step_n(steps, random_actions=True, action_seed=5)
    obs = sim.observations_tensor().to_torch().contiguous()
    gathered = [torch.empty_like(obs) for _ in range(world)]
    dist.all_gather(gathered, obs)
    if rank == 0:
        q.put(torch.cat(gathered).numpy())
    dist.destroy_process_group()


def test_sharded_ranks_equal_single_process():
    W, steps = 128, 150
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, W, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from tests.helpers import make_sim
    from madrona_basketball_amd import ExecMode
    full = make_sim(ExecMode.CPU, W, per_world_rng=True)
    full.step_n(steps, random_actions=True, action_seed=5)
    assert np.array_equal(got.view(np.uint32), full.observations_tensor().to_torch().numpy().view(np.uint32))


def _rollout_worker(rank, world, port, W, K, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.helpers import make_sim
    from madrona_basketball_amd import ExecMode
    shard = W // world
    sim = make_sim(ExecMode.CPU, shard, per_world_rng=True, world_offset=rank * shard)
    acts = sim.stage_random_actions(K, action_seed=8, step0=0)  # keyed by global world index
    buf = sim.rollout_buffers(K)
    sim.rollout(acts, buf["obs"], buf["reward"], buf["done"])
    out = []
    for key in ("obs", "reward", "done"):
        t = buf[key].transpose(0, 1).contiguous()  # worlds first for the gather
        g = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(g, t)
        out.append(torch.cat(g).transpose(0, 1).contiguous())
    if rank == 0:
        q.put([o.numpy() for o in out])
    dist.destroy_process_group()


def test_sharded_rollouts_equal_single_process():
    """World-sharded K-step rollouts (bb_rollout, no collective on the path)
    gather to the unsharded rollout's recorded outputs, bit for bit."""
    W, K = 96, 40
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_rollout_worker, args=(r, 2, port, W, K, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from tests.helpers import make_sim
    from madrona_basketball_amd import ExecMode
    full = make_sim(ExecMode.CPU, W, per_world_rng=True)
    acts = full.stage_random_actions(K, action_seed=8, step0=0)
    buf = full.rollout_buffers(K)
    full.rollout(acts, buf["obs"], buf["reward"], buf["done"])
    for g, key in zip(got, ("obs", "reward", "done")):
        assert np.array_equal(g.view(np.uint32), buf[key].numpy().view(np.uint32)), key


def _gather_worker(rank, world, port, W, steps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.helpers import make_sim
    from madrona_basketball_amd import ExecMode
    from madrona_basketball_amd.sharding import gather_observations, shard
    off, n = shard(W, rank, world)
    sim = make_sim(ExecMode.CPU, n, per_world_rng=True, world_offset=off)
    sim.step_n(steps, random_actions=True, action_seed=5)
    full = gather_observations(sim)
    one = gather_observations(sim, agent=1)
    if rank == 0:
        q.put((full.numpy().copy(), one.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_observations_two_ranks():
    """The optional observation all-gather of SURVEY 8(e) (madrona_basketball_amd.sharding):
    two shards' rows gathered == the unsharded simulator's rows, whole and per agent."""
    from tests.helpers import make_sim
    from madrona_basketball_amd import ExecMode
    W, steps, world = 256, 40, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, W, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, one = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = make_sim(ExecMode.CPU, W, per_world_rng=True)
    ref.step_n(steps, random_actions=True, action_seed=5)
    obs = ref.observations_tensor().to_torch().numpy()
    assert np.array_equal(full.view(np.uint32), obs.view(np.uint32))
    assert np.array_equal(one.view(np.uint32), obs[:, 1].copy().view(np.uint32))


def test_shard_ranges():
    from madrona_basketball_amd.sharding import shard
    assert [shard(262144, r, 8) for r in (0, 7)] == [(0, 32768), (229376, 32768)]
    with pytest.raises(ValueError):
        shard(1000, 0, 3)
