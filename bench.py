"""Throughput benchmark of the MI355X basketball step (BASELINE.json metric).

python bench.py [--gpus N] [--steps K] [--warmup W] [--worlds 65536] [--agents 2]
Multi-GPU: python bench.py --gpus N starts N ranks itself (one process per
GPU); under a launcher (python -m torch.distributed.run --nproc-per-node N ...
bench.py --gpus N) --gpus must equal WORLD_SIZE.

A "step" = one step of every world on this GPU, reading that step's
synthetic random actions (the stand-in for the Python `actions[:] = ...` of
scripts/env.py:147), which are generated on-device and resident in HBM before
the timed region starts ([steps, W, N, 6] int32).  Worlds are sharded across
ranks (weak scaling: --worlds per GPU); there is no collective on the step
path, only a barrier and a max-reduce of the elapsed time around the timed
region.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env steps/sec (whole node) at 65 536 worlds; 1→8 GPU scaling"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
EVENT_MIN_LAUNCHES = 200  # kernel-time averages over at least this many launches


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _cpu_worker(job):
    """One process of the CPU baseline: the oracle (a single-threaded C
    restatement of the reference's CPU executor) stepping its own worlds."""
    num_agents, seconds, worlds = job
    from oracle.oracle import Oracle
    from oracle import oracle as O
    o = Oracle(worlds, num_agents=num_agents, flags=O.FLAG_PER_WORLD_RNG)
    o.run_random(5, 321, 0)  # warm
    steps, elapsed = 0, 0.0
    while elapsed < seconds:
        elapsed += o.run_random(10, 321, 5 + steps)
        steps += 10
    return worlds, steps, elapsed


def cpu_model() -> str:
    """The host CPU's model name and thread count (SURVEY §8(d) asks for both)."""
    try:
        with open("/proc/cpuinfo") as f:
            names = [l.split(":", 1)[1].strip() for l in f if l.startswith("model name")]
        return f"{names[0]} ({len(names)} threads visible)" if names else "unknown"
    except OSError:
        return "unknown"


def cpu_baseline(num_agents: int, seconds: float, procs: int):
    """The oracle on `procs` host cores (one process each, spawned before this
    process touches the GPU), each on a bounded sample of the same workload;
    the rates of the concurrent processes add up."""
    worlds = 2048
    if procs <= 1:
        res = [_cpu_worker((num_agents, seconds, worlds))]
    else:
        import multiprocessing as mp
        with mp.get_context("spawn").Pool(procs) as pool:
            res = pool.map(_cpu_worker, [(num_agents, seconds, worlds)] * procs)
    value = sum(w * st / el for w, st, el in res)
    steps = min(st for _, st, _ in res)
    return {"value": value, "unit": "env-steps/s", "cores": procs, "kind": "port", "cpu_model": cpu_model(),
            "sample": f"{procs} process(es) x {worlds} worlds x >= {steps} steps each, {num_agents} agents, "
                      f"threefry random actions, ~{seconds:.0f} s per process, rates summed"}


def _executor_worker(job):
    """The product's own CPU executor (ExecMode.CPU, bb_host.hip: `threads`
    std::threads over contiguous world ranges) on the same workload."""
    num_agents, seconds, worlds, threads = job
    os.environ["BB_CPU_THREADS"] = str(threads)
    import madrona_basketball_amd as mba
    sim = mba.SimpleGridworldSimulator(
        discrete_x=32, discrete_y=17, start_x=31.515 / 2.0, start_y=16.764000000000003 / 2.0,
        max_episode_length=39600, exec_mode=mba.ExecMode.CPU, num_worlds=worlds, gpu_id=-1,
        num_agents=num_agents, per_world_rng=True)
    sim.step_n(3, random_actions=True, action_seed=321, step0=0)  # warm
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        sim.step_n(5, random_actions=True, action_seed=321, step0=3 + steps)
        steps += 5
    return worlds, steps, time.perf_counter() - t0


def cpu_executor_baseline(num_agents: int, seconds: float, threads: int):
    """The product's CPU executor in a child process (spawned before this
    process touches the GPU)."""
    import multiprocessing as mp
    worlds = 2048 * max(1, threads)  # the oracle leg's total sample
    with mp.get_context("spawn").Pool(1) as pool:
        w, st, el = pool.apply(_executor_worker, ((num_agents, seconds, worlds, threads),))
    return {"value": w * st / el, "unit": "env-steps/s", "cores": threads, "kind": "product host executor",
            "sample": f"{w} worlds x {st} steps on {threads} threads, {num_agents} agents, threefry random actions"}


def load_traffic(workload_key: str):
    """HBM bytes per step-kernel launch from the committed PMC passes
    (tools/traffic.py; FETCH_SIZE x2 + WRITE_SIZE), or None."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(workload_key)
        return None if e is None else e["bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        return None


def launch_ranks(n: int) -> int:
    """`--gpus N` (N > 1) without a launcher: start N ranks of this same
    command as child processes, one per GPU (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* in their environment, as torch.distributed.run would set them).
    This parent never imports torch, so it never touches a GPU; it waits for
    the ranks, stops the others if one fails, and returns the first failing
    rank's exit status (0 when all succeed).  Rank 0 prints the JSON line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                log(f"bench.py: rank {procs.index(p)} exited with status {code}; stopping the other ranks")
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--worlds", type=int, default=65536, help="worlds per GPU")
    ap.add_argument("--agents", type=int, default=2)
    ap.add_argument("--seed", type=int, default=321)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=min(16, os.cpu_count() or 1),
                    help="host processes for the CPU baseline (the GPU box's share is 16 cores)")
    ap.add_argument("--rollout", type=int, default=0,
                    help="K > 0: bb_rollout of K steps per call (observations / rewards / dones recorded "
                         "into [K, W, N, ...] buffers; one k_rollout launch at 2 agents); 0: one step per call")
    ap.add_argument("--policy", action="store_true",
                    help="every step: the fused policy (reference Agent, random init) acts for every agent "
                         "into the action tensor, then the step (env.py + ppo.py's inference, on the device)")
    ap.add_argument("--no-record", action="store_true",
                    help="diagnostics: rollouts without recorded outputs (each step rewrites the sim's own tensors)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the end-to-end leg (env.py's step through Python: slice write, step, 3 clones)")
    ap.add_argument("--no-configs", "--no-beyond-cache", dest="no_configs", action="store_true",
                    help="skip the lines of the other BASELINE configs (262144 x 2 beyond the Infinity Cache, "
                         "8192 x 2 per step and K=32, the 32768 x 2 shard, 65536 x 4, 65536 x 10) reported "
                         "beside the 65536-world headline")
    ap.add_argument("--dist", action="store_true",
                    help="start the process group (RCCL on the GPU) even at world size 1: exercises the "
                         "multi-rank barrier / max-reduce path on one device")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend on the GPU (nccl = RCCL; gloo only to rehearse the "
                         "multi-rank path with several ranks sharing one GPU)")
    ap.add_argument("--exec", choices=["cuda", "cpu"], default="cuda",
                    help="cpu = host executor + gloo (tests of the multi-rank path)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(launch_ranks(args.gpus))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if world_size != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world_size} rank(s) "
                         "(WORLD_SIZE); they must agree")
    rank = int(os.environ.get("RANK", "0"))
    cpu = cpu_exec = None
    # the CPU baselines: rank 0 at N = 1 only, before any GPU call
    if rank == 0 and world_size == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.agents, args.cpu_seconds, args.cpu_procs)
        cpu_exec = cpu_executor_baseline(args.agents, min(args.cpu_seconds, 8.0), args.cpu_procs)

    import torch
    import torch.distributed as dist

    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    on_gpu = args.exec == "cuda"
    if on_gpu:
        # (ranks beyond the node's GPUs share them round-robin: a rehearsal of
        # the multi-rank path on a smaller box, with --dist-backend gloo)
        torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()) if world_size > 1 else 0)
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    use_dist = world_size > 1 or args.dist
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        if on_gpu:
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world_size)
            else:
                dist.init_process_group("gloo", rank=rank, world_size=world_size)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world_size)

    import madrona_basketball_amd as mba
    from madrona_basketball_amd import _lib
    fused = bool(_lib.load().bb_rollout_fused(args.agents)) if on_gpu else False

    W = args.worlds
    sim = mba.SimpleGridworldSimulator(
        discrete_x=32, discrete_y=17, start_x=31.515 / 2.0, start_y=16.764000000000003 / 2.0,
        max_episode_length=39600, exec_mode=mba.ExecMode.CUDA if on_gpu else mba.ExecMode.CPU,
        num_worlds=W, gpu_id=dev.index if on_gpu else -1,
        num_agents=args.agents, per_world_rng=True, world_offset=rank * W)

    def sync():
        if on_gpu:
            torch.cuda.synchronize(dev)

    def barrier():
        sync()
        if use_dist:
            dist.barrier()
        sync()

    def max_over_ranks(x: float) -> float:
        if not use_dist:
            return x
        gloo = not on_gpu or args.dist_backend == "gloo"
        t = torch.tensor([x], dtype=torch.float64, device="cpu" if gloo else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # synthetic inputs resident in HBM before the timed region: the random
    # action rows of every step, [steps, W, N, 6] int32 (3.1 GB at 1000 x 65 536 x 2)
    # warmup (untimed), through the launch the timed region makes: the staged
    # steps' kernel (the resident loop at 2 agents) is first launched here, so
    # its code-object load and scratch allocation stay out of the timed region
    if not args.rollout and not args.policy and args.warmup >= 2:
        warm = sim.stage_random_actions(args.warmup, action_seed=args.seed, step0=0)
        sim.step_n_staged(warm)
        del warm
    else:
        sim.step_n(args.warmup, random_actions=True, action_seed=args.seed, step0=0)
    staged = sim.stage_random_actions(args.steps, action_seed=args.seed, step0=args.warmup)
    barrier()

    K = args.rollout
    if K:
        if args.steps % K:
            raise SystemExit("--steps must be a multiple of --rollout")
        bufs = None if args.policy else sim.rollout_buffers(K)  # reused by every chunk, like PPO's storage

    if args.policy:
        from madrona_basketball_amd.policy import FusedPolicy, make_agent
        pol = FusedPolicy.from_agent(make_agent(0).to(dev))
        lp = torch.empty((W,), dtype=torch.float32, device=dev)
        val = torch.empty((W,), dtype=torch.float32, device=dev)
        if K:  # PPO's rollout storage (scripts/buffers.py), reused by every chunk
            pbufs = pol.rollout_buffers(sim, K)

    def run(actions, time_kernels=False, steps=None):
        """All staged steps: one step per launch, or chunks of K via bb_rollout."""
        steps = args.steps if steps is None else steps
        if args.policy and K:  # PPO's rollout on the device (bb_rollout_policy), K steps per call
            ms = 0.0
            for i in range(0, steps, K):
                ms += pol.rollout(sim, K, pbufs, trainee=0, stochastic=True, seed=args.seed, step0=i,
                                  time_kernels=time_kernels) or 0.0
            return ms
        if args.policy:  # actions come from the policy, not the staged rows
            for t in range(steps):
                for a in range(args.agents):
                    pol.act(sim, a, lp, val, stochastic=True, seed=args.seed, step=t)
                sim.step()
            return None
        if not K:
            return sim.step_n_staged(actions, time_kernels=time_kernels)
        ms = 0.0
        for i in range(0, steps, K):
            if args.no_record:
                r = sim.rollout(actions[i:i + K], time_kernels=time_kernels)
            else:
                r = sim.rollout(actions[i:i + K], bufs["obs"], bufs["reward"], bufs["done"],
                                time_kernels=time_kernels)
            ms += r or 0.0
        return ms

    # timed region: exactly K steps, step k reading staged[k] (scripts/run.py:10-15)
    t0 = time.perf_counter()
    run(staged)
    sync()
    elapsed = time.perf_counter() - t0
    barrier()
    elapsed = max_over_ranks(elapsed)

    # the drop-in path's own timed region: the same number of steps, each one
    # launch of the kernel SimpleGridworldSimulator.step() issues (k_step,
    # scripts/env.py:155 inside scripts/run.py:10-15's loop), reading its
    # staged action rows; bit-identical results to the headline's launch
    per_call_s = None
    if on_gpu and not K and not args.policy:
        del staged
        staged = sim.stage_random_actions(args.steps, action_seed=args.seed, step0=args.warmup + args.steps)
        with _lib.diag(step_loop=0):
            sim.step_n_staged(staged[:1].clone())  # (untimed: the kernel's first launch)
            barrier()
            t0 = time.perf_counter()
            run(staged)
            sync()
            per_call_s = time.perf_counter() - t0
            barrier()
        per_call_s = max_over_ranks(per_call_s)

    # kernel timing: the step kernel's own start/end (hipExtLaunchKernel
    # events on the launch stream) over the same workload, re-staged; at
    # least EVENT_MIN_LAUNCHES launches whatever --steps is, so the line's
    # frac is an average as long as the committed rocprof summaries'
    del staged
    L = _lib.load()
    staged_path = int(L.bb_step_staged_path(sim._h, max(args.steps, EVENT_MIN_LAUNCHES)))
    loop_main = on_gpu and not K and not args.policy and staged_path != 0
    if on_gpu and (not args.policy or K):
        per_launch = K if (K and (fused or args.policy)) else 1
        ev_steps = max(args.steps, EVENT_MIN_LAUNCHES * per_launch)
        if K:
            ev_steps = (ev_steps + K - 1) // K * K
        staged = sim.stage_random_actions(ev_steps, action_seed=args.seed, step0=args.warmup + args.steps)
        barrier()
        kernel_ms = run(staged, time_kernels=True, steps=ev_steps)
        barrier()
        launches = ev_steps // per_launch
        avg_kernel_s = max_over_ranks(kernel_ms / 1e3 / launches)
        del staged
        one_launch_s = reload_s = None
        if loop_main:  # the same workload as one k_step launch per step (bb_diag_step_loop)
            staged = sim.stage_random_actions(ev_steps, action_seed=args.seed, step0=args.warmup + args.steps + ev_steps)
            L.bb_diag_step_loop(0)
            barrier()
            one_launch_s = max_over_ranks(run(staged, time_kernels=True, steps=ev_steps) / 1e3 / ev_steps)
            barrier()
            L.bb_diag_step_loop(-1)
            del staged
            if staged_path == 2:  # and as the k_step_loop launch that reloads the state every step
                staged = sim.stage_random_actions(ev_steps, action_seed=args.seed,
                                                  step0=args.warmup + args.steps + 2 * ev_steps)
                L.bb_diag_step_loop(1)
                barrier()
                reload_s = max_over_ranks(run(staged, time_kernels=True, steps=ev_steps) / 1e3 / ev_steps)
                barrier()
                L.bb_diag_step_loop(-1)
                del staged
    else:
        launches = args.steps // K if (K and fused) else args.steps
        ev_steps = args.steps
        avg_kernel_s = elapsed / launches

    # end-to-end leg (scripts/run.py:10-15 over scripts/env.py:147,167-170):
    # per step the trainee's int64 action rows are written into the action
    # tensor by a torch slice assignment, SimpleGridworldSimulator.step() is
    # called from Python, and obs / reward / done of the trainee are cloned
    e2e = None
    if not args.no_e2e and not args.policy and not K:
        import torch
        views = {k: getattr(sim, k)().to_torch() for k in
                 ("action_tensor", "observations_tensor", "reward_tensor", "done_tensor")}
        trainee = sim.stage_random_actions(args.steps, action_seed=args.seed,
                                           step0=args.warmup + 2 * args.steps)[:, :, 0].to(torch.int64)
        acts, obs_t, rew_t, done_t = (views[k] for k in ("action_tensor", "observations_tensor",
                                                          "reward_tensor", "done_tensor"))
        barrier()
        t0 = time.perf_counter()
        for t in range(args.steps):
            acts[:, 0] = trainee[t]
            sim.step()
            obs_t[:, 0].detach().clone()
            rew_t[:, 0].detach().clone()
            done_t[:, 0].detach().clone()
        sync()
        e2e_s = time.perf_counter() - t0
        barrier()
        e2e_s = max_over_ranks(e2e_s)
        del trainee
        # the same loop with SimpleGridworldSimulator.step() alone (Python + ctypes
        # + the launch, no torch kernels): the per-call cost of the binding
        barrier()
        t0 = time.perf_counter()
        for t in range(args.steps):
            sim.step()
        sync()
        step_only_s = max_over_ranks(time.perf_counter() - t0)
        e2e = {"value": W * world_size * args.steps / e2e_s, "unit": "env-steps/s",
               "ms_per_step": e2e_s * 1e3 / args.steps,
               "step_call_only_us": step_only_s * 1e6 / args.steps,
               "harness": "scripts/run.py loop over env.step(): int64 trainee actions -> actions[:, 0] "
                          "(env.py:147), SimpleGridworldSimulator.step() via ctypes, obs/reward/done "
                          "[:, 0].clone() (env.py:167-170); agent 1 acts through the hard-coded defence"}

    # beside the headline, every other BASELINE.json config as its own line:
    # the same step at 262 144 worlds (1664 B of state and rows per world:
    # 436 MB, beyond the 256 MiB Infinity Cache, where PMC traffic is HBM
    # traffic), the C2 training batch (8 192 x 2, per step and as PPO's
    # 32-step rollouts), the C4 per-GPU shard (32 768 x 2) and the "2v2" /
    # "5v5" extensions (65 536 x 4 / x 10); each events-timed over
    # >= EVENT_MIN_LAUNCHES launches like the headline kernel
    extra = {}
    if (on_gpu and not args.no_configs and not args.policy and not K
            and W == 65536 and args.agents == 2):
        L0 = _lib.load()

        def config_line(W2, n2, K2=0, launches=EVENT_MIN_LAUNCHES):
            """W2 worlds per rank (world_offset = rank * W2); wall time and
            kernel time are the maxima over ranks, value = all ranks' worlds."""
            steps2 = launches * (K2 or 1)
            sim2 = mba.SimpleGridworldSimulator(
                discrete_x=32, discrete_y=17, start_x=31.515 / 2.0, start_y=16.764000000000003 / 2.0,
                max_episode_length=39600, exec_mode=mba.ExecMode.CUDA, num_worlds=W2, gpu_id=dev.index,
                num_agents=n2, per_world_rng=True, world_offset=rank * W2)
            if K2:
                sim2.step_n(20, random_actions=True, action_seed=args.seed, step0=0)
            else:  # warmed up through the staged launch itself (as the headline)
                sim2.step_n_staged(sim2.stage_random_actions(20, action_seed=args.seed, step0=0))
            bufs2 = sim2.rollout_buffers(K2) if K2 else None
            if K2:  # one untimed rollout: the rollout kernel's first launch outside the timed region
                w2 = sim2.stage_random_actions(K2, action_seed=args.seed, step0=0)
                sim2.rollout(w2, bufs2["obs"], bufs2["reward"], bufs2["done"])
                del w2

            def go(acts, timed):
                if not K2:
                    return sim2.step_n_staged(acts, time_kernels=timed)
                ms = 0.0
                for i in range(0, steps2, K2):
                    ms += sim2.rollout(acts[i:i + K2], bufs2["obs"], bufs2["reward"], bufs2["done"],
                                       time_kernels=timed) or 0.0
                return ms
            acts2 = sim2.stage_random_actions(steps2, action_seed=args.seed, step0=20)
            barrier()
            t0 = time.perf_counter()
            go(acts2, False)
            sync()
            wall2 = time.perf_counter() - t0
            barrier()
            wall2 = max_over_ranks(wall2)
            acts2 = sim2.stage_random_actions(steps2, action_seed=args.seed, step0=20 + steps2)
            barrier()
            k2 = max_over_ranks(go(acts2, True) / 1e3 / launches)
            barrier()
            path2 = int(L0.bb_step_staged_path(sim2._h, steps2)) if not K2 else 0
            loop2 = path2 != 0
            k1 = None
            if loop2:  # the same steps as one k_step launch each (bb_diag_step_loop)
                acts2 = sim2.stage_random_actions(steps2, action_seed=args.seed, step0=20 + 2 * steps2)
                L0.bb_diag_step_loop(0)
                barrier()
                k1 = max_over_ranks(go(acts2, True) / 1e3 / launches)
                barrier()
                L0.bb_diag_step_loop(-1)
            fused2 = bool(L0.bb_rollout_fused(n2)) and K2 > 0
            if fused2:
                # + at N = 2 the last step's rows into the sim's own tensor (recorded)
                b2 = W2 * (K2 * L0.bb_rollout_bytes_per_world_step(n2) + L0.bb_rollout_state_bytes_per_world(n2)
                           + (L0.bb_rollout_bytes_per_world_step(n2) - 32 * n2 if n2 == 2 else 0))
            elif loop2:  # per step, of the one launch's bytes (the resident loop reads the state once)
                b2 = L0.bb_step_staged_bytes(sim2._h, steps2) / steps2
            else:
                b2 = L0.bb_algorithmic_bytes_per_world(n2) * W2 * (K2 or 1)
            b1 = L0.bb_algorithmic_bytes_per_world(n2) * W2  # one k_step launch
            key = f"W{W2}_N{n2}" + (f"_R{K2}" if K2 else "")
            line = {"worlds": W2 * world_size, "worlds_per_gpu": W2, "n_gpus": world_size, "agents": n2,
                    "steps": steps2, "value": W2 * world_size * steps2 / wall2, "unit": "env-steps/s",
                    "ms_per_step": wall2 * 1e3 / steps2,
                    "kernel": _lib.kernel_name(sim2._h, 2 if K2 else 1, K2 or steps2),
                    "launches_timed": 1 if loop2 else launches, "kernel_avg_us": k2 * 1e6,
                    "kernel_us_per_step": k2 * 1e6 / (K2 or 1), "achieved": b2 / k2 / 1e9,
                    "frac": b2 / k2 / 1e9 / HBM_PEAK_GBS, "traffic": load_traffic(key),
                    "algorithmic_bytes_per_launch": b2}
            if K2:
                line["rollout"] = K2
            if loop2:
                line["steps_per_launch"] = steps2
                line["kernel_avg_us_note"] = "per step: the one launch's events / its steps"
                if path2 == 2:
                    line["algorithmic_bytes_note"] = ("resident loop: per step B(N) less the state reads "
                                                      "(made once per launch), bb_step_staged_bytes / steps")
                line["one_launch_per_step"] = {"kernel": "bb::k_step<%d>" % n2, "launches_timed": launches,
                                               "kernel_avg_us": k1 * 1e6, "frac": b1 / k1 / 1e9 / HBM_PEAK_GBS}
            del sim2, acts2, bufs2
            torch.cuda.empty_cache()
            return line

        def ppo_line(W2, K2=32, rollouts=10):
            """PPO's rollout loop on the device (bb_rollout_policy): K2 x (policy on
            agent 0's rows, step, buffer stores) + the next-value pass."""
            from madrona_basketball_amd.policy import FusedPolicy, make_agent
            sim2 = mba.SimpleGridworldSimulator(
                discrete_x=32, discrete_y=17, start_x=31.515 / 2.0, start_y=16.764000000000003 / 2.0,
                max_episode_length=39600, exec_mode=mba.ExecMode.CUDA, num_worlds=W2, gpu_id=dev.index,
                num_agents=2, per_world_rng=True)
            pol2 = FusedPolicy.from_agent(make_agent(0).to(dev))
            b2 = pol2.rollout_buffers(sim2, K2)
            for i in range(2):
                pol2.rollout(sim2, K2, b2, seed=args.seed, step0=i * K2)
            sync()
            t0 = time.perf_counter()
            for i in range(rollouts):
                pol2.rollout(sim2, K2, b2, seed=args.seed, step0=(2 + i) * K2)
            sync()
            wall2 = time.perf_counter() - t0
            ev = sum(pol2.rollout(sim2, K2, b2, seed=args.seed, step0=(2 + rollouts + i) * K2, time_kernels=True)
                     for i in range(rollouts)) / rollouts
            # algorithmic bytes per PPO step of the path this call takes
            # (bb_rollout_policy_bytes): what that loop as built
            # must move per call of K2 steps with every record, over K2
            path = int(L0.bb_rollout_policy_path(sim2._h, 0, 0))
            step_bytes = W2 * int(L0.bb_rollout_policy_bytes(sim2._h, 0, 0, K2)) / K2
            us_step = ev * 1e3 / K2
            line = {"worlds": W2, "agents": 2, "rollout": K2, "rollouts": rollouts,
                    "value": W2 * K2 * rollouts / wall2, "unit": "env-steps/s",
                    "us_per_step": wall2 * 1e6 / (K2 * rollouts), "rollout_avg_us_events": ev * 1e3,
                    "path": {1: "k_rollout_policy (one launch per rollout)",
                             2: "k_rollout_ppo: the first policy pass, then K x (the step + the next policy "
                                "pass), one launch (k_policy + one k_step_ppo per step with the "
                                "ppo_step_loop path override = 0)",
                             3: "k_policy + k_step per step"}.get(path, str(path)),
                    "roofline": {"bound": "hbm", "scope": "whole PPO step (policy pass + world step + records)",
                                 "algorithmic_bytes_per_step": step_bytes,
                                 "achieved": step_bytes / us_step / 1e3, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": step_bytes / us_step / 1e3 / HBM_PEAK_GBS,
                                 "mfma_flops_per_step": W2 * 2 * (128 * 32 + 32 * 32 + 32 * 20),
                                 "traffic": load_traffic(f"W{W2}_PPO_R{K2}")},
                    "what": "bb_rollout_policy: per step the fused policy acts for agent 0 of every world, the "
                            "step, obs/actions/log-probs/values/rewards/dones recorded ([K, W, ...]); then the "
                            "next-value pass (scripts/ppo.py:61-141)"}
            del sim2, pol2, b2
            torch.cuda.empty_cache()
            return line

        if world_size == 1:
            extra["roofline_beyond_cache"] = config_line(262144, 2)
            extra["config_c2_8192x2"] = config_line(8192, 2)
            extra["config_c2_8192x2_rollout32"] = config_line(8192, 2, 32, launches=EVENT_MIN_LAUNCHES // 4)
            extra["config_c4_shard_32768x2"] = config_line(32768, 2)
            extra["config_2v2_65536x4"] = config_line(65536, 4)
            # the "2v2" configuration as K = 32 rollouts (one k_rollout_shared
            # launch per 32 steps; 8 launches: the staged actions are 6 MB a step)
            extra["config_2v2_65536x4_rollout32"] = config_line(65536, 4, 32, launches=8)
            extra["config_c5_65536x10"] = config_line(65536, 10)
            extra["ppo_rollout32_8192x2"] = ppo_line(8192)
            extra["ppo_rollout32_65536x2"] = ppo_line(65536)
        else:
            # BASELINE configs[3] as stated: 32 768 worlds per GPU, all ranks
            # stepping their shard together (262 144 worlds at 8 GPUs)
            extra["config_c4_32768_per_gpu"] = config_line(32768, 2)

    total_worlds = W * world_size
    value = total_worlds * args.steps / elapsed
    if K and fused:
        # per launch: the state once in and out, and per step only the action
        # rows in and the recorded rows (obs, reward, done) out;
        # recorded, the last step's rows also into the sim's own tensor
        mirror = (0 if args.no_record or args.agents != 2
                  else L.bb_rollout_bytes_per_world_step(args.agents) - 32 * args.agents)
        bytes_per_launch = W * (K * L.bb_rollout_bytes_per_world_step(args.agents)
                                + L.bb_rollout_state_bytes_per_world(args.agents) + mirror)
    elif loop_main:  # per step, of the one launch's bytes
        bytes_per_launch = L.bb_step_staged_bytes(sim._h, ev_steps) / ev_steps
    else:
        bytes_per_launch = L.bb_algorithmic_bytes_per_world(args.agents) * W
    achieved_gbs = bytes_per_launch / avg_kernel_s / 1e9
    workload_key = f"W{W}_N{args.agents}" + (f"_R{K}" if K else "")
    traffic = load_traffic(workload_key)

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world_size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": f"{W} worlds per GPU x {args.agents} agents ("
                        + ("reference 1v1 game, NUM_AGENTS=2" if args.agents == 2 else
                           f"extension: the reference game rules with NUM_AGENTS={args.agents}, obs row "
                           f"{L.bb_obs_width(args.agents)} floats") + "), threefry random actions per step (buckets "
                        f"[2,8,3,2,2,2]) staged in HBM before the timed region, per-world RNG"
                        + (f"; rollouts of {K} steps per call (bb_rollout), observations/rewards/dones "
                           f"of every step recorded into [{K}, W, N, ...] buffers" if K and not args.policy
                           else ("" if K else (("; the timed steps in one bb_step_n_staged call = one "
                                                + ("k_step_loop launch (each wave steps its worlds once per "
                                                   "staged step" if staged_path == 1 else
                                                   "resident-loop launch (the worlds in registers between "
                                                   "steps, every step's state columns, rows, rewards and done "
                                                   "flags stored")
                                                + "; bit-identical to one k_step launch per step, the "
                                                "one_launch_per_step object)") if loop_main
                                               else "; one k_step launch per step")))
                        + ((f"; PPO's rollout on the device (bb_rollout_policy: per step the fused policy "
                            f"-- reference Agent layout, random init, categorical sampling -- acts for agent 0, the "
                            f"step, and obs/actions/log-probs/values/rewards/dones recorded into [{K}, W, ...] "
                            f"buffers; agent 1 by the in-sim defence AI; the staged random rows are unused)"
                            if K else "; actions from the fused policy (reference Agent layout, random init, "
                            "categorical sampling) for every agent before each step") if args.policy else ""),
            "worlds_per_gpu": W,
            "total_worlds": total_worlds,
            "agents_per_world": args.agents,
            "parallelism": f"world-sharded x{world_size}, no collectives on the step path",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved_gbs / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel": _lib.kernel_name(sim._h, 2 if K else (1 if loop_main else 0), K or ev_steps),
            "kernel_avg_us": avg_kernel_s * 1e6,
            "algorithmic_bytes_per_launch": bytes_per_launch,
        },
    }
    if loop_main and on_gpu:
        # kernel_avg_us (and achieved / frac) are per step: one k_step_loop
        # launch's events over its steps (rocprof shows the launch: x steps)
        out["roofline"]["algorithmic_bytes_per_step"] = bytes_per_launch
        out["roofline"]["steps_per_launch"] = ev_steps
        b1 = L.bb_algorithmic_bytes_per_world(args.agents) * W  # one k_step launch
        out["roofline"]["one_launch_per_step"] = {
            "kernel": "bb::k_step<%d>" % args.agents, "kernel_avg_us": one_launch_s * 1e6,
            "achieved": b1 / one_launch_s / 1e9,
            "frac": b1 / one_launch_s / 1e9 / HBM_PEAK_GBS}
        if reload_s is not None:
            out["roofline"]["algorithmic_bytes_note"] = (
                "resident loop: per step B(N) less the state reads, which it makes once per launch "
                "(bb_step_staged_bytes / steps); every step's state columns, rows, rewards, done flags "
                "and action write-backs are stored")
            out["roofline"]["state_reload_loop"] = {
                "kernel": "bb::k_step_loop<%d>" % args.agents, "kernel_avg_us": reload_s * 1e6,
                "achieved": b1 / reload_s / 1e9, "frac": b1 / reload_s / 1e9 / HBM_PEAK_GBS,
                "what": "the same steps with every state column reloaded each step (k_step_loop, step_loop path "
                        "override = 1)"}
    if not on_gpu:
        out["roofline"] = None
        out["config"]["parallelism"] += " (host executor, gloo)"
    if args.policy:
        out["roofline"] = None  # several kernels per step: see the rocprof summary
        if K and on_gpu:
            out["policy_rollout"] = {"rollout_avg_us": avg_kernel_s * 1e6, "us_per_step": avg_kernel_s * 1e6 / K,
                                     "rollouts_timed": launches,
                                     "timing": "events around each bb_rollout_policy call (its K policy passes, "
                                               "K steps and the next-value pass)"}
    if per_call_s is not None:
        pc = {"value": total_worlds * args.steps / per_call_s, "unit": "env-steps/s",
              "ms_per_step": per_call_s * 1e3 / args.steps, "kernel": "bb::k_step<%d>" % args.agents,
              "what": "the per-call path: one k_step launch per step, the launch SimpleGridworldSimulator.step() "
                      "makes (scripts/env.py:155, scripts/run.py:10-15's loop without Python), timed over the "
                      "same number of steps as the headline; bit-identical outputs"}
        if loop_main and one_launch_s is not None:
            pc["kernel_avg_us"] = one_launch_s * 1e6
            pc["frac"] = out["roofline"]["one_launch_per_step"]["frac"]
            pc["algorithmic_bytes_per_launch"] = L.bb_algorithmic_bytes_per_world(args.agents) * W
            pc["traffic"] = load_traffic(f"W{W}_N{args.agents}_per_call")
        out["per_call_step"] = pc
        out["headline"] = ("value = the staged steps as one launch (" + out["roofline"]["kernel"] + "); every step "
                           "stores all its outputs as a per-call step does, but no consumer runs between steps: an "
                           "upper bound of the per-call path, whose own rate is per_call_step.value (the drop-in "
                           "path) and e2e.value (env.py's Python loop)") if loop_main else "one k_step launch per step"
    if e2e is not None:
        out["e2e"] = e2e
    out.update(extra)
    if rank == 0:
        out["cpu_baseline"] = cpu
        out["cpu_executor"] = cpu_exec
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
