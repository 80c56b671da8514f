#!/usr/bin/env python
"""Headline benchmark: humanoid env steps/sec (whole node), 'stand' task -- BASELINE.json metric.

One "step" = one batched env step of every env on the rank: frame_skip=3 physics substeps
(full mj_step pipeline incl. contacts + Newton solve), the 352-value observation, the device
stand reward, termination/truncation and auto-reset -- one launch of the fused step kernel (plus
the wide-contact-tier launch, which re-runs the rare envs whose contacts overflow the resident
tier and otherwise exits at once).  Workload (BASELINE.json configs[1]): 4096 humanoid.xml envs
per GPU, stand reward, frame_skip 3, duration 10, computed in float64 like the reference's
MuJoCo (mjtNum); actions come from a pre-generated U(-1,1) action tape already resident in HBM
(sim-only mode).

Representative window: before the warm-up, env i's clock is set to i/N of the episode and the
batch runs one full episode (667 env steps, untimed), so every env is at a different point of
its episode (auto-resets included) and ANY timed window averages over standing, falling and
lying humanoids -- the whole-episode mix of training, not the first 20 steps after a reset.

N GPUs run N independent env shards (weak scaling, no data-path collective).  ``--gpus N``
without a launcher spawns the N ranks itself (torch.distributed.run, 127.0.0.1); under an
external launcher WORLD_SIZE must equal N.  Rank 0 prints one JSON line.

Extra keys: fp32 sim-only, the same window as one open-loop tape launch (hs_step_tape),
full-episode legs on tapes T0/T1/T2, rollout (+ PPO.collect_rollouts fused vs
per-step) / train / GAE, configs[3]/[4] (+ tape and fused-collect variants), the step-kernel
roofline (HBM bytes vs 8 TB/s, live HIP events on the launch stream) and the CPU baseline (the
reference's n_envs=8 SubprocVecEnv path, on the oracle's fp64 C restatement of mj_step because
MuJoCo is not installable: kind "port").
"""
import argparse
import json
import math
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")

N_ENVS_PER_GPU = 4096
FRAME_SKIP = 3
DURATION = 10.0
TIMESTEP = 0.005
EPISODE = math.ceil(DURATION / (FRAME_SKIP * TIMESTEP) - 1e-9)   # 667 env steps (custom_env.py:213)
HBM_PEAK_GBS = 8000.0
PROFILE_TRAFFIC = os.path.join(ROOT, "profiles", "traffic_step_kernel.json")
FLOPS_JSON = os.path.join(ROOT, "profiles", "flops_per_env_step.json")     # oracle/flops.py
# vector (VALU) peaks: FP32 157.3 TFLOP/s (MI355X_MICROARCH.md); FP64 vector runs at half that rate
# (78.6 TFLOP/s, AMD's MI355X spec)
VALU_PEAK_TFLOPS = {"fp32": 157.3, "fp64": 78.6}


def algo_bytes_per_env_step(es):
    """Algorithmic HBM bytes of one env step of the fused kernel, state and obs of
    element size ``es``: read qpos 28 + qvel 27 + qacc_warmstart 27 + time 1 (state) and the f32
    action 21; write qpos/qvel/warmstart/time 83 + obs 352 + reward 1; + 2 B of done flags.
    fp32: 2162 B; fp64: 4238 B."""
    return 83 * es + 21 * 4 + 436 * es + 2


L2_PEAK_GBS = 18800.0      # MI355X_MICROARCH.md "Indexed rows": rows shared by every workgroup, served by the XCD L2s
PROFILE_ROLLOUT_TRAFFIC = os.path.join(ROOT, "profiles", "traffic_rollout_kernel.json")


def rollout_algo_bytes(D, A, k, es=8, nq=28, nv=27, H=256):
    """Algorithmic bytes per env step of the fused rollout kernel (hs_rollout) over a
    launch of k env steps.  HBM: per env step the rollout rows written -- obs row (f32 D), actions
    (f32 A), log-prob, episode start, reward (f32 each), done (1 B), episode return (f64), bootstrap
    flag (1 B) -- plus, once per launch and env (amortised over k): the state read and written
    (qpos / qvel / warm start / time in es bytes, step count / episode / 5 warning ints / return),
    the obs_last row (f32 D), the batch's obs row (es D), the clipped action in and out (f32 A),
    ep_acc in and out (f64) and episode_start (f32).  L2: the pi net's weights and biases (f32),
    streamed once per wave and env step for the wave's two envs."""
    rows = 4 * D + 4 * A + 4 + 4 + 4 + 1 + 8 + 1
    per_launch = 2 * ((nq + 2 * nv + 1) * es + 7 * 4 + es) + 4 * D + es * D + 2 * 4 * A + 2 * 8 + 4
    hbm = rows + per_launch / k
    weights = 4 * (D * H + H * H + H * A + H + H + A)
    return hbm, weights / 2


# ----------------------------------------------------------------------------- CPU baseline
def _cpu_worker(conn, seed):
    """SubprocVecEnv._worker equivalent around the fp64 oracle env (train_sb3.py:203)."""
    from oracle.env import OracleHumanoidEnv
    env = OracleHumanoidEnv({"model_path": XML, "duration": DURATION, "reward_config": {"type": "stand"},
                             "frame_skip": FRAME_SKIP})
    env.reset(seed=seed)
    while True:
        cmd, data = conn.recv()
        if cmd == "step":
            obs, r, term, trunc, info = env.step(data)
            if term or trunc:
                info["terminal_observation"] = obs
                obs, _ = env.reset()
            conn.send((obs, r, term or trunc, info))
        elif cmd == "close":
            conn.close()
            return


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(n_envs=8, vec_steps=1500):
    ctx = mp.get_context("fork")
    pipes, procs = [], []
    for i in range(n_envs):
        a, b = ctx.Pipe()
        p = ctx.Process(target=_cpu_worker, args=(b, i), daemon=True)
        p.start()
        pipes.append(a)
        procs.append(p)
    rng = np.random.default_rng(0)
    acts = rng.uniform(-1, 1, (vec_steps + 20, n_envs, 21)).astype(np.float32)

    def vec_step(k):
        for i, c in enumerate(pipes):
            c.send(("step", acts[k, i]))
        return [c.recv() for c in pipes]
    for k in range(20):
        vec_step(k)
    t = time.perf_counter()
    for k in range(vec_steps):
        vec_step(20 + k)
    dt = time.perf_counter() - t
    for c in pipes:
        c.send(("close", None))
    for p in procs:
        p.join(timeout=10)
    return dict(value=n_envs * vec_steps / dt, unit="env_steps/s", cores=n_envs, kind="port",
                cpu_model=_cpu_model(), nproc=os.cpu_count(),
                sample=f"{n_envs} worker processes x {vec_steps} env steps (stand, frame_skip 3, U(-1,1) actions, "
                       f"pipe IPC per step as SB3 SubprocVecEnv) on the fp64 oracle restatement of mj_step "
                       f"(numpy/ctypes host glue, one process per env, single-threaded each); {dt:.1f} s wall")


# ----------------------------------------------------------------------------- launcher
def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(nproc):
    """Spawn ``nproc`` ranks of this script (one process per GPU) with torch.distributed.run on
    127.0.0.1; this parent never touches the GPU.  Returns the launcher's exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def selftest_launch(args, world, rank):
    """--selftest-launch: the multi-rank plumbing of the bench (rendezvous, barrier, max-over-ranks
    timing, the JSON line) with a trivial CPU loop instead of the GPU work (CPU test of --gpus N)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    ws = dist.get_world_size() if world > 1 else 1
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    x = np.zeros(1000)
    for k in range(args.steps):
        x += k
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "selftest", "value": args.steps * ws / max(float(el.item()), 1e-9),
                          "unit": "steps/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup}))
    if world > 1:
        dist.destroy_process_group()


# ----------------------------------------------------------------------------- GPU
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--envs", type=int, default=N_ENVS_PER_GPU, help="envs per GPU")
    ap.add_argument("--precision", default="fp64", choices=["fp32", "fp64"],
                    help="headline arithmetic (fp64 = the reference's mjtNum; fp32 is an extra leg)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--schedule", default="auto", help=argparse.SUPPRESS)   # A/B runs (HsBatch.configure)
    ap.add_argument("--no-rollout", action="store_true")
    ap.add_argument("--no-gae", action="store_true")
    ap.add_argument("--train-iters", type=int, default=2, help="PPO iterations of the train mode (0: skip)")
    ap.add_argument("--no-configs", action="store_true", help="skip the configs[3]/[4] legs")
    ap.add_argument("--no-fp32", action="store_true", help="skip the fp32 sim-only leg")
    ap.add_argument("--no-tape", action="store_true", help="skip the open-loop tape leg (hs_step_tape)")
    ap.add_argument("--no-episodes", action="store_true", help="skip the full-episode T0/T1/T2 legs")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the drop-in leg (SB3 VecEnv step_async/step_wait in numpy mode, HumanoidEnv.step)")
    ap.add_argument("--no-precondition", action="store_true",
                    help="time from a synchronized reset (standing humanoids only) instead of the staggered mix")
    ap.add_argument("--free-groups", type=int, default=0, help="extra sim-only leg: this many free-running stream "
                                                                "groups (0: skip)")
    ap.add_argument("--protocol-tape", action="store_true",
                    help="with --protocol: time the 10000 steps as hs_step_tape calls of 500 steps (open loop)")
    ap.add_argument("--protocol", action="store_true",
                    help="SURVEY 8d protocol instead of the default run: 1000 warm-up + 10000 timed env steps "
                         "per tape T0/T1/T2 and base seed {0,1,2} (~2 min per precision)")
    ap.add_argument("--dist-backend", default=os.environ.get("HSIM_BENCH_BACKEND", "nccl"),
                    help="nccl (= RCCL over xGMI; the real multi-GPU run) or gloo (multi-rank rehearsal on one GPU)")
    ap.add_argument("--cpu-steps", type=int, default=60000, help="vec steps of the CPU baseline (~13 s)")
    ap.add_argument("--selftest-launch", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (one rank per GPU)")
    if args.selftest_launch:
        return selftest_launch(args, world, rank)
    cpu_res = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_res = cpu_baseline(vec_steps=args.cpu_steps)   # before any GPU/torch init (fork-safe)

    import torch
    import torch.distributed as dist
    if cpu_res is not None:
        cpu_res["torch_threads"] = torch.get_num_threads()
    gloo = args.dist_backend == "gloo"
    # gloo rehearsal: ranks may share a GPU; nccl: one process per GPU (LOCAL_RANK = device)
    dev_index = local_rank % max(1, torch.cuda.device_count()) if gloo else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    red_dev = torch.device("cpu") if gloo else dev      # device of the timing reductions
    ranks = dist.get_world_size() if world > 1 else 1

    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    cfg = {"model_path": XML, "duration": DURATION, "reward_config": {"type": "stand"}, "frame_skip": FRAME_SKIP}
    model = HsModel(XML)
    n = args.envs
    stream = torch.cuda.current_stream(dev)

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def max_over_ranks(x):
        t = torch.tensor([x], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def make_tape(kind, length, n_x, seed):
        g = torch.Generator(device=dev).manual_seed(seed)
        if kind == "T0":
            return torch.zeros(length, n_x, model.nu, device=dev)
        if kind == "T2":
            return (torch.randn(length, n_x, model.nu, device=dev, generator=g) * 0.1).clamp_(-1, 1)
        return (torch.rand(length, n_x, model.nu, device=dev, generator=g) * 2 - 1).contiguous()

    def make_env(precision, seed, cfg_x=cfg, n_x=n, stats=False):
        e = HumanoidVecEnv(cfg_x, n_envs=n_x, device=dev_index, precision=precision, seed=seed + 7919 * rank,
                           model=model)
        # sim-only timing writes what a trainer needs; the aux row / ctrl copy only when stats are read
        e.batch.configure(aux=stats, ctrl=False, schedule=args.schedule)
        e.reset_tensors()
        return e

    def precondition(e, tape):
        """Staggered episode phases: env i's clock starts at i/N of the episode, then one full
        episode runs, so env i ends up ~i/N of the way into a genuine episode (after its first
        auto-reset); untimed."""
        if args.no_precondition:
            return
        nx = e.num_envs
        t0 = np.floor(np.arange(nx) * EPISODE / nx) * FRAME_SKIP * TIMESTEP + TIMESTEP
        e.batch.set_state(time=t0)
        for k in range(EPISODE):
            e.step_tensors(tape[k % tape.shape[0]])

    def timed(e, tape, steps, warmup, offset=0):
        """warm-up, then ``steps`` env steps bracketed by barrier + synchronize; returns
        (wall seconds max over ranks, HIP-event ms per step on the launch stream)."""
        for k in range(warmup):
            e.step_tensors(tape[(offset + k) % tape.shape[0]])
        barrier()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for k in range(steps):
            e.step_tensors(tape[(offset + warmup + k) % tape.shape[0]])
        ev1.record(stream)
        barrier()
        return max_over_ranks(time.perf_counter() - t0), ev0.elapsed_time(ev1) / steps

    def timed_tape(e, tape, steps, warmup, offset=0, chunk=None):
        """The same window as ``timed`` as ONE tape launch (HsBatch.step_tape: K env steps, each env
        pair's step t + 1 starting once its own step t is committed); open loop, bitwise the step
        loop's results (tests/test_gpu_tape.py).  Every step's obs / reward / done flags are written
        (per-step output slices), as the per-step launches write them.  ``chunk``: step_tape calls of
        at most that many steps (bounds the per-step output slices of long windows).  Returns (wall
        seconds max over ranks, ms per env step)."""
        for k in range(warmup):
            e.step_tensors(tape[(offset + k) % tape.shape[0]])
        idx = torch.arange(offset + warmup, offset + warmup + steps, device=dev) % tape.shape[0]
        tp = tape.index_select(0, idx).contiguous()
        chunk = chunk or steps
        barrier()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for c in range(0, steps, chunk):
            e.batch.step_tape(tp[c:c + chunk], outputs=True)
        ev1.record(stream)
        barrier()
        return max_over_ranks(time.perf_counter() - t0), ev0.elapsed_time(ev1) / steps

    def ints_over_ranks(vals, op):
        """elementwise MAX / SUM of a list of per-rank integer counters over all ranks"""
        t = torch.tensor(vals, dtype=torch.int64, device=red_dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
        return [int(x) for x in t.tolist()]

    def warn_stats(e):
        """per-env warning counters (bad qpos / qvel / qacc, contact overflow) summed over the
        rank's envs, reported as the MAX over ranks (and the node SUM), plus wide-tier re-runs"""
        w = [int(x) for x in e.batch.warning.sum(0).tolist()]
        rr = int(e.batch.wide_reruns())
        return dict(warnings=ints_over_ranks(w, "max"), warnings_node_sum=ints_over_ranks(w, "sum"),
                    wide_tier_reruns=ints_over_ranks([rr], "max")[0])

    def stats_of(e, tape, k0, steps=3):
        """aux-row statistics of a few further (untimed) steps of the same batch (this rank's envs;
        the warning counters are reduced over ranks)."""
        e.batch.configure(aux=True)
        for k in range(steps):
            e.step_tensors(tape[(k0 + k) % tape.shape[0]])
        a = e.batch.aux.double()
        e.batch.configure(aux=False)
        return dict(mean_contacts=float(a[:, 35].mean()), max_contacts=int(a[:, 35].max()),
                    mean_rows=float(a[:, 36].mean()), max_rows=int(a[:, 36].max()),
                    mean_newton_iters=float(a[:, 37].mean()),
                    fallen_frac=float((e.batch.qpos[:, 2] < 0.8).double().mean()), **warn_stats(e))

    if args.protocol:
        tfn = (lambda e, tp, steps, warmup: timed_tape(e, tp, steps, warmup, chunk=500)) if args.protocol_tape else timed
        return run_protocol(args, rank, world, ranks, make_env, make_tape, precondition, tfn, stats_of)

    # ---- headline: configs[1], fp64, staggered whole-episode mix
    tape = make_tape("T1", 1024, n, 1 + rank)
    env = make_env(args.precision, 1000)
    precondition(env, tape)
    elapsed, step_ms = timed(env, tape, args.steps, args.warmup, offset=EPISODE)
    value = n * args.steps * ranks / elapsed
    stats = stats_of(env, tape, EPISODE + args.warmup + args.steps)
    kernel_ms = step_ms
    queued = env.batch.queued()
    env.close()

    # ---- fp32 sim-only leg (the throughput engine; tolerance-based parity, not the headline)
    fp32_leg = None
    if args.precision == "fp64" and not args.no_fp32:
        e = make_env("fp32", 5000)
        precondition(e, tape)
        el, ms = timed(e, tape, args.steps, args.warmup, offset=EPISODE)
        fp32_leg = dict(value=n * args.steps * ranks / el, unit="env_steps/s", dtype="f32", steps=args.steps,
                        kernel_ms_per_launch=ms, stats=stats_of(e, tape, EPISODE + args.warmup + args.steps),
                        note="same workload and staggered episode mix, fp32 engine (parity within fp32 tolerances, "
                             "not the reference's fp64: see DESIGN.md 4)")
        e.close()

    # ---- open-loop tape leg: the same fp64 window as one tape launch (not the headline: a policy in
    # the loop steps one env step per launch)
    tape_leg = None
    if not args.no_tape:
        e = make_env(args.precision, 1000)
        precondition(e, tape)
        el, ms = timed_tape(e, tape, args.steps, args.warmup, offset=EPISODE)
        tape_leg = dict(value=n * args.steps * ranks / el, unit="env_steps/s", dtype="f64" if args.precision == "fp64"
                        else "f32", steps=args.steps, ms_per_env_step=ms, tape_aborts=e.batch.tape_aborts(),
                        note="same workload, window and action tape as the headline, all timed env steps in ONE "
                             "hs_step_tape launch with every step's obs / reward / done written (open loop: each env "
                             "pair's step t+1 starts when its own step t is committed, so steps do not end on their "
                             "slowest pair); bitwise the per-step results")
        e.close()

    # ---- full episodes from a synchronized reset on tapes T0 / T1 / T2, per phase
    episodes = None
    if not args.no_episodes:
        episodes = {}
        phases = [(0, 50), (50, 100), (100, 200), (200, 300), (300, 400), (400, 500), (500, 600), (600, EPISODE)]
        for kind in ("T0", "T1", "T2"):
            tp = make_tape(kind, EPISODE, n, 11 + rank)
            e = make_env(args.precision, 6000, stats=True)
            per, tot_t = [], 0.0
            for a, b in phases:
                barrier()
                t0 = time.perf_counter()
                for k in range(a, b):
                    e.step_tensors(tp[k])
                barrier()
                dt = max_over_ranks(time.perf_counter() - t0)
                tot_t += dt
                ax = e.batch.aux.double()
                per.append(dict(steps=[a, b], env_steps_per_s=n * (b - a) * ranks / dt,
                                mean_contacts=float(ax[:, 35].mean()), mean_rows=float(ax[:, 36].mean()),
                                mean_newton_iters=float(ax[:, 37].mean()),
                                fallen_frac=float((e.batch.qpos[:, 2] < 0.8).double().mean())))
            episodes[kind] = dict(value=n * EPISODE * ranks / tot_t, unit="env_steps/s", steps=EPISODE,
                                  phases=per, **warn_stats(e))
            e.close()

    # ---- rollout mode: policy MLP[256,256] forward + sampling + env step (on device)
    rollout = None
    if not args.no_rollout:
        from mujocoposelearning_amd.ppo import ActorCritic, ppo_act
        e = make_env(args.precision, 7000)
        precondition(e, tape)
        pol = ActorCritic(e.batch.obs_dim, model.nu, (256, 256), activation=torch.nn.ReLU).to(dev)
        pol.pack_heads()
        ls = pol.log_std.detach()
        start = torch.zeros(n, device=dev)
        act, clip = torch.empty(n, model.nu, device=dev), torch.empty(n, model.nu, device=dev)
        logp, val, st_out = (torch.empty(n, device=dev) for _ in range(3))
        obs = e.batch.obs

        def policy_step(obs, k):
            # the PPO rollout's policy half (ppo.PPO._collect_rollouts_device): packed pi/vf GEMM
            # chain (fp32, as SB3's policy) + hs_ppo_act (Gaussian sample, log-prob, clip), then the env
            mean, value_ = pol.heads(obs.float())
            ppo_act(mean, value_, ls, start, 1 + rank, k, False, act, clip, logp, val, st_out)
            return e.step_tensors(clip)[0]

        with torch.no_grad():
            for k in range(5):
                obs = policy_step(obs, k)
            barrier()
            tr0 = time.perf_counter()
            rs = max(10, args.steps // 2)
            for k in range(rs):
                obs = policy_step(obs, 5 + k)
            barrier()
            rel = max_over_ranks(time.perf_counter() - tr0)
        rollout = dict(value=n * rs * ranks / rel, unit="env_steps/s",
                       note="policy MLP[256,256] (pi+vf, packed GEMM chain, fp32) forward + hs_ppo_act "
                            "(diag-Gaussian sample, log-prob, clip) + env step")
        e.close()
        # PPO.collect_rollouts end to end (32 steps: sample, env step, buffers, values, GAE), the fused
        # rollout (hs_rollout: the pi net inside the env kernel, one launch per rollout) against the
        # per-step path (policy GEMMs + hs_ppo_act + env launch + hs_ppo_post per step, one HIP graph)
        from mujocoposelearning_amd import ppo as ppo_mod
        collect = {}
        for fused in (True, False):
            ppo_mod.FUSED_ROLLOUT = fused
            e = make_env(args.precision, 6000)
            p = ppo_mod.PPO(e, n_steps=32, batch_size=32768, n_epochs=1, seed=0,
                            policy_kwargs={"net_arch": {"pi": [256, 256], "vf": [256, 256]}, "activation_fn": "ReLU"})
            kk = np.floor(np.arange(n) * EPISODE / n)              # staggered episode clocks (the window's mix)
            e.batch.t["time"].copy_(torch.as_tensor(kk * FRAME_SKIP * TIMESTEP + TIMESTEP, dtype=e.batch.dtype,
                                                    device=dev))
            e.batch.t["step_count"].copy_(torch.as_tensor(kk, dtype=torch.int32, device=dev))
            for _ in range(2):
                p.collect_rollouts()
            barrier()
            tc0 = time.perf_counter()
            R = 4
            for _ in range(R):
                p.collect_rollouts()
            barrier()
            collect["fused" if fused else "per_step"] = dict(
                value=n * 32 * R * ranks / max_over_ranks(time.perf_counter() - tc0), unit="env_steps/s",
                used_fused=p._fused_rollout_args() is not None, fallbacks=getattr(p, "fused_fallbacks", 0))
            e.close()
        ppo_mod.FUSED_ROLLOUT = True
        rollout["collect_rollouts"] = dict(
            **collect, n_steps=32, note="PPO.collect_rollouts (sampling, env steps, rollout buffers, values, GAE) "
                                        "from staggered episode clocks; fused = hs_rollout (policy forward in the "
                                        "env kernel, one launch per rollout), per_step = one HIP graph of per-step "
                                        "launches")

    # ---- drop-in leg: the north star's unchanged call sites (train_sb3.py:203 SubprocVecEnv ->
    # HumanoidVecEnv, numpy actions in, numpy obs / rewards / dones / infos out; custom_env.py:152-230
    # HumanoidEnv.step for one env), PCIe-inclusive
    dropin = None
    if not args.no_dropin:
        from mujocoposelearning_amd.env import HumanoidEnv
        dropin = {}
        rng_np = np.random.default_rng(3 + rank)
        for n_x, ks in ((8, 400), (16, 400), (64, 200), (256, 100), (n, 30)):
            e = make_env(args.precision, 9000, n_x=n_x)
            precondition(e, tape[:, :n_x])
            acts_np = rng_np.uniform(-1, 1, (ks + 5, n_x, model.nu)).astype(np.float32)
            for k in range(ks):                  # warm-up: pinned staging blocks, clocks
                e.step_async(acts_np[k % ks])
                e.step_wait()
            res = {}
            for consume in (False, True):
                barrier()
                t0 = time.perf_counter()
                for k in range(ks):
                    e.step_async(acts_np[k % ks])
                    obs_, rew_, done_, infos_ = e.step_wait()
                    if consume:      # SB3 collect_rollouts' per-step reads (_update_info_buffer, TimeLimit bootstrap)
                        for i, info in enumerate(infos_):
                            info.get("episode")
                            if done_[i] and info.get("terminal_observation") is not None:
                                info.get("TimeLimit.truncated", False)
                barrier()
                el = max_over_ranks(time.perf_counter() - t0)
                res["with_sb3_info_reads" if consume else "step_wait"] = dict(
                    value=n_x * ks * ranks / el, unit="env_steps/s", ms_per_step=el / ks * 1e3)
            dropin[f"vec_env_{n_x}"] = dict(n_envs_per_gpu=n_x, steps=ks, **res)
            e.close()
        he = HumanoidEnv({"model_path": XML, "duration": DURATION, "reward_config": {"type": "stand"},
                          "frame_skip": FRAME_SKIP, "device": dev_index, "precision": args.precision})
        ha = rng_np.uniform(-1, 1, (300, model.nu)).astype(np.float32)
        for k in range(20):
            he.step(ha[k])
        t0 = time.perf_counter()
        for k in range(200):
            _, _, term_, trunc_, _ = he.step(ha[20 + k])
            if term_ or trunc_:
                he.reset()
        hl = (time.perf_counter() - t0) / 200
        he.close()
        dropin["humanoid_env_step"] = dict(ms_per_step=hl * 1e3, value=1.0 / hl, unit="env_steps/s", n_envs=1)
        dropin["note"] = ("numpy surfaces of the reference's call sites, PCIe-inclusive: HumanoidVecEnv.step_async / "
                          "step_wait (SB3 VecEnv API, SubprocVecEnv semantics; obs / rewards / dones / final-step info "
                          "in one packed pinned copy, infos built lazily) at configs[0]'s 8 envs, 16 / 64 / 256 (where the GPU "
                          "passes the 8-process CPU baseline) and configs[1]'s 4096, from staggered episode clocks; with_sb3_info_reads also touches every info as SB3's "
                          "collect_rollouts does; humanoid_env_step: the single-env Gym step() latency")

    # ---- extra sim-only leg: free-running stream groups (opt-in)
    grouped = None
    if args.free_groups > 1:
        eg = HumanoidVecEnv(cfg, n_envs=n, device=dev_index, precision=args.precision, seed=3000 + rank,
                            model=model, groups=args.free_groups)
        eg.batch.configure(aux=False, ctrl=False)
        eg.reset_tensors()
        for k in range(args.warmup):
            eg.batch.step(tape[k], join=False)
        eg.batch.join()
        barrier()
        tg = time.perf_counter()
        for k in range(args.steps):
            eg.batch.step(tape[(args.warmup + k) % tape.shape[0]], join=False)
        eg.batch.join()
        barrier()
        grouped = dict(value=n * args.steps * ranks / max_over_ranks(time.perf_counter() - tg), unit="env_steps/s",
                       groups=args.free_groups,
                       note="envs split into free-running stream groups (HsBatch join=False), from a reset")
        eg.close()

    # ---- BASELINE.json configs[3] (kneeling reward, 4096 envs) and configs[4] (full-state obs,
    # 8192 envs over 8 GPUs = 1024 per GPU): same staggered sim-only protocol
    config_legs = None
    if not args.no_configs:
        def leg(cfg_x, n_x, label):
            e = make_env(args.precision, 4000, cfg_x=cfg_x, n_x=n_x)
            tp = tape[:, :n_x] if n_x <= n else make_tape("T1", 1024, n_x, 5)
            precondition(e, tp)
            ks = min(args.steps, 50)
            el, _ = timed(e, tp, ks, args.warmup, offset=EPISODE)
            r = dict(value=n_x * ks * ranks / el, unit="env_steps/s", n_envs_per_gpu=n_x, obs_dim=e.obs_dim,
                     workload=label)
            e.close()
            if not args.no_rollout and cfg_x.get("full_state_obs"):
                # configs[4] in the trainer: PPO.collect_rollouts with the fused rollout (hs_rollout)
                from mujocoposelearning_amd import ppo as ppo_mod
                e = make_env(args.precision, 4100, cfg_x=cfg_x, n_x=n_x)
                p = ppo_mod.PPO(e, n_steps=32, batch_size=8192, n_epochs=1, seed=0,
                                policy_kwargs={"net_arch": {"pi": [256, 256], "vf": [256, 256]},
                                               "activation_fn": "ReLU"})
                kk = np.floor(np.arange(n_x) * EPISODE / n_x)
                e.batch.t["time"].copy_(torch.as_tensor(kk * FRAME_SKIP * TIMESTEP + TIMESTEP, dtype=e.batch.dtype,
                                                        device=dev))
                e.batch.t["step_count"].copy_(torch.as_tensor(kk, dtype=torch.int32, device=dev))
                for _ in range(2):
                    p.collect_rollouts()
                barrier()
                tc0 = time.perf_counter()
                for _ in range(4):
                    p.collect_rollouts()
                barrier()
                r["collect_rollouts_fused"] = dict(value=n_x * 32 * 4 * ranks / max_over_ranks(time.perf_counter() - tc0),
                                                   unit="env_steps/s", used_fused=p._fused_rollout_args() is not None)
                e.close()
            if not args.no_tape:   # the same window as one open-loop tape launch
                e = make_env(args.precision, 4000, cfg_x=cfg_x, n_x=n_x)
                precondition(e, tp)
                elt, _ = timed_tape(e, tp, ks, args.warmup, offset=EPISODE)
                r["tape"] = dict(value=n_x * ks * ranks / elt, unit="env_steps/s", tape_aborts=e.batch.tape_aborts())
                e.close()
            return r
        config_legs = {
            "configs[3]": leg({**cfg, "reward_config": {"type": "kneeling"}}, n,
                              "kneeling (robust_kneeling_reward) device reward, humanoid.xml x 4096 envs per GPU"),
            "configs[4]": leg({**cfg, "full_state_obs": True}, 1024,
                              "full-state obs (+cfrc_ext[1:], 448 values; subtree_linvel), 1024 envs per GPU "
                              "(8192 over 8 GPUs)"),
        }

    # ---- train mode (SURVEY 8d iii): end-to-end on-device PPO iterations (rollout with the
    # MLP[256,256] policy + GAE + clipped-surrogate updates with the per-step gradient all-reduce)
    train_res = None
    if args.train_iters > 0:
        from mujocoposelearning_amd.ppo import PPO
        e = make_env(args.precision, 8000)
        tk = dict(n_steps=32, batch_size=32768, n_epochs=4, learning_rate=3e-4, stagger_episodes=True,
                  policy_kwargs={"net_arch": {"pi": [256, 256], "vf": [256, 256]}, "activation_fn": "ReLU"})
        ppo = PPO(e, seed=0, world_size=world, rank=rank, **tk)
        ppo.learn(ppo.num_timesteps + n * tk["n_steps"] * world)          # warm-up iteration
        ppo.rollout_launches = []
        barrier()
        t_tr = time.perf_counter()
        ppo.learn(ppo.num_timesteps + args.train_iters * n * tk["n_steps"] * world)
        barrier()
        ts = max_over_ranks(time.perf_counter() - t_tr)
        # roofline of the train leg's dominant kernel: the fused rollout launch (hs_rollout), its mean
        # duration from HIP events recorded around it on its stream (hs_last_tape_ms)
        rl = getattr(ppo, "rollout_launches", [])
        train_roof = None
        if rl:
            env_steps = sum(s for s, _ in rl) / len(rl)
            kms = max_over_ranks(sum(ms for _, ms in rl) / len(rl))
            ksteps = env_steps / n
            hbm_b, l2_b = rollout_algo_bytes(e.batch.obs_dim, model.nu, ksteps)
            ach = hbm_b * env_steps / (kms * 1e-3) / 1e9
            l2a = l2_b * env_steps / (kms * 1e-3) / 1e9
            rtr = None
            if os.path.exists(PROFILE_ROLLOUT_TRAFFIC):
                rtr = json.load(open(PROFILE_ROLLOUT_TRAFFIC))
            train_roof = dict(
                bound="hbm", achieved=ach, peak=HBM_PEAK_GBS, unit="GB/s", frac=ach / HBM_PEAK_GBS,
                traffic=(rtr["hbm_bytes_per_launch"] * env_steps / rtr["env_steps_per_launch"]) if rtr else None,
                kernel="step_kernel_queue<double,27,false,true> (fused rollout, hs_rollout)",
                kernel_ms_per_launch=kms, env_steps_per_launch=env_steps, launches=len(rl),
                algo_bytes_per_env_step=hbm_b,
                l2_weight_stream=dict(bytes_per_env_step=l2_b, achieved=l2a, peak=L2_PEAK_GBS, unit="GB/s",
                                      frac=l2a / L2_PEAK_GBS,
                                      note="pi-net weights (f32) each wave streams per env step for its two envs; "
                                           "peak: MI355X_MICROARCH.md shared-row L2 rate"),
                profile=rtr.get("source") if rtr else None,
                note="HIP events around each hs_rollout kernel launch (hs_last_tape_ms), timed iterations; "
                     "algorithmic bytes: bench.rollout_algo_bytes (rollout rows per env step + the state, obs and "
                     "action rows once per launch and env); traffic: 2*FETCH+WRITE of the committed profile scaled "
                     "to this launch size")
        train_res = dict(value=args.train_iters * n * tk["n_steps"] * ranks / ts, unit="env_steps/s",
                         iterations=args.train_iters, ms_per_iteration=ts / args.train_iters * 1e3,
                         env_precision=args.precision,
                         config={k: v for k, v in tk.items() if k != "policy_kwargs"} | {"net_arch": "[256,256] ReLU"},
                         roofline=train_roof,
                         roofline_frac=train_roof["frac"] if train_roof else None,
                         l2_weight_frac=train_roof["l2_weight_stream"]["frac"] if train_roof else None,
                         kernel_ms_per_launch=train_roof["kernel_ms_per_launch"] if train_roof else None,
                         note="rollout (policy forward + env step) + GAE + 4 epochs of minibatch updates, "
                              "one gradient all-reduce per optimizer step")
        e.close()

    # ---- GAE leg: the rollout-end reverse scan (hs_gae) over an n_steps=2048 x n-env buffer
    gae_res = None
    if not args.no_gae:
        from mujocoposelearning_amd.ppo import gae_device
        Tg = 2048
        gg = torch.Generator(device=dev).manual_seed(11)
        rb = [torch.randn(Tg, n, device=dev, generator=gg) for _ in range(2)]
        stg = (torch.rand(Tg, n, device=dev, generator=gg) < 1 / 667).float()
        lvg, ldg = torch.randn(n, device=dev, generator=gg), torch.zeros(n, device=dev)
        for _ in range(3):
            gae_device(rb[0], rb[1], stg, lvg, ldg, 0.99, 0.95)
        torch.cuda.synchronize(dev)
        reps = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            gae_device(rb[0], rb[1], stg, lvg, ldg, 0.99, 0.95)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        gms = e0.elapsed_time(e1) / reps
        gbs = 20.0 * Tg * n / (gms * 1e-3) / 1e9
        gae_res = {"kernel": "gae_kernel", "T": Tg, "n_envs": n, "ms_per_rollout": gms,
                   "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": gbs / HBM_PEAK_GBS, "algo_bytes_per_element": 20}}

    if rank == 0:
        es = 8 if args.precision == "fp64" else 4
        abytes = algo_bytes_per_env_step(es)
        achieved = abytes * n / (kernel_ms * 1e-3) / 1e9
        traffic = issue = None
        if os.path.exists(PROFILE_TRAFFIC):
            try:
                tr = json.load(open(PROFILE_TRAFFIC)).get(args.precision, {})
                if tr.get("n_envs") == n:
                    traffic = tr.get("hbm_bytes_per_launch")
                    # what bounds it: the share of the waves' lifetime their SIMD's VALU spends on them
                    # (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, same counter units) -- fp64 VALU ops issue at
                    # half the fp32 rate, so an instruction count priced at a fixed cycles-per-op would
                    # understate it; and the share parked on s_waitcnt (SQ_WAIT_ANY / SQ_WAVE_CYCLES)
                    sq = tr.get("sq", {})
                    if sq.get("SQ_ACTIVE_INST_VALU") and sq.get("SQ_WAVE_CYCLES"):
                        wc = sq["SQ_WAVE_CYCLES"]
                        issue = {"frac": sq["SQ_ACTIVE_INST_VALU"] / wc,
                                 "wait_frac": sq.get("SQ_WAIT_ANY", 0.0) / wc,
                                 "issue_any_frac": sq.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
                                 "source": f"SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES of the committed profile "
                                           f"({tr.get('tag')})"}
            except Exception:
                traffic = None
        kname = ("step_kernel_queue" if queued else "step_kernel") + (
            "<double,27>" if args.precision == "fp64" else "<float,27>")
        vflops = None
        if os.path.exists(FLOPS_JSON):
            fpe = json.load(open(FLOPS_JSON))["mean_total"]
            ach = fpe * n / (kernel_ms * 1e-3) / 1e12
            vflops = {"flops_per_env_step": fpe, "achieved_tflops": ach,
                      "peak_tflops": VALU_PEAK_TFLOPS[args.precision], "frac": ach / VALU_PEAK_TFLOPS[args.precision],
                      "source": "oracle restatement FLOP count per env step (oracle/flops.py, mean of tapes "
                                "T0/T1/T2) x envs / live launch time; an upper bound on the kernel's useful FLOPs"}
        out = {
            "metric": "env steps/sec (whole node), humanoid 'stand' task, 1/2/4/8 MI355X",
            "value": value,
            "unit": "env_steps/s",
            "n_gpus": ranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if args.precision == "fp64" else "f32",
            "data": "synthetic (reset distribution of custom_env.py:97-121; U(-1,1) action tape in HBM; "
                    "staggered episode phases, see config.window)",
            "config": {"workload": "configs[1]: humanoid.xml x 4096 envs per GPU, 'stand' reward, frame_skip 3, "
                                   "duration 10 (sim-only env steps, fp64 physics like the reference's mjtNum)",
                       "n_envs_per_gpu": n, "n_envs_total": n * ranks, "frame_skip": FRAME_SKIP,
                       "reward": "stand", "parallelism": f"dp{ranks} (env shards, no collective)",
                       "window": ("synchronized reset (standing phase only)" if args.no_precondition else
                                  f"staggered: env i starts at episode step ~{EPISODE}*i/N, then one untimed "
                                  f"{EPISODE}-step episode; every timed window averages the whole-episode mix")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kname,
                         "kernel_ms_per_launch": kernel_ms, "envs_per_launch": n,
                         "schedule": ("chunk queue: persistent grid of resident waves, two items per env step "
                                      "(DESIGN.md 3.1)" if queued else "one wave per env pair"),
                         "algo_bytes_per_env_step": abytes, "valu_busy": issue, "valu_flops": vflops,
                         # flat copies of the nested figures (the driver's record keeps flat keys only)
                         "valu_flops_frac": vflops["frac"] if vflops else None,
                         "valu_busy_frac": issue["frac"] if issue else None,
                         "wait_frac": issue["wait_frac"] if issue else None,
                         "traffic_over_algo": traffic / (abytes * n) if traffic else None,
                         "note": "latency-bound kernel (see valu_busy and DESIGN.md 3.1); HBM fraction reported per "
                                 "BASELINE.json; HIP events over the timed steps on the launch stream (the step "
                                 "kernel + the wide-tier launch, which exits at once when no env overflowed)"},
            "cpu_baseline": cpu_res,
            "sim_stats": stats,
            "sim_only_fp32": fp32_leg,
            "sim_only_episode": episodes,
            "rollout": rollout,
            "train": train_res,
            "gae": gae_res,
            "sim_only_stream_groups": grouped,
            "sim_only_tape": tape_leg,
            "dropin": dropin,
            "other_configs": config_legs,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def run_protocol(args, rank, world, ranks, make_env, make_tape, precondition, timed, stats_of):
    """SURVEY 8d protocol: per tape T0/T1/T2 and base seed {0,1,2}: reset (synchronized, as in
    training: all envs reset together every 667 steps), 1000 warm-up env steps, then 10000 timed."""
    res = {}
    for kind in ("T0", "T1", "T2"):
        for seed in (0, 1, 2):
            tp = make_tape(kind, 1024, args.envs, 100 * seed + rank)
            e = make_env(args.precision, seed)
            el, ms = timed(e, tp, 10000, 1000)
            res[f"{kind}/seed{seed}"] = dict(value=args.envs * 10000 * ranks / el, kernel_ms_per_launch=ms,
                                             stats=stats_of(e, tp, 11000))
            e.close()
            if rank == 0:
                print(json.dumps({kind + "/seed" + str(seed): res[f"{kind}/seed{seed}"]}), flush=True)
    if rank == 0:
        vals = [r["value"] for r in res.values()]
        print(json.dumps({"protocol": "SURVEY 8d: 1000 warm-up + 10000 timed env steps", "precision": args.precision,
                          "launches": "hs_step_tape, 500 steps per call" if args.protocol_tape else "one per env step",
                          "n_envs_per_gpu": args.envs, "n_gpus": ranks, "mean_value": float(np.mean(vals)),
                          "min_value": float(np.min(vals)), "runs": res}))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
