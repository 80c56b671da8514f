#!/usr/bin/env python
"""Headline benchmark: humanoid env steps/sec (whole node), 'stand' task -- BASELINE.json metric.

One "step" = one batched env step of every env on the rank: frame_skip=3 physics substeps
(full mj_step pipeline incl. contacts + Newton solve), the 352-float observation, the device
stand reward, termination/truncation and auto-reset -- one launch of the fused step kernel.
Workload (BASELINE.json configs[1]): 4096 humanoid.xml envs per GPU, stand reward,
frame_skip 3, duration 10; actions come from a pre-generated U(-1,1) action tape already
resident in HBM (sim-only mode).  N GPUs run N independent env shards (weak scaling, no
data-path collective).  rank 0 prints one JSON line.

Also reported (extra keys): the rollout mode (MLP[256,256] policy forward + Gaussian sampling
+ env step, all on device), the step-kernel roofline (HBM bytes vs 8 TB/s, measured live with
HIP events on the launch stream) and the CPU baseline (the reference's n_envs=8
SubprocVecEnv-style path, run on the oracle's fp64 C restatement of mj_step because MuJoCo is
not installable: kind "port").
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
XML = os.path.join(ROOT, "tests", "golden", "humanoid.xml")

N_ENVS_PER_GPU = 4096
FRAME_SKIP = 3
DURATION = 10.0
# algorithmic HBM bytes per env step of the fused kernel: read qpos 28 + qvel 27
# + qacc_warmstart 27 + time 1 + action 21 floats; write qpos/qvel/warmstart/time 83 + obs 352
# + reward 1 floats; + 2 B done flags
ALGO_BYTES_PER_ENV_STEP = (104 + 436) * 4 + 2
HBM_PEAK_GBS = 8000.0
PROFILE_TRAFFIC = os.path.join(ROOT, "profiles", "traffic_step_kernel.json")


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
                sample=f"{n_envs} worker processes x {vec_steps} env steps (stand, frame_skip 3, U(-1,1) actions, "
                       f"pipe IPC per step as SB3 SubprocVecEnv) on the fp64 oracle restatement of mj_step; "
                       f"{dt:.1f} s wall; host nproc={os.cpu_count()}")


# ----------------------------------------------------------------------------- GPU
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--envs", type=int, default=N_ENVS_PER_GPU, help="envs per GPU")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-rollout", action="store_true")
    ap.add_argument("--no-gae", action="store_true")
    ap.add_argument("--train-iters", type=int, default=2, help="PPO iterations of the train mode (0: skip)")
    ap.add_argument("--groups", default="1", help="stream groups for the headline run (1 = one launch per step)")
    ap.add_argument("--no-configs", action="store_true", help="skip the configs[3]/[4] legs")
    ap.add_argument("--no-fp64", action="store_true", help="skip the fp64 (parity-mode) sim-only leg")
    ap.add_argument("--free-groups", type=int, default=4, help="extra sim-only leg: this many free-running stream "
                                                                "groups (0: skip)")
    ap.add_argument("--dist-backend", default=os.environ.get("HSIM_BENCH_BACKEND", "nccl"),
                    help="nccl (= RCCL over xGMI; the real multi-GPU run) or gloo (multi-rank rehearsal on one GPU)")
    ap.add_argument("--cpu-steps", type=int, default=60000, help="vec steps of the CPU baseline (~13 s)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    cpu_res = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_res = cpu_baseline(vec_steps=args.cpu_steps)   # before any GPU/torch init (fork-safe)

    import torch
    import torch.distributed as dist
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
    red_dev = torch.device("cpu") if gloo else dev      # device of the timing reductions

    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    cfg = {"model_path": XML, "duration": DURATION, "reward_config": {"type": "stand"}, "frame_skip": FRAME_SKIP}
    model = HsModel(XML)
    n = args.envs
    groups = args.groups if args.groups == "auto" else int(args.groups)
    env = HumanoidVecEnv(cfg, n_envs=n, device=dev_index, precision=args.precision, seed=1000 + rank,
                         model=model, groups=groups)
    n_groups = len(env.batch._groups)
    env.reset_tensors()
    g = torch.Generator(device=dev).manual_seed(rank)
    tape_len = min(args.steps + args.warmup, 256)
    tape = (torch.rand(tape_len, n, model.nu, device=dev, generator=g) * 2 - 1).contiguous()

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for k in range(args.warmup):
        env.step_tensors(tape[k % tape_len])
    barrier()
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(args.steps):
        env.step_tensors(tape[(args.warmup + k) % tape_len])
    ev1.record(stream)
    barrier()
    elapsed = time.perf_counter() - t0
    step_ms = ev0.elapsed_time(ev1) / args.steps
    t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    total_env_steps = n * args.steps * world
    value = total_env_steps / elapsed
    warn = env.batch.warning.sum(0).tolist()
    aux = env.batch.aux
    stats = dict(mean_contacts=float(aux[:, 35].float().mean()), mean_rows=float(aux[:, 36].float().mean()),
                 mean_newton_iters=float(aux[:, 37].float().mean()), warnings=warn)

    # rollout mode: policy MLP[256,256] forward + sampling + env step (on device)
    rollout = None
    if not args.no_rollout:
        from mujocoposelearning_amd.ppo import ActorCritic, ppo_act
        pol = ActorCritic(env.batch.obs_dim, model.nu, (256, 256), activation=torch.nn.ReLU).to(dev)
        pol.pack_heads()
        ls = pol.log_std.detach()
        start = torch.zeros(n, device=dev)
        act, clip = torch.empty(n, model.nu, device=dev), torch.empty(n, model.nu, device=dev)
        logp, val, st_out = (torch.empty(n, device=dev) for _ in range(3))
        obs = env.batch.obs

        def policy_step(obs, k):
            # the PPO rollout's policy half (ppo.PPO._collect_rollouts_device): packed pi/vf GEMM
            # chain + hs_ppo_act (Gaussian sample, log-prob, clip, buffer writes), then the env
            mean, value = pol.heads(obs)
            ppo_act(mean, value, ls, start, 1 + rank, k, False, act, clip, logp, val, st_out)
            return env.step_tensors(clip)[0]

        with torch.no_grad():
            for k in range(5):
                obs = policy_step(obs, k)
            barrier()
            tr0 = time.perf_counter()
            rs = max(10, args.steps // 2)
            for k in range(rs):
                obs = policy_step(obs, 5 + k)
            barrier()
            rel = time.perf_counter() - tr0
        t = torch.tensor([rel], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rollout = dict(value=n * rs * world / float(t.item()), unit="env_steps/s",
                       note="policy MLP[256,256] (pi+vf, packed GEMM chain) forward + hs_ppo_act (diag-Gaussian sample, log-prob, clip) + env step")

    # extra sim-only leg: the same n envs as free-running stream groups (no per-step join; the
    # action tape is open-loop, so every env still takes exactly the same steps)
    grouped = None
    if args.free_groups > 1:
        envg = HumanoidVecEnv(cfg, n_envs=n, device=dev_index, precision=args.precision, seed=3000 + rank,
                              model=model, groups=args.free_groups)
        envg.reset_tensors()
        for k in range(args.warmup):
            envg.batch.step(tape[k % tape_len], join=False)
        envg.batch.join()
        barrier()
        tg = time.perf_counter()
        for k in range(args.steps):
            envg.batch.step(tape[(args.warmup + k) % tape_len], join=False)
        envg.batch.join()
        barrier()
        t = torch.tensor([time.perf_counter() - tg], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        grouped = dict(value=n * args.steps * world / float(t.item()), unit="env_steps/s", groups=args.free_groups,
                       note="same workload as value, envs split into free-running stream groups (HsBatch "
                            "join=False): one group's Newton tail overlaps the others' launches")
        envg.close()

    # parity-mode leg: the fp64 engine (the one the oracle parity tests pin at 1e-9 per stage and
    # that tracks the oracle over 1000 substeps) on the same workload and protocol as value
    fp64_leg = None
    if args.precision == "fp32" and not args.no_fp64:
        e64 = HumanoidVecEnv(cfg, n_envs=n, device=dev_index, precision="fp64", seed=5000 + rank, model=model)
        e64.reset_tensors()
        for k in range(min(args.warmup, 5)):
            e64.step_tensors(tape[k % tape_len])
        barrier()
        k64 = max(10, args.steps // 4)
        t64 = time.perf_counter()
        for k in range(k64):
            e64.step_tensors(tape[k % tape_len])
        barrier()
        t = torch.tensor([time.perf_counter() - t64], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        fp64_leg = dict(value=n * k64 * world / float(t.item()), unit="env_steps/s", dtype="f64", steps=k64,
                        note="same workload, fp64 engine (parity mode: <=1e-9 per stage vs the fp64 oracle, "
                             "tracks it over 1000 substeps; profiles/parity_report.md)")
        e64.close()

    # BASELINE.json configs[3] (kneeling reward, 4096 envs) and configs[4] (full-state obs, 8192
    # envs over 8 GPUs = 1024 per GPU): same sim-only protocol, one launch per step
    config_legs = None
    if not args.no_configs:
        def leg(cfg_x, n_x, label):
            e = HumanoidVecEnv(cfg_x, n_envs=n_x, device=dev_index, precision=args.precision, seed=4000 + rank,
                               model=model)
            e.reset_tensors()
            tp = tape[:, :n_x] if n_x <= n else (torch.rand(tape_len, n_x, model.nu, device=dev) * 2 - 1)
            for k in range(args.warmup):
                e.step_tensors(tp[k % tape_len])
            barrier()
            tl = time.perf_counter()
            ks = min(args.steps, 50)
            for k in range(ks):
                e.step_tensors(tp[(args.warmup + k) % tape_len])
            barrier()
            tt = torch.tensor([time.perf_counter() - tl], dtype=torch.float64, device=red_dev)
            if world > 1:
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            r = dict(value=n_x * ks * world / float(tt.item()), unit="env_steps/s", n_envs_per_gpu=n_x,
                     obs_dim=e.obs_dim, workload=label)
            e.close()
            return r
        config_legs = {
            "configs[3]": leg({**cfg, "reward_config": {"type": "kneeling"}}, n,
                              "kneeling (robust_kneeling_reward) device reward, humanoid.xml x 4096 envs per GPU"),
            "configs[4]": leg({**cfg, "full_state_obs": True}, 1024,
                              "full-state obs (+cfrc_ext[1:], 448 floats; subtree_linvel), 1024 envs per GPU "
                              "(8192 over 8 GPUs)"),
        }

    # roofline pass: the step kernel with all n envs in ONE launch per step (groups=1), HIP events on
    # the stream it is launched on -- the per-launch figure rocprofv3 reports for profiles/collect.sh
    if n_groups == 1:
        kernel_ms = step_ms
    else:
        env1 = HumanoidVecEnv(cfg, n_envs=n, device=dev_index, precision=args.precision, seed=2000 + rank,
                              model=model, groups=1)
        env1.reset_tensors()
        for k in range(args.warmup):
            env1.step_tensors(tape[k % tape_len])
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        rsteps = min(args.steps, 50)
        for k in range(rsteps):
            env1.step_tensors(tape[(args.warmup + k) % tape_len])
        e1.record(stream)
        torch.cuda.synchronize(dev)
        kernel_ms = e0.elapsed_time(e1) / rsteps
        env1.close()

    # train mode (SURVEY 8d iii): end-to-end on-device PPO iterations (rollout with the
    # MLP[256,256] policy + GAE + clipped-surrogate updates with the per-step gradient all-reduce)
    train_res = None
    if args.train_iters > 0:
        from mujocoposelearning_amd.ppo import PPO
        tk = dict(n_steps=32, batch_size=32768, n_epochs=4, learning_rate=3e-4,
                  policy_kwargs={"net_arch": {"pi": [256, 256], "vf": [256, 256]}, "activation_fn": "ReLU"})
        ppo = PPO(env, seed=0, world_size=world, rank=rank, **tk)
        ppo.learn(ppo.num_timesteps + n * tk["n_steps"] * world)          # warm-up iteration
        barrier()
        t_tr = time.perf_counter()
        ppo.learn(ppo.num_timesteps + args.train_iters * n * tk["n_steps"] * world)
        barrier()
        t = torch.tensor([time.perf_counter() - t_tr], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ts = float(t.item())
        train_res = dict(value=args.train_iters * n * tk["n_steps"] * world / ts, unit="env_steps/s",
                         iterations=args.train_iters, ms_per_iteration=ts / args.train_iters * 1e3,
                         config={k: v for k, v in tk.items() if k != "policy_kwargs"} | {"net_arch": "[256,256] ReLU"},
                         note="rollout (policy forward + env step) + GAE + 4 epochs of minibatch updates, "
                              "one gradient all-reduce per optimizer step")

    # GAE leg: the rollout-end reverse scan (hs_gae) over an n_steps=2048 x n-env buffer -- an
    # HBM-bound kernel (12 B read + 8 B written per element), timed with HIP events on its stream
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
        achieved = ALGO_BYTES_PER_ENV_STEP * n / (kernel_ms * 1e-3) / 1e9
        traffic = None
        issue = None
        if os.path.exists(PROFILE_TRAFFIC):
            try:
                tr = json.load(open(PROFILE_TRAFFIC))
                if tr.get("n_envs") == n and tr.get("precision") == args.precision:
                    traffic = tr.get("hbm_bytes_per_launch")
                    # VALU-issue view of the same kernel (what actually bounds it): VALU wave-instructions
                    # per launch from the profile's PMC pass over the live launch time; a SIMD issues one
                    # wave64 VALU op per 2 cycles at 2.4 GHz (MI355X_MICROARCH.md, wave scheduling)
                    valu = tr.get("sq", {}).get("SQ_INSTS_VALU")
                    if valu:
                        peak = 256 * 4 * 2.4e9 / 2
                        ach = valu / (kernel_ms * 1e-3)
                        issue = {"valu_wave_instr_per_s": ach, "peak": peak, "frac": ach / peak,
                                 "source": f"SQ_INSTS_VALU per launch from profiles ({tr.get('tag')})"}
            except Exception:
                traffic = None
        out = {
            "metric": "env steps/sec (whole node), humanoid 'stand' task, 1/2/4/8 MI355X",
            "value": value,
            "unit": "env_steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if args.precision == "fp32" else "f64",
            "data": "synthetic (reset distribution of custom_env.py:97-121; U(-1,1) action tape in HBM)",
            "config": {"workload": "configs[1]: humanoid.xml x 4096 envs per GPU, 'stand' reward, frame_skip 3, "
                                   "duration 10 (sim-only env steps)",
                       "n_envs_per_gpu": n, "n_envs_total": n * world, "frame_skip": FRAME_SKIP,
                       "reward": "stand", "parallelism": f"dp{world} (env shards, no collective)",
                       "stream_groups": n_groups},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "step_kernel<float,27>" if args.precision == "fp32" else "step_kernel<double,27>",
                         "kernel_ms_per_launch": kernel_ms, "envs_per_launch": n,
                         "algo_bytes_per_env_step": ALGO_BYTES_PER_ENV_STEP, "valu_issue": issue,
                         "note": "latency-bound kernel (see valu_issue and DESIGN.md 3.1); HBM fraction reported per BASELINE.json; measured "
                                 "with all envs in one launch per step (the headline value uses "
                                 f"{n_groups} stream groups; step time {step_ms:.3f} ms)"},
            "cpu_baseline": cpu_res,
            "rollout": rollout,
            "gae": gae_res,
            "sim_only_stream_groups": grouped,
            "sim_only_fp64": fp64_leg,
            "other_configs": config_legs,
            "train": train_res,
            "sim_stats": stats,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
