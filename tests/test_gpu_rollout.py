"""Fused PPO rollouts (hs_rollout, PPO._rollout_fused): SB3 collect_rollouts' per-step loop --
policy forward, Gaussian sample, clip, env step, buffer bookkeeping -- as one launch of the fp64
engine's chunk-queue kernel per chunk of steps, the pi net evaluated on each env's wave
(hs_kernels.hip policy_mean / step_pair).

Checked against the pieces the per-step path is built from:
* the env: stepping a copy of the batch with the rollout's own clipped actions, one hs_step per
  step, reproduces every buffered obs, reward and done flag BITWISE (auto-resets included);
* the policy: for every step, hs_ppo_act on the GEMM chain's mean with the same noise counter
  reproduces the buffered sample and log-prob to fp32 rounding of the mean (the in-kernel forward
  sums in another order), and episode_starts are the previous step's dones;
* the returns: episode_returns / ep_acc follow from the rewards and dones exactly;
* an overflow of the resident contact tier makes the library undo the launch and the trainer run
  the rest of the rollout step by step, with the same checks holding.
"""
import numpy as np
import pytest
import torch

from conftest import XML

pytestmark = pytest.mark.gpu

KW = dict(batch_size=1024, n_epochs=1, seed=0,
          policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [256, 256], "vf": [256, 256]}})


def _env(n, seed=0, full_state=False, duration=10.0):
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    cfg = {"model_path": XML, "duration": duration, "frame_skip": 3,
           "reward_config": {"type": "kneeling" if full_state else "stand"}}
    if full_state:
        cfg["full_state_obs"] = True        # BASELINE.json configs[4]: 448-value obs
    return HumanoidVecEnv(cfg, n_envs=n, model=HsModel(XML), seed=seed, precision="fp64")


def _stagger(env, episode_len=667):
    n = env.num_envs
    k = np.floor(np.arange(n) * episode_len / n)
    env.batch.t["time"].copy_(torch.as_tensor(k * 0.015 + 0.005, dtype=env.batch.dtype, device=env.device))
    env.batch.t["step_count"].copy_(torch.as_tensor(k, dtype=torch.int32, device=env.device))


def _check_rollout(ppo, replay, ep_acc0, start0, ctr0):
    from mujocoposelearning_amd.ppo import ppo_act
    b, T = ppo.buf, ppo.n_steps
    N = ppo.env.num_envs
    # 1. the env, stepped with the rollout's clipped actions one hs_step at a time: bitwise
    for t in range(T):
        obs, rew, term, trunc = replay.step_tensors(b["act"][t].clamp(-1, 1))
        nxt = b["obs"][t + 1] if t + 1 < T else ppo.obs
        assert torch.equal(obs.float(), nxt), t
        assert torch.equal(rew.float(), b["rew"][t]), t            # (no TimeLimit bootstrap at duration 10)
        assert torch.equal((term != 0) | (trunc != 0), b["done"][t]), t
    # 2. the policy: the per-step sampler on the GEMM chain's mean, same noise counters
    ls = ppo.policy.log_std.detach()
    base = torch.tensor([ctr0], dtype=torch.int64, device="cuda")
    zero = torch.zeros(N, device="cuda")
    for t in range(T):
        with torch.no_grad():
            mean = ppo.policy.net_forward(b["obs"][t], 0)
        out = [torch.empty(N, 21, device="cuda"), torch.empty(N, 21, device="cuda")] + \
              [torch.empty(N, device="cuda") for _ in range(3)]
        st_in = start0 if t == 0 else b["done"][t - 1].float()
        ppo_act(mean, zero, ls, st_in, ppo._noise_seed, t, False, *out, counter_base=base)
        assert torch.allclose(b["act"][t], out[0], rtol=1e-5, atol=2e-5), (t, float((b["act"][t] - out[0]).abs().max()))
        assert torch.allclose(b["logp"][t], out[2], rtol=1e-5, atol=2e-4), t
        assert torch.equal(b["start"][t], out[4]), t
    # 3. episode returns (float64 accumulation of the float rewards, reset at done)
    acc = ep_acc0.clone()
    for t in range(T):
        acc = acc + b["rew"][t].double()
        assert torch.equal(b["epret"][t], acc), t
        acc = torch.where(b["done"][t], torch.zeros_like(acc), acc)
    assert torch.equal(ppo.ep_acc, acc)
    assert torch.equal(ppo.episode_start, b["done"][T - 1].float())
    assert torch.equal(ppo._act_clip, b["act"][T - 1].clamp(-1, 1))


def _copy_env(src, dst):
    for k, v in src.batch.t.items():
        dst.batch.t[k].copy_(v)


@pytest.mark.parametrize("n,T,full,duration", [(4096, 20, False, 10.0), (777, 30, False, 10.0),
                                               (1024, 16, True, 10.0), (512, 80, False, 0.5)])
def test_fused_rollout_matches_env_replay_and_policy(n, T, full, duration):
    """The last case: 0.5 s episodes (33 env steps), so hs_rollout_max_steps is 32 and the 80-step
    rollout is three launches, with every env auto-resetting two or three times."""
    from mujocoposelearning_amd.ppo import PPO
    env, replay = _env(n, full_state=full, duration=duration), _env(n, full_state=full, duration=duration)
    ppo = PPO(env, n_steps=T, **KW)
    ppo.policy.pack_heads()
    assert ppo._fused_rollout_args() is not None
    if duration < 1.0:
        from mujocoposelearning_amd import _lib
        assert _lib.check(_lib.lib().hs_rollout_max_steps(env.rollout_handle())) < T // 2
    _stagger(env, round(duration / 0.015))
    for it in range(2):            # the second rollout continues from the first (obs, ep_acc, starts, noise)
        _copy_env(env, replay)
        ep_acc0, start0, ctr0 = ppo.ep_acc.clone(), ppo.episode_start.clone(), int(ppo._noise_ctr.item())
        ppo.collect_rollouts()
        torch.cuda.synchronize()
        assert getattr(ppo, "fused_fallbacks", 0) == 0
        assert int(ppo.buf["done"].sum()) > 0                     # episodes ended inside the rollout
        _check_rollout(ppo, replay, ep_acc0, start0, ctr0)
    env.close()
    replay.close()


@pytest.mark.parametrize("T", [6, 1])
def test_fused_rollout_overflow_falls_back_step_by_step(T):
    """T = 1: a one-step rollout launch, whose only step is also its last (it hands nothing over):
    the overflow must still undo the launch."""
    from oracle.oracle import Oracle
    from test_gpu_contacts import lying_states
    from mujocoposelearning_amd.ppo import PPO
    n = 4096
    q = np.stack(lying_states(Oracle(XML), 16, seed=11))
    idx = np.arange(16) * 255 + 7
    env, replay = _env(n), _env(n)
    ppo = PPO(env, n_steps=T, **KW)
    st = env.batch.get_state()
    st["qpos"][idx] = q
    st["qvel"][idx] = 0.0
    st["qacc_warmstart"][idx] = 0.0
    env.batch.set_state(**st)
    _copy_env(env, replay)
    ep_acc0, start0, ctr0 = ppo.ep_acc.clone(), ppo.episode_start.clone(), int(ppo._noise_ctr.item())
    ppo.collect_rollouts()
    torch.cuda.synchronize()
    assert getattr(ppo, "fused_fallbacks", 0) == 1 and env.batch.tape_aborts() == 1
    assert env.batch.wide_reruns() >= len(idx)
    _check_rollout(ppo, replay, ep_acc0, start0, ctr0)
    env.close()
    replay.close()


def test_hs_rollout_refuses_what_it_cannot_run():
    """hs_rollout fails loudly (HsimError with the reason) for an fp32 batch and for a policy whose
    obs width is not the batch's, and PPO falls back to the per-step path for them."""
    import ctypes as C

    from mujocoposelearning_amd import _lib
    from mujocoposelearning_amd._lib import HsimError
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.ppo import PPO
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    env32 = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3},
                           n_envs=64, model=HsModel(XML), seed=0, precision="fp32")
    assert env32.rollout_handle() is None
    p32 = PPO(env32, n_steps=4, **KW)
    p32.policy.pack_heads()
    assert p32._fused_rollout_args() is None
    env = _env(64)
    p = PPO(env, n_steps=4, **KW)
    p.policy.pack_heads()
    h, pol, keep = p._fused_rollout_args()
    b = p.buf
    rb = _lib.hs_rollout_bufs(b["obs"].data_ptr(), p.obs.data_ptr(), b["act"].data_ptr(), b["logp"].data_ptr(),
                              b["start"].data_ptr(), b["rew"].data_ptr(), b["done"].data_ptr(), b["epret"].data_ptr(),
                              b["boot"].data_ptr(), b["tobs"].data_ptr(), p.ep_acc.data_ptr(),
                              p.episode_start.data_ptr(), p._act_clip.data_ptr(), p._noise_ctr.data_ptr(), 1, 0)
    bad = _lib.hs_policy(*[t.data_ptr() for t in keep], 512, 348, 21)          # obs width != the batch's
    with pytest.raises(HsimError, match="policy shape"):
        _lib.check(_lib.lib().hs_rollout(h, C.byref(bad), C.byref(rb), 0, 4, 4, None))
    h32 = env32.batch._groups[0][0]
    with pytest.raises(HsimError, match="fp64"):
        _lib.check(_lib.lib().hs_rollout(h32, C.byref(pol), C.byref(rb), 0, 4, 4, None))
    with pytest.raises(HsimError, match="n_steps"):
        _lib.check(_lib.lib().hs_rollout(h, C.byref(pol), C.byref(rb), 0, 5, 4, None))
    env.close()
    env32.close()


def _fused_world2_worker(rank, world, port, out_dir):
    import os
    import torch.distributed as dist
    from mujocoposelearning_amd.ppo import PPO
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)     # both ranks share the one GPU
    try:
        env = _env(512, seed=10 + rank)
        ppo = PPO(env, n_steps=16, batch_size=2048, n_epochs=2, seed=0,
                  policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [256, 256], "vf": [256, 256]}})
        ppo.learn(3 * 16 * 512 * world)
        flat = torch.cat([q.detach().reshape(-1) for q in ppo.policy.parameters()]).cpu()
        torch.save({"w": flat, "fused": ppo._fused_rollout_args() is not None,
                    "fallbacks": getattr(ppo, "fused_fallbacks", 0), "steps": ppo.num_timesteps},
                   os.path.join(out_dir, f"r{rank}.pt"))
        env.close()
    finally:
        dist.destroy_process_group()


def test_fused_rollouts_multi_rank_lockstep(tmp_path):
    """world 2 (gloo rehearsal, two ranks on one GPU, different env seeds): PPO.learn with fused
    rollouts on both ranks, one gradient all-reduce per optimizer step -- both ranks end with the
    same weights (train_sb3.py:203's envs sharded over GPUs)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_fused_world2_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(2)]
    assert r[0]["fused"] and r[1]["fused"] and r[0]["fallbacks"] == r[1]["fallbacks"] == 0
    assert r[0]["steps"] == r[1]["steps"] == 3 * 16 * 512 * 2
    assert torch.equal(r[0]["w"], r[1]["w"]), "ranks diverged"
