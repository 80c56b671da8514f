"""CPU tests of the on-device PPO module (ppo.py) and the train_humanoid mirror (train.py).

SB3 is not installed here: PPO parity with SB3 2.3.2 is unpinned.  The tests
check the restated pieces that have an exact definition (GAE reverse scan, parameter count of
the [256,256] MlpPolicy, SB3's init) and the multi-process behaviour (one gradient all-reduce
per optimizer step over gloo, identical weights on every rank).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from mujocoposelearning_amd.ppo import PPO, ActorCritic, gae
from mujocoposelearning_amd.train import _resolve_activation, env_config_from_kwargs, shard_envs


class ToyEnv:
    """Device vec-env protocol stand-in on the CPU: reward = -|a - tanh(W obs)|^2, episodes of
    ``horizon`` steps ending by truncation (exercises the timeout bootstrap)."""

    def __init__(self, n=16, obs_dim=6, act_dim=3, horizon=8, seed=0):
        g = torch.Generator().manual_seed(1234)          # same task on every rank
        self.W = torch.randn(act_dim, obs_dim, generator=g) * 0.5
        self.g = torch.Generator().manual_seed(seed)
        self.num_envs, self.obs_dim, self.act_dim, self.device = n, obs_dim, act_dim, torch.device("cpu")
        self.horizon = horizon
        self.t = torch.zeros(n, dtype=torch.long)
        self.obs = torch.randn(n, obs_dim, generator=self.g)
        self.terminal_obs = torch.zeros(n, obs_dim)

    def reset_tensors(self):
        self.t.zero_()
        self.obs = torch.randn(self.num_envs, self.obs_dim, generator=self.g)
        return self.obs

    def step_tensors(self, a):
        target = torch.tanh(self.obs @ self.W.T)
        rew = -((a - target) ** 2).sum(-1)
        self.t += 1
        trunc = self.t >= self.horizon
        term = torch.zeros_like(trunc)
        nxt = torch.randn(self.num_envs, self.obs_dim, generator=self.g)
        self.terminal_obs = nxt.clone()
        fresh = torch.randn(self.num_envs, self.obs_dim, generator=self.g)
        self.obs = torch.where(trunc[:, None], fresh, nxt)
        self.t[trunc] = 0
        return self.obs, rew, term, trunc


def _sb3_gae(rewards, values, episode_starts, last_values, dones, gamma, lam):
    """SB3 2.3.2 RolloutBuffer.compute_returns_and_advantage (stable_baselines3/common/buffers.py),
    restated with scalar loops."""
    T, N = rewards.shape
    adv = np.zeros((T, N))
    for n in range(N):
        last = 0.0
        for step in reversed(range(T)):
            if step == T - 1:
                nnt, nv = 1.0 - dones[n], last_values[n]
            else:
                nnt, nv = 1.0 - episode_starts[step + 1, n], values[step + 1, n]
            delta = rewards[step, n] + gamma * nv * nnt - values[step, n]
            last = delta + gamma * lam * nnt * last
            adv[step, n] = last
    return adv, adv + values


def test_gae_matches_sb3_restatement():
    rng = np.random.default_rng(0)
    T, N = 37, 5
    r, v = rng.normal(size=(T, N)), rng.normal(size=(T, N))
    starts = (rng.uniform(size=(T, N)) < 0.1).astype(np.float64)
    lv, ld = rng.normal(size=N), (rng.uniform(size=N) < 0.3).astype(np.float64)
    ea, er = _sb3_gae(r, v, starts, lv, ld, 0.99, 0.95)
    t = lambda x: torch.tensor(x, dtype=torch.float64)
    adv, ret = gae(t(r), t(v), t(starts), t(lv), t(ld), 0.99, 0.95)
    np.testing.assert_allclose(adv.numpy(), ea, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(ret.numpy(), er, rtol=1e-12, atol=1e-12)


def test_policy_param_count_and_init():
    # pi 161,578 + vf 156,417 = 317,995 parameters at net_arch [256, 256]
    p = ActorCritic(352, 21, [256, 256], [256, 256])
    assert sum(x.numel() for x in p.parameters()) == 317_995
    assert torch.all(p.log_std == 0)
    for lin in (p.action_net, p.value_net):
        assert torch.all(lin.bias == 0)
    w = p.action_net.weight                  # orthogonal init with gain 0.01 (rows orthonormal * gain)
    np.testing.assert_allclose((w @ w.T).detach().numpy(), 1e-4 * np.eye(21), atol=1e-9)


def test_shard_envs_and_config_mirror():
    for n, w in ((32768, 8), (8192, 8), (10, 3), (5, 5)):
        ranges = [shard_envs(n, w, r) for r in range(w)]
        assert ranges[0][0] == 0 and ranges[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
        sizes = [b - a for a, b in ranges]
        assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_envs(3, 4, 0)
    cfg = env_config_from_kwargs({"reward_function": "stand", "frame_skip": 3})
    assert cfg["duration"] == 10.0 and cfg["reward_config"] == {"type": "stand"} and cfg["frame_skip"] == 3
    assert env_config_from_kwargs({})["reward_config"]["type"] == "walk"      # train_sb3.py:189 default
    kw = _resolve_activation({"policy_kwargs": {"activation_fn": "ReLU", "net_arch": {"pi": [8], "vf": [8]}}})
    assert kw["policy_kwargs"]["activation_fn"] is torch.nn.ReLU


def test_ppo_learns_toy_task():
    env = ToyEnv(n=32)
    model = PPO(env, learning_rate=3e-3, n_steps=16, batch_size=64, n_epochs=4,
                policy_kwargs={"net_arch": {"pi": [32, 32], "vf": [32, 32]}, "activation_fn": torch.nn.Tanh})
    rets = []      # mean raw episode return of the last 100 episodes, per iteration
    model.learn(total_timesteps=32 * 16 * 25,
                callback=lambda m: rets.append(m.logger["ep_rew_mean"]) or True)
    first, last = np.mean(rets[:3]), np.mean(rets[-3:])
    assert model.num_timesteps == 32 * 16 * 25
    assert last > first + 2.0, (first, last)
    assert model.ep_returns, "truncated episodes must be recorded"


def test_save_load_roundtrip(tmp_path):
    env = ToyEnv(n=4)
    kw = dict(n_steps=4, batch_size=8, n_epochs=1, policy_kwargs={"net_arch": [8, 8]})
    a = PPO(env, **kw)
    a.learn(16)
    path = tmp_path / "m.pt"
    a.save(path)
    b = PPO(ToyEnv(n=4), seed=5, **kw).load(path)
    for pa, pb in zip(a.policy.parameters(), b.policy.parameters()):
        assert torch.equal(pa, pb)
    assert b.num_timesteps == a.num_timesteps


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _dist_worker(rank, world, port, out_dir, n_envs=None, stop_rank=None):
    """One rank of a gloo world: a ToyEnv holding this rank's shard of ``n_envs`` envs (8 per
    rank when None).  ``stop_rank``: that rank's callback alone asks to stop after iteration 1."""
    import torch.distributed as dist
    from mujocoposelearning_amd.train import init_distributed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    assert init_distributed("gloo") == (world, rank, rank)
    calls = []
    real = dist.all_reduce

    def counting(t, *a, **k):
        calls.append(t.numel())
        return real(t, *a, **k)
    dist.all_reduce = counting
    try:
        lo, hi = shard_envs(n_envs, world, rank) if n_envs else (8 * rank, 8 * rank + 8)
        env = ToyEnv(n=hi - lo, seed=100 + rank)            # different data per rank (env shard)
        model = PPO(env, n_steps=8, batch_size=16, n_epochs=2,
                    policy_kwargs={"net_arch": {"pi": [16, 16], "vf": [16, 16]}})
        assert model.world_size == world and model.rank == rank
        total = n_envs or 8 * world
        cb = (lambda m: not (rank == stop_rank and m.logger["iteration"] == 1)) if stop_rank is not None else None
        model.learn(total_timesteps=8 * total * 2, callback=cb)
        flat = torch.cat([p.detach().reshape(-1) for p in model.policy.parameters()])
        torch.save({"flat": flat, "calls": calls, "steps": model.num_timesteps, "n_mb": model.n_minibatches,
                    "bounds": model._mb_bounds, "w": model._mb_weight},
                   os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.all_reduce = real
        dist.destroy_process_group()


def _run_world(tmp_path, world, **kw):
    port = _free_port()
    mp.start_processes(_dist_worker, args=(world, port, str(tmp_path), kw.get("n_envs"), kw.get("stop_rank")),
                       nprocs=world, join=True, start_method="spawn")
    return [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(world)]


def test_gloo_world2_one_allreduce_per_step_identical_weights(tmp_path):
    world = 2
    r = _run_world(tmp_path, world)
    assert torch.equal(r[0]["flat"], r[1]["flat"]), "ranks diverged: gradient all-reduce missing"
    n_params = r[0]["flat"].numel()
    # 2 iterations x 2 epochs x (64 samples / 16 per minibatch) = 16 optimizer steps, one bucket each
    for x in r:
        assert [c for c in x["calls"] if c == n_params] == [n_params] * 16
        assert x["steps"] == 8 * 8 * world * 2
        assert x["w"] == [0.5] * 4


def test_gloo_world3_uneven_shards_stay_in_lockstep(tmp_path):
    """n_envs=10 over 3 ranks (shards 4/3/3, train_sb3.py:203 accepts any n_envs): every rank runs
    the same number of minibatches and all-reduces, the global timestep count, and ends with the
    same weights; gradients are weighted by the rank's sample share."""
    world = 3
    r = _run_world(tmp_path, world, n_envs=10)
    n_params = r[0]["flat"].numel()
    for x in r[1:]:
        assert torch.equal(r[0]["flat"], x["flat"]), "ranks diverged"
        assert x["calls"] == r[0]["calls"], "ranks issued different collectives (an RCCL hang)"
    for i, x in enumerate(r):
        assert x["steps"] == 8 * 10 * 2                    # global env count, not world x local
        assert x["n_mb"] == 2                              # max over ranks of ceil(8 * N_r / 16)
        m = 8 * (4 if i == 0 else 3)
        assert x["bounds"] == [0, m // 2, m]
        assert all(abs(w - m / 80) < 1e-15 for w in x["w"])
        # 2 iterations x 2 epochs x 2 minibatches
        assert [c for c in x["calls"] if c == n_params] == [n_params] * 8
    for j in range(2):
        assert abs(sum(x["w"][j] for x in r) - 1.0) < 1e-12


def test_minibatch_weights_uneven_chunks_sum_to_one():
    """Shards 3/2/2 x 5 steps over 3 minibatches: chunk sizes 5/5/5, 3/3/4, 3/3/4 -- each
    minibatch's weights are the chunks' shares of that global minibatch (11, 11, 13 samples)."""
    from mujocoposelearning_amd.ppo import minibatch_weights
    w = [minibatch_weights([3, 2, 2], r, 5, 3) for r in range(3)]
    assert w[0] == [5 / 11, 5 / 11, 5 / 13]
    assert w[1] == [3 / 11, 3 / 11, 4 / 13]
    for j in range(3):
        assert abs(sum(x[j] for x in w) - 1.0) < 1e-15


def test_gloo_world2_callback_stop_on_one_rank_stops_all(tmp_path):
    r = _run_world(tmp_path, 2, stop_rank=1)
    assert r[0]["steps"] == r[1]["steps"] == 8 * 16          # both left after iteration 1
    assert r[0]["calls"] == r[1]["calls"]


def test_init_distributed_without_launcher_and_without_gpu(monkeypatch):
    from mujocoposelearning_amd.train import init_distributed
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert init_distributed() == (1, 0, 0)
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError, match="no GPU"):
            init_distributed()


def test_ppo_sync_without_group_raises():
    with pytest.raises(RuntimeError, match="process group"):
        PPO(ToyEnv(n=4), n_steps=4, batch_size=8, world_size=2, rank=0)


def test_minibatch_plan_world1_is_sb3():
    m = PPO(ToyEnv(n=5), n_steps=4, batch_size=8)           # M = 20: 8, 8, 4 (SB3's short last batch)
    assert m._mb_bounds == [0, 8, 16, 20] and m._chunk is None and m.n_envs_global == 5
    m = PPO(ToyEnv(n=4), n_steps=4, batch_size=8)
    assert m._mb_bounds == [0, 8, 16] and m._chunk == 8


def test_train_module_cli_loads_reference_style_config(tmp_path):
    from mujocoposelearning_amd.train import load_config_from_file
    p = tmp_path / "config.py"
    p.write_text('config = {"env_kwargs": {"n_envs": 8, "reward_function": "stand"}, '
                 '"ppo_kwargs": {"policy_kwargs": {"activation_fn": "ReLU"}}}\n')
    cfg = load_config_from_file(str(p))
    assert cfg["env_kwargs"]["n_envs"] == 8
    bad = tmp_path / "bad.py"
    bad.write_text("x = 1\n")
    with pytest.raises(ValueError):
        load_config_from_file(str(bad))


SB3_MLP_KEYS = {   # ActorCriticPolicy state_dict of MlpPolicy, net_arch=dict(pi=[256,256], vf=[256,256])
    "log_std": (21,),
    "mlp_extractor.policy_net.0.weight": (256, 352), "mlp_extractor.policy_net.0.bias": (256,),
    "mlp_extractor.policy_net.2.weight": (256, 256), "mlp_extractor.policy_net.2.bias": (256,),
    "mlp_extractor.value_net.0.weight": (256, 352), "mlp_extractor.value_net.0.bias": (256,),
    "mlp_extractor.value_net.2.weight": (256, 256), "mlp_extractor.value_net.2.bias": (256,),
    "action_net.weight": (21, 256), "action_net.bias": (21,),
    "value_net.weight": (1, 256), "value_net.bias": (1,),
}


def test_sb3_zip_layout_names_and_optimizer_order(tmp_path):
    import zipfile
    import io
    from mujocoposelearning_amd.sb3_format import save_sb3_zip, to_sb3_names
    p = ActorCritic(352, 21, [256, 256], [256, 256])
    names = list(to_sb3_names(p.state_dict()))
    assert {k: tuple(v.shape) for k, v in to_sb3_names(p.state_dict()).items()} == SB3_MLP_KEYS
    # SB3 parameters() order: the policy's own log_std, then mlp_extractor (pi, vf), action_net, value_net
    order = [n for n, _ in p.named_parameters()]
    assert [k for k in to_sb3_names(dict.fromkeys(order))] == [
        "log_std", "mlp_extractor.policy_net.0.weight", "mlp_extractor.policy_net.0.bias",
        "mlp_extractor.policy_net.2.weight", "mlp_extractor.policy_net.2.bias", "mlp_extractor.value_net.0.weight",
        "mlp_extractor.value_net.0.bias", "mlp_extractor.value_net.2.weight", "mlp_extractor.value_net.2.bias",
        "action_net.weight", "action_net.bias", "value_net.weight", "value_net.bias"]
    opt = torch.optim.Adam(p.parameters(), lr=3e-4, eps=1e-5)
    path = save_sb3_zip(tmp_path / "final_model", p, opt, {"gamma": 0.99})
    assert path.endswith("final_model.zip")
    with zipfile.ZipFile(path) as z:
        assert {"data", "policy.pth", "policy.optimizer.pth", "pytorch_variables.pth",
                "_stable_baselines3_version", "system_info.txt"} <= set(z.namelist())
        sd = torch.load(io.BytesIO(z.read("policy.pth")), weights_only=True)
        assert set(sd) == set(names)
        assert z.read("_stable_baselines3_version") == b"2.3.2"
        od = torch.load(io.BytesIO(z.read("policy.optimizer.pth")), weights_only=True)
        assert od["param_groups"][0]["eps"] == 1e-5 and len(od["param_groups"][0]["params"]) == 13


def test_load_sb3_named_zip_and_predict(tmp_path):
    """A zip written with SB3's names (as SB3's own save produces) loads into our PPO."""
    import zipfile
    import io
    env = ToyEnv(n=4)
    model = PPO(env, n_steps=4, batch_size=8, policy_kwargs={"net_arch": {"pi": [8, 8], "vf": [8, 8]}})
    src = ActorCritic(6, 3, [8, 8], [8, 8], torch.nn.Tanh)
    with torch.no_grad():
        for prm in src.parameters():
            prm.normal_()
    sd = {k.replace("pi_net.", "mlp_extractor.policy_net.").replace("vf_net.", "mlp_extractor.value_net."): v
          for k, v in src.state_dict().items()}
    buf = io.BytesIO()
    torch.save(sd, buf)
    path = tmp_path / "sb3_model.zip"
    with zipfile.ZipFile(path, "w") as z:
        z.writestr("policy.pth", buf.getvalue())
        z.writestr("data", '{"num_timesteps": 1234, "policy_class": {":type:": "<class \'abc.ABCMeta\'>", '
                           '":serialized:": "gAWVOwAAAAAAAACM"}}')
    model.load(path)
    assert model.num_timesteps == 1234
    for a, b in zip(model.policy.parameters(), src.parameters()):
        assert torch.equal(a, b)
    obs = np.random.default_rng(0).normal(size=(5, 6))
    act, state = model.predict(obs, deterministic=True)
    assert state is None and act.shape == (5, 3) and np.all(np.abs(act) <= 1)
    mean = src(torch.tensor(obs, dtype=torch.float32))[0].clamp(-1, 1).detach().numpy()
    np.testing.assert_allclose(act, mean, rtol=1e-6, atol=1e-6)
    a1, _ = model.predict(obs[0], deterministic=True)
    assert a1.shape == (3,)


@pytest.mark.gpu
def test_splitk_linear_grads_match_dense_linear():
    """The split-K weight gradient (ppo.Linear on large device minibatches) equals nn.Linear's
    gradient to fp32 summation-order tolerance (rel 1e-4 of the gradient's scale)."""
    from mujocoposelearning_amd import ppo as ppo_mod
    torch.manual_seed(0)
    dev = "cuda"
    for rows, out in ((2 * ppo_mod._SPLITK_ROWS, 256), (16 * ppo_mod._SPLITK_ROWS, 256),
                      (16 * ppo_mod._SPLITK_ROWS, 1)):
        lin = ppo_mod.Linear(352, out).to(dev)
        ref = torch.nn.Linear(352, out).to(dev)
        ref.load_state_dict(lin.state_dict())
        x = torch.randn(rows, 352, device=dev, requires_grad=True)
        g = torch.randn(rows, out, device=dev)
        (lin(x) * g).sum().backward()
        gx, gw, gb = x.grad.clone(), lin.weight.grad, lin.bias.grad
        x.grad = None
        (ref(x) * g).sum().backward()
        for a, b in ((gx, x.grad), (gw, ref.weight.grad), (gb, ref.bias.grad)):
            assert torch.allclose(a, b, rtol=1e-4, atol=1e-4 * float(b.abs().max())), float((a - b).abs().max())


def test_packed_heads_match_two_nets():
    """ActorCritic.pack_heads/heads (the rollout forward as one stacked GEMM chain) equals the
    separate pi/vf MLP forward; unequal nets fall back to the two-net forward."""
    torch.manual_seed(0)
    pol = ActorCritic(352, 21, (256, 256), (256, 256), torch.nn.ReLU)
    for p in pol.parameters():                    # non-trivial biases too
        torch.nn.init.normal_(p, std=0.05)
    obs = torch.randn(64, 352)
    assert pol.pack_heads() is not None
    mean, value = pol.heads(obs)
    rm, rv = pol(obs)
    assert torch.allclose(mean, rm, atol=1e-5) and torch.allclose(value, rv, atol=1e-5)
    pol2 = ActorCritic(352, 21, (64, 64), (32,), torch.nn.ReLU)
    assert pol2.pack_heads() is None
    m2, v2 = pol2.heads(obs)
    r2m, r2v = pol2(obs)
    assert torch.equal(m2, r2m) and torch.equal(v2, r2v)


@pytest.mark.gpu
def test_fused_linear_relu_matches_modules():
    """mlp_forward's fused Linear+ReLU (GEMM epilogue + masked split-K backward) equals the
    module-by-module Linear, ReLU forward and gradients."""
    from mujocoposelearning_amd import ppo as ppo_mod
    torch.manual_seed(0)
    seq = torch.nn.Sequential(ppo_mod.Linear(352, 256), torch.nn.ReLU(), ppo_mod.Linear(256, 256),
                              torch.nn.ReLU()).cuda()
    x = torch.randn(4 * ppo_mod._SPLITK_ROWS, 352, device="cuda")
    g = torch.randn(x.shape[0], 256, device="cuda")
    out = []
    for fused in (True, False):
        seq.zero_grad()
        y = ppo_mod.mlp_forward(seq, x) if fused else seq(x)
        (y * g).sum().backward()
        out.append([y.detach()] + [p.grad.clone() for p in seq.parameters()])
    for a, b in zip(*out):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-4 * float(b.abs().max())), float((a - b).abs().max())


def test_net_forward_matches_heads():
    """ActorCritic.net_forward (one net from the packed weights, used by the device rollout) equals
    the corresponding output of heads() / forward()."""
    torch.manual_seed(1)
    pol = ActorCritic(352, 21, (256, 256), (256, 256), torch.nn.ReLU)
    for p in pol.parameters():
        torch.nn.init.normal_(p, std=0.05)
    obs = torch.randn(32, 352)
    pol.pack_heads()
    mean, value = pol.heads(obs)
    assert torch.allclose(pol.net_forward(obs, 0), mean, atol=1e-5)
    assert torch.allclose(pol.net_forward(obs, 1), value, atol=1e-5)


# ---- equal-result check of the multi-rank update (train_sb3.py:203,208-214) ------------
EQ_T, EQ_BS, EQ_STEPS = 4, 6, 2          # n_steps, per-rank batch_size, optimizer steps compared


def _eq_data(rank, m, policy, gen_seed=1000):
    """Rank ``rank``'s synthetic rollout slice (m samples): obs, actions, old log-probs (the initial
    policy's, perturbed so that some ratios clip), advantages, returns."""
    g = torch.Generator().manual_seed(gen_seed + rank)
    obs = torch.randn(m, 6, generator=g)
    act = torch.randn(m, 3, generator=g)
    with torch.no_grad():
        mean, _ = policy(obs)
        old = policy._logp(mean, act) + 0.3 * torch.randn(m, generator=g)
    adv = 2.0 * torch.randn(m, generator=g) + 0.5
    ret = torch.randn(m, generator=g)
    return obs, act, old, adv, ret


def _eq_worker(rank, world, port, out_dir, shards):
    """One rank: for normalize_advantage in (True, False), EQ_STEPS optimizer steps on the rank's
    minibatch chunks j = 0, 1, ... (in order, unpermuted) through the product's update path
    (_minibatch_loss -> backward -> weighted flat all-reduce -> clip + Adam); saves the all-reduced
    gradient and the parameters after each step."""
    import torch.distributed as dist
    from mujocoposelearning_amd.train import init_distributed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    init_distributed("gloo")
    try:
        out = {}
        for norm in (True, False):
            m = PPO(ToyEnv(n=shards[rank], seed=rank), n_steps=EQ_T, batch_size=EQ_BS, n_epochs=1, seed=3,
                    ent_coef=0.01, normalize_advantage=norm, policy_kwargs={"net_arch": {"pi": [16, 16], "vf": [16, 16]}})
            data = _eq_data(rank, EQ_T * shards[rank], m.policy)
            grads, params = [], []
            for j in range(EQ_STEPS):
                m.grad_weight = m._mb_weight[j]
                idx = torch.arange(m._mb_bounds[j], m._mb_bounds[j + 1])
                loss, _, _ = m._minibatch_loss(*data, idx)
                m.opt.zero_grad(set_to_none=True)
                loss.backward()
                m._allreduce_grads()
                grads.append(torch.cat([p.grad.reshape(-1) for p in m.policy.parameters()]).clone())
                m._clip_and_step()
                params.append(torch.cat([p.detach().reshape(-1) for p in m.policy.parameters()]).clone())
            out[norm] = {"grads": grads, "params": params, "bounds": m._mb_bounds, "w": m._mb_weight}
        torch.save(out, os.path.join(out_dir, f"eq{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _world1_reference(shards, norm, bounds):
    """World 1 on the concatenation of every rank's chunk j: one PPO whose loss is the plain mean over
    the union (normalize_advantage off).  With ``norm`` the advantages are first normalised per rank
    chunk exactly as each rank normalises its own (SB3's per-minibatch mean / unbiased std + 1e-8), so
    the union's loss is the one the world-W step optimises; without it, raw advantages on both sides."""
    m = PPO(ToyEnv(n=sum(shards)), n_steps=EQ_T, batch_size=EQ_BS, n_epochs=1, seed=3, ent_coef=0.01,
            normalize_advantage=False, world_size=1, rank=0, sync_grads=False,
            policy_kwargs={"net_arch": {"pi": [16, 16], "vf": [16, 16]}})
    p0 = PPO(ToyEnv(n=1), n_steps=EQ_T, batch_size=EQ_BS, seed=3, world_size=1, rank=0, sync_grads=False,
             policy_kwargs={"net_arch": {"pi": [16, 16], "vf": [16, 16]}}).policy   # the initial weights
    data = [_eq_data(r, EQ_T * shards[r], p0) for r in range(len(shards))]
    grads, params = [], []
    for j in range(EQ_STEPS):
        parts = []
        for r, (obs, act, old, adv, ret) in enumerate(data):
            s, e = bounds[r][j], bounds[r][j + 1]
            a = adv[s:e]
            if norm and a.numel() > 1:
                a = (a - a.mean()) / (a.std() + 1e-8)
            parts.append((obs[s:e], act[s:e], old[s:e], a, ret[s:e]))
        union = [torch.cat([p[k] for p in parts]) for k in range(5)]
        loss, _, _ = m._minibatch_loss(*union, torch.arange(union[0].shape[0]))
        m.opt.zero_grad(set_to_none=True)
        loss.backward()
        grads.append(torch.cat([p.grad.reshape(-1) for p in m.policy.parameters()]).clone())
        m._clip_and_step()
        params.append(torch.cat([p.detach().reshape(-1) for p in m.policy.parameters()]).clone())
    return grads, params


@pytest.mark.parametrize("shards", [[4, 4], [5, 3], [2] * 8, [3, 2, 2, 3, 2, 1, 2, 2]],
                         ids=["w2-equal", "w2-uneven", "w8-equal", "w8-uneven"])
def test_gloo_multirank_step_equals_world1_step_on_the_union(tmp_path, shards):
    """SURVEY 4.6's equal-result check of the one collective on the path (train_sb3.py:203 fan-out,
    :208-214 update): after each optimizer step, the share-weighted all-reduced gradient of a world-W
    run equals the world-1 gradient of the plain mean loss over the union of the ranks' minibatch
    chunks, and so do the parameters after clip_grad_norm + Adam, to 1e-6 relative.  Equal shards
    (configs[2]'s 32768 envs / 8 ranks in shape) and uneven ones (chunk sizes differ by rank and by
    minibatch, so a wrong share weight shows).  Advantage normalisation: on (per rank chunk, matched
    on the world-1 side by normalising each chunk's advantages before the union) and off."""
    world = len(shards)
    port = _free_port()
    mp.start_processes(_eq_worker, args=(world, port, str(tmp_path), shards), nprocs=world, join=True,
                       start_method="spawn")
    ranks = [torch.load(tmp_path / f"eq{r}.pt", weights_only=True) for r in range(world)]
    for norm in (True, False):
        bounds = [x[norm]["bounds"] for x in ranks]
        for j in range(EQ_STEPS):
            assert abs(sum(x[norm]["w"][j] for x in ranks) - 1.0) < 1e-12
        g1, p1 = _world1_reference(shards, norm, bounds)
        for j in range(EQ_STEPS):
            gw = ranks[0][norm]["grads"][j]
            for x in ranks[1:]:
                assert torch.equal(x[norm]["grads"][j], gw) and torch.equal(x[norm]["params"][j], ranks[0][norm]["params"][j])
            rel = (gw - g1[j]).norm() / g1[j].norm()
            assert rel < 1e-6, (norm, j, float(rel))
            prel = (ranks[0][norm]["params"][j] - p1[j]).norm() / p1[j].norm()
            assert prel < 1e-6, (norm, j, float(prel))
