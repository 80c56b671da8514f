"""HIP PPO rollout kernels (ppo.hip: hs_ppo_act / hs_ppo_post) against the torch restatement of
SB3 2.3.2 collect_rollouts' per-step semantics (ppo.PPO._collect_rollouts_torch), and the device
rollout's buffers against the policy they were sampled from.  SB3 itself is not importable here,
so parity with SB3 is unpinned; these pin the kernels to the torch path's formulas."""
import math

import numpy as np
import pytest
import torch

from conftest import XML

pytestmark = pytest.mark.gpu


def _act_inputs(N=4096, A=21, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    head = torch.randn(N, A + 3, device="cuda", generator=g)           # mean with a leading dim > A
    value = torch.randn(N, 5, device="cuda", generator=g)              # value at stride 5
    log_std = 0.3 * torch.randn(A, device="cuda", generator=g)
    start = (torch.rand(N, device="cuda", generator=g) < 0.3).float()
    return head[:, :A], value[:, 0], log_std, start


def _run_act(mean, value, log_std, start, seed, counter, det):
    from mujocoposelearning_amd.ppo import ppo_act
    N, A = mean.shape
    out = [torch.full((N, A), float("nan"), device="cuda") for _ in range(2)] + \
          [torch.full((N,), float("nan"), device="cuda") for _ in range(3)]
    ppo_act(mean, value, log_std, start, seed, counter, det, *out)
    torch.cuda.synchronize()
    return out


def test_ppo_act_deterministic_and_logp():
    mean, value, log_std, start = _act_inputs()
    a, ac, lp, v, st = _run_act(mean, value, log_std, start, 1, 0, True)
    assert torch.equal(a, mean) and torch.equal(ac, mean.clamp(-1, 1))
    assert torch.equal(v, value) and torch.equal(st, start)
    ref = (-log_std - 0.5 * math.log(2 * math.pi)).sum().expand_as(lp)
    assert torch.allclose(lp, ref, rtol=1e-6, atol=1e-5)


def test_ppo_act_sample_matches_diag_gaussian_log_prob():
    from mujocoposelearning_amd.ppo import ActorCritic
    mean, value, log_std, start = _act_inputs(seed=1)
    a, ac, lp, v, st = _run_act(mean, value, log_std, start, 12345, 7, False)
    # log_prob of the returned actions under the torch DiagGaussian formula (ActorCritic._logp)
    pol = ActorCritic(8, mean.shape[1]).cuda()
    with torch.no_grad():
        pol.log_std.copy_(log_std)
        ref = pol._logp_torch(mean, a)
    assert torch.allclose(lp, ref, rtol=1e-5, atol=2e-4), float((lp - ref).abs().max())
    assert torch.equal(ac, a.clamp(-1, 1)) and torch.equal(v, value) and torch.equal(st, start)
    z = (a - mean) / log_std.exp()
    assert abs(float(z.mean())) < 0.02 and abs(float(z.std()) - 1) < 0.02
    # per-action-column moments (no lane/column bias) and no correlation between neighbours
    assert float(z.mean(0).abs().max()) < 0.06 and float((z.std(0) - 1).abs().max()) < 0.06
    assert abs(float((z[:, :-1] * z[:, 1:]).mean())) < 0.02
    # counter-based stream: reproducible from (seed, counter), fresh for counter + 1
    a2 = _run_act(mean, value, log_std, start, 12345, 7, False)[0]
    a3 = _run_act(mean, value, log_std, start, 12345, 8, False)[0]
    assert torch.equal(a, a2) and not torch.equal(a, a3)


def test_ppo_act_rejects_bad_shapes():
    from mujocoposelearning_amd import _lib
    L = _lib.lib()
    assert L.hs_ppo_act(None, 40, None, 1, None, None, 0, 0, None, 0, None, None, None, None, None, 8, 33, None) < 0
    assert b"A <= 32" in L.hs_last_error()
    assert L.hs_ppo_act(None, 4, None, 1, None, None, 0, 0, None, 0, None, None, None, None, None, 8, 8, None) < 0
    assert L.hs_ppo_post(None, None, None, None, None, None, None, 0, 0.9, None, None, 0, None, None, None, None, None,
                         4, None) < 0


def test_ppo_post_matches_torch_bookkeeping():
    from mujocoposelearning_amd.ppo import ppo_post
    N, D, gamma = 4097, 351, 0.99          # odd sizes: exercises the non-float4 obs copy
    g = torch.Generator(device="cuda").manual_seed(3)
    rew = torch.randn(N, device="cuda", generator=g)
    term = (torch.rand(N, device="cuda", generator=g) < 0.2).to(torch.uint8)
    trunc = (torch.rand(N, device="cuda", generator=g) < 0.2).to(torch.uint8)
    tv = torch.randn(N, device="cuda", generator=g)
    obs = torch.randn(N, D, device="cuda", generator=g)
    acc0 = torch.randn(N, device="cuda", generator=g).double()
    for d in (D, 352):
        o = obs if d == D else torch.randn(N, d, device="cuda", generator=g)
        obs_out = torch.zeros_like(o)
        rew_out = torch.zeros(N, device="cuda")
        done = torch.zeros(N, dtype=torch.bool, device="cuda")
        acc = acc0.clone()
        epret = torch.zeros(N, dtype=torch.float64, device="cuda")
        start = torch.full((N,), 0.5, device="cuda")
        ppo_post(rew, term, trunc, tv, gamma, o, obs_out, rew_out, done, acc, epret, start)
        # deferred mode: raw rewards, boot flags and the boot envs' terminal-obs rows
        tobs = torch.randn(N, 7, device="cuda", generator=g)
        bobs = torch.zeros(N, 7, device="cuda")
        bflag = torch.zeros(N, dtype=torch.bool, device="cuda")
        rew_d = torch.zeros(N, device="cuda")
        acc_d = acc0.clone()
        ppo_post(rew, term, trunc, None, gamma, o, torch.zeros_like(o), rew_d, torch.zeros_like(done), acc_d,
                 torch.zeros_like(epret), torch.zeros_like(start), terminal_obs=tobs, boot_obs_out=bobs,
                 boot_out=bflag)
        torch.cuda.synchronize()
        # the torch restatement (PPO._collect_rollouts_torch)
        t, tr = term.bool(), trunc.bool()
        boot = (tr & ~t).float()
        r_ref = rew + gamma * torch.where(boot > 0, tv, torch.zeros_like(tv))
        d_ref = t | tr
        acc_ref = acc0 + rew.double()
        assert torch.allclose(rew_out, r_ref, rtol=1e-6, atol=1e-6)
        assert torch.equal(done, d_ref) and torch.equal(epret, acc_ref)
        assert torch.equal(acc, acc_ref.masked_fill(d_ref, 0.0)) and torch.equal(start, d_ref.float())
        assert torch.equal(obs_out, o)
        bt = tr & ~t
        assert torch.equal(rew_d, rew) and torch.equal(bflag, bt) and torch.equal(acc_d, acc)
        assert torch.equal(bobs[bt], tobs[bt]) and not bobs[~bt].any()
        # the deferred bootstrap applied afterwards == the immediate one
        rew_d[bt] += gamma * tv[bt]
        assert torch.allclose(rew_d, r_ref, rtol=1e-6, atol=1e-6)


def test_device_rollout_buffers_consistent_with_policy():
    """One device rollout on the humanoid batch: the buffered log-probs and values are the
    policy's own on the buffered (obs, action) pairs, obs slots chain step to step, and the
    clipped actions the env stepped with are the buffered actions clipped."""
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.ppo import PPO
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv({"model_path": XML, "duration": 0.2, "reward_config": {"type": "stand"}, "frame_skip": 3},
                         n_envs=256, model=HsModel(XML), seed=0)
    ppo = PPO(env, n_steps=24, batch_size=1024, n_epochs=1, seed=0,
              policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [256, 256], "vf": [256, 256]}})
    obs0 = ppo.obs.clone()
    adv, ret = ppo.collect_rollouts()
    b = ppo.buf
    torch.cuda.synchronize()
    assert torch.equal(b["obs"][0], obs0)
    with torch.no_grad():
        T, N = b["obs"].shape[:2]
        logp, _, v = ppo.policy.evaluate(b["obs"].reshape(T * N, -1), b["act"].reshape(T * N, -1))
    assert torch.allclose(logp, b["logp"].reshape(-1), rtol=1e-4, atol=2e-3)
    assert torch.allclose(v, b["val"].reshape(-1), rtol=1e-4, atol=1e-4)
    assert torch.equal(ppo._act_clip, b["act"][-1].clamp(-1, 1))
    # duration 0.2 s (~13 env steps): the envs, reset together, all finish at the same step inside
    # the 24-step rollout, and the next step's episode_start flags are set
    all_done = [t for t in range(T - 1) if bool(b["done"][t].all())]
    assert all_done and bool((b["start"][all_done[0] + 1] == 1).all()) and len(ppo.ep_returns) >= N
    assert not bool(b["done"][:all_done[0]].any())
    assert torch.isfinite(adv).all() and torch.isfinite(ret).all()
    env.close()


@pytest.mark.parametrize("rows,cols", [(32768, 256), (32768, 21), (32768, 1), (16, 90112), (2, 5), (100, 300),
                                       (0, 7)])
def test_colsum_matches_fp64_sum(rows, cols):
    from mujocoposelearning_amd.ppo import colsum
    g = torch.Generator(device="cuda").manual_seed(rows + cols)
    x = torch.randn(rows, cols, device="cuda", generator=g)
    out = colsum(x)
    out2 = colsum(x)
    ref = x.double().sum(0).float()
    assert torch.equal(out, out2)                                   # fixed summation order
    assert torch.allclose(out, ref, rtol=1e-5, atol=1e-5 * max(1.0, rows ** 0.5)), float((out - ref).abs().max())
    w = torch.randn(rows, device="cuda", generator=g)               # weighted rows (rank-1 weight gradient)
    outw = colsum(x, w)
    refw = (x.double() * w.double()[:, None]).sum(0).float()
    assert torch.allclose(outw, refw, rtol=1e-5, atol=1e-5 * max(1.0, rows ** 0.5)), float((outw - refw).abs().max())


def test_gauss_logp_forward_backward_match_torch():
    """hs_gauss_logp / hs_gauss_logp_grad (the update's log-prob) == the torch DiagGaussian
    formula and its autograd gradients (mean through a strided view, as the packed heads give)."""
    from mujocoposelearning_amd.ppo import ActorCritic
    N, A = 32768, 21
    g = torch.Generator(device="cuda").manual_seed(5)
    pol = ActorCritic(8, A).cuda()
    with torch.no_grad():
        pol.log_std.copy_(0.4 * torch.randn(A, device="cuda", generator=g))
    base = torch.randn(N, A + 1, device="cuda", generator=g)
    act = torch.randn(N, A, device="cuda", generator=g)
    w = torch.randn(N, device="cuda", generator=g)
    out = []
    for fn in (pol._logp, pol._logp_torch):
        m = base.clone().requires_grad_()
        pol.log_std.grad = None
        lp = fn(m[:, :A], act)
        (lp * w).sum().backward()
        out.append((lp.detach(), m.grad[:, :A].clone(), pol.log_std.grad.clone()))
    (lp, gm, gls), (lp_r, gm_r, gls_r) = out
    assert torch.allclose(lp, lp_r, rtol=1e-5, atol=1e-4)
    assert torch.allclose(gm, gm_r, rtol=1e-5, atol=1e-5)
    assert torch.allclose(gls, gls_r, rtol=1e-4, atol=1e-3 * float(gls_r.abs().max())), float((gls - gls_r).abs().max())


@pytest.mark.parametrize("batch", [2048, 128])
def test_graphed_update_matches_eager_update(batch):
    """PPO.train replayed as HIP graphs takes the same optimizer steps as the eager loop: same
    rollout, same minibatch permutations -> same weights and losses.  World 1 replays one graph per
    epoch (every minibatch's fwd+bwd, clip and Adam); batch 128 is the reference's README config
    (64 minibatches per epoch here)."""
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.ppo import PPO
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3},
                         n_envs=512, model=HsModel(XML), seed=0)
    kw = dict(n_steps=16, batch_size=batch, n_epochs=2, seed=0,
              policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [256, 256], "vf": [256, 256]}})
    pa, pb = PPO(env, **kw), PPO(env, **kw)
    pb.graphs = False
    adv, ret = pa.collect_rollouts()
    for k in pa.buf:
        pb.buf[k].copy_(pa.buf[k])
    res = []
    for p in (pa, pb):
        for it in range(2):                 # the second call replays the graphs captured by the first
            torch.manual_seed(100 + it)
            res.append(p.train(adv, ret))
    assert pa._graphs is not None and pb._graphs is None and pa._epoch_graph is not None
    for x, y in zip(pa.policy.parameters(), pb.policy.parameters()):
        assert torch.allclose(x, y, rtol=1e-4, atol=1e-6), float((x - y).abs().max())
    for ra, rb in zip(res[:2], res[2:]):
        assert abs(ra["policy_loss"] - rb["policy_loss"]) < 1e-4 and abs(ra["value_loss"] - rb["value_loss"]) < 1e-3 * (
            1 + abs(rb["value_loss"]))
    env.close()


def _graphed_world2_worker(rank, world, port, out_dir):
    import os
    import torch.distributed as dist
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.ppo import PPO
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)     # both ranks share the one GPU
    calls = []
    real = dist.all_reduce

    def counting(t, *a, **k):
        calls.append(t.numel())
        return real(t, *a, **k)
    dist.all_reduce = counting
    try:
        env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "reward_config": {"type": "stand"},
                              "frame_skip": 3}, n_envs=256, model=HsModel(XML), seed=10 + rank)
        kw = dict(n_steps=8, batch_size=1024, n_epochs=2, seed=0,
                  policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [64, 64], "vf": [64, 64]}})
        pa, pb = PPO(env, **kw), PPO(env, **kw)
        pb.graphs = False
        adv, ret = pa.collect_rollouts()
        for k in pa.buf:
            pb.buf[k].copy_(pa.buf[k])
        for p in (pa, pb):
            torch.manual_seed(7)
            p.train(adv, ret)
        flat = [torch.cat([q.detach().reshape(-1) for q in p.policy.parameters()]).cpu() for p in (pa, pb)]
        torch.save({"graphed": flat[0], "eager": flat[1], "calls": calls}, os.path.join(out_dir, f"r{rank}.pt"))
        env.close()
    finally:
        dist.all_reduce = real
        dist.destroy_process_group()


def test_graphed_update_world2_allreduce(tmp_path):
    """world 2 (gloo rehearsal, two ranks on one GPU): the graphed update packs the gradient
    bucket in G1, all-reduces it once per optimizer step between the replays, and ends with the
    same weights as the eager update on both ranks."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_graphed_world2_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(2)]
    assert torch.equal(r[0]["graphed"], r[1]["graphed"]), "ranks diverged in the graphed update"
    assert torch.allclose(r[0]["graphed"], r[0]["eager"], rtol=1e-4, atol=1e-6)
    n = r[0]["graphed"].numel()
    # 2 epochs x (8 x 256 / 1024) minibatches, graphed + eager: 8 buckets of n (plus the env-count
    # agreement of each PPO's construction)
    assert [c for c in r[0]["calls"] if c == n] == [n] * 8
    assert r[0]["calls"] == r[1]["calls"]


def test_rccl_world1_bucket_allreduce_between_graph_replays():
    """RCCL really executes: a world-1 ``nccl`` process group (RCCL on ROCm) with the gradient
    sync forced on runs the graphed update's bucket all-reduce as an eager device collective
    between the G1 and G2 replays of every optimizer step.  With one rank the all-reduce is the
    identity, so the weights must equal those of the same update without the collective."""
    import socket
    import torch.distributed as dist
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.ppo import PPO
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    calls = []
    real = dist.all_reduce

    def counting(t, *a, **k):
        calls.append((t.numel(), t.device.type))
        return real(t, *a, **k)
    dist.all_reduce = counting
    try:
        assert dist.get_backend() == "nccl"
        env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "reward_config": {"type": "stand"},
                              "frame_skip": 3}, n_envs=256, model=HsModel(XML), seed=3)
        kw = dict(n_steps=8, batch_size=1024, n_epochs=2, seed=0,
                  policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [64, 64], "vf": [64, 64]}})
        pa, pb = PPO(env, sync_grads=True, **kw), PPO(env, **kw)
        assert pa.sync_grads and not pb.sync_grads and pa.grad_weight == 1.0
        adv, ret = pa.collect_rollouts()
        for k in pa.buf:
            pb.buf[k].copy_(pa.buf[k])
        for p in (pa, pb):
            for it in range(2):                 # the second call replays the captured graphs
                torch.manual_seed(11 + it)
                p.train(adv, ret)
        torch.cuda.synchronize()
        assert pa._graphs is not None and pb._graphs is not None
        n = sum(q.numel() for q in pa.policy.parameters())
        buckets = [c for c in calls if c[0] == n]
        # 2 train calls x 2 epochs x (8 x 256 / 1024) minibatches, every bucket on the device
        assert buckets == [(n, "cuda")] * 8, calls
        for x, y in zip(pa.policy.parameters(), pb.policy.parameters()):
            assert torch.allclose(x, y, rtol=1e-5, atol=1e-7), float((x - y).abs().max())
        env.close()
    finally:
        dist.all_reduce = real
        dist.destroy_process_group()


def test_device_rollout_deferred_timelimit_bootstrap():
    """max_steps 10 < duration: every env is truncated (not terminated) at env step 10, so the
    device rollout's deferred bootstrap must add gamma V(terminal obs) to exactly those rewards
    (the reference's truncated reward itself is 0, custom_env.py:201-206)."""
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.ppo import PPO
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3},
                         n_envs=128, model=HsModel(XML), seed=0)
    env.batch.configure(max_steps=10)
    ppo = PPO(env, n_steps=16, batch_size=512, n_epochs=1, seed=0, gamma=0.9,
              policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [64, 64], "vf": [64, 64]}})
    ppo.collect_rollouts()
    b = ppo.buf
    torch.cuda.synchronize()
    steps = [t for t in range(16) if bool(b["boot"][t].any())]
    assert len(steps) == 1 and bool(b["boot"][steps[0]].all()), steps
    t = steps[0]
    with torch.no_grad():
        expect = 0.9 * ppo.policy.value(b["tobs"][t])
    assert torch.allclose(b["rew"][t], expect, rtol=1e-5, atol=1e-6)
    assert bool(b["done"][t].all()) and bool((b["start"][t + 1] == 1).all())
    # the kept terminal obs is the pre-reset state, not the post-reset obs of slot t+1
    assert float((b["tobs"][t] - b["obs"][t + 1]).abs().max()) > 1e-3
    others = [k for k in range(16) if k != t]
    assert not bool(b["tobs"][others].any())
    env.close()


@pytest.mark.parametrize("prec,n,steps", [("fp32", 256, 12), ("fp64", 4096, 6)])
def test_graphed_rollout_matches_eager_rollout(prec, n, steps, monkeypatch):
    """The device rollout captured as one HIP graph (PPO._capture_rollout) writes exactly what the
    eager loop writes: two identical envs + policies, one graphed and one eager, two rollouts
    each (the second replays the graph with fresh noise and a reset inside).  The fp64 case at
    configs[1] size runs the env steps on the chunk-queue schedule (persistent grid, self-resetting
    claim counter and pair flags) inside the replayed graph."""
    from mujocoposelearning_amd import ppo as ppo_mod
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.ppo import PPO
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    monkeypatch.setattr(ppo_mod, "FUSED_ROLLOUT", False)     # this test is about the per-step graph path
    model = HsModel(XML)
    cfg = {"model_path": XML, "duration": 0.2 if prec == "fp32" else 0.1, "reward_config": {"type": "stand"},
           "frame_skip": 3}
    envs = [HumanoidVecEnv(cfg, n_envs=n, model=model, seed=0, precision=prec) for _ in range(2)]
    assert envs[0].batch.queued() == (prec == "fp64")
    kw = dict(n_steps=steps, batch_size=min(1024, n * steps), n_epochs=1, seed=0,
              policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [256, 256], "vf": [256, 256]}})
    pa, pb = PPO(envs[0], **kw), PPO(envs[1], **kw)
    pb.graphs = False
    assert envs[0].graph_safe
    for it in range(2):
        ra, rb = pa.collect_rollouts(), pb.collect_rollouts()
        torch.cuda.synchronize()
        assert pa._rollout_graph is not None and pb._rollout_graph is None
        for k in ("obs", "act", "rew", "start", "val", "logp", "done", "epret"):
            assert torch.equal(pa.buf[k], pb.buf[k]), (it, k)
        assert torch.equal(ra[0], rb[0]) and torch.equal(ra[1], rb[1])
        assert pa.ep_returns == pb.ep_returns
    for e in envs:
        e.close()


@pytest.mark.parametrize("B", [32768, 777, 1])
def test_fused_ppo_loss_matches_torch(B):
    """hs_ppo_loss / hs_ppo_loss_grad == the torch restatement of SB3 PPO.train's minibatch loss
    (PPO._minibatch_loss's CPU branch) and its autograd gradients, with ratios inside and outside
    the clip range."""
    from mujocoposelearning_amd.ppo import ppo_loss
    g = torch.Generator(device="cuda").manual_seed(B)
    M, clip = 50000, 0.2
    adv = torch.randn(M, device="cuda", generator=g) * 3 + 0.5
    ret = torch.randn(M, device="cuda", generator=g)
    old = torch.randn(M, device="cuda", generator=g) * 0.1 - 20
    idx = torch.randperm(M, device="cuda", generator=g)[:B].contiguous()
    lp0 = old[idx] + 0.3 * torch.randn(B, device="cuda", generator=g)     # ratios ~ exp(N(0, 0.3))
    v0 = torch.randn(B, device="cuda", generator=g)
    out = []
    for fused in (True, False):
        lp, v = lp0.clone().requires_grad_(), v0.clone().requires_grad_()
        if fused:
            pg, vf = ppo_loss(lp, v, idx, adv, ret, old, clip)
        else:
            a = adv[idx]
            if B > 1:
                a = (a - a.mean()) / (a.std() + 1e-8)
            r = torch.exp(lp - old[idx])
            pg = -torch.min(a * r, a * r.clamp(1 - clip, 1 + clip)).mean()
            vf = torch.nn.functional.mse_loss(ret[idx], v)
        (pg + 0.5 * vf).backward()
        out.append((float(pg), float(vf), lp.grad.clone(), v.grad.clone()))
    (pg, vf, glp, gv), (pg_r, vf_r, glp_r, gv_r) = out
    assert abs(pg - pg_r) <= 1e-5 * (1 + abs(pg_r)) and abs(vf - vf_r) <= 1e-5 * (1 + abs(vf_r))
    assert torch.allclose(glp, glp_r, rtol=1e-4, atol=1e-6 * float(glp_r.abs().max()) + 1e-12)
    assert torch.allclose(gv, gv_r, rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize("hidden", [1, 20])
def test_adam_clip_matches_torch_clip_and_adam(hidden):
    """hs_adam_clip (clip_grad_norm_ + Adam in three launches) == torch.nn.utils.clip_grad_norm_ +
    torch.optim.Adam over several steps, on an MLP's parameter list, clipping active and not.
    hidden=20: 42 tensors, three chunks of the 16-tensor kernel sharing one clip coefficient."""
    from mujocoposelearning_amd.ppo import adam_clip_step
    torch.manual_seed(0)

    def mlp():
        layers = [torch.nn.Linear(352, 64), torch.nn.ReLU()]
        for _ in range(hidden - 1):
            layers += [torch.nn.Linear(64, 64), torch.nn.ReLU()]
        return torch.nn.Sequential(*layers, torch.nn.Linear(64, 21)).cuda()
    nets = [mlp() for _ in range(2)]
    nets[1].load_state_dict(nets[0].state_dict())
    opts = [torch.optim.Adam(n.parameters(), lr=3e-4, eps=1e-5) for n in nets]
    g = torch.Generator(device="cuda").manual_seed(1)
    ws = None
    for step, (scale, max_norm) in enumerate([(10.0, 0.5), (0.01, 0.5), (3.0, 0.5), (1.0, 0.0), (5.0, 0.5)]):
        grads = [torch.randn(p.shape, device="cuda", generator=g) * scale for p in nets[0].parameters()]
        for n in nets:
            for p, gr in zip(n.parameters(), grads):
                p.grad = gr.clone()
        ws = adam_clip_step(opts[0], list(nets[0].parameters()), max_norm, ws)
        if max_norm > 0:
            torch.nn.utils.clip_grad_norm_(nets[1].parameters(), max_norm)
        opts[1].step()
        for a, b in zip(nets[0].parameters(), nets[1].parameters()):
            assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (step, float((a - b).abs().max()))
    sa, sb = opts[0].state_dict()["state"], opts[1].state_dict()["state"]
    for k in sa:
        assert float(sa[k]["step"]) == float(sb[k]["step"]) == 5
        for key in ("exp_avg", "exp_avg_sq"):
            x, y = sa[k][key], sb[k][key]
            err = float((x - y).abs().max()) / float(y.abs().max())
            assert err < 1e-5, (k, key, err)


def test_relu_grad_colsum_and_pair():
    """hs_relu_grad_colsum (ReLU mask + first bias-sum pass) and hs_colsum_pair (two finishes in
    one launch) == threshold_backward and fp64 column sums."""
    from mujocoposelearning_amd.ppo_ops import colsum_pair, relu_grad_colsum
    gen = torch.Generator(device="cuda").manual_seed(9)
    for rows, cols in ((32768, 256), (32768, 21), (100, 7)):
        g = torch.randn(rows, cols, device="cuda", generator=gen)
        y = torch.relu(torch.randn(rows, cols, device="cuda", generator=gen))
        gm, part = relu_grad_colsum(g, y)
        ref = torch.ops.aten.threshold_backward(g, y, 0)
        assert torch.equal(gm, ref)
        p2 = torch.randn(16, 3 * cols, device="cuda", generator=gen)
        s0, s1 = colsum_pair(p2, part)
        assert torch.allclose(s0, p2.double().sum(0).float(), rtol=1e-5, atol=1e-5)
        assert torch.allclose(s1, ref.double().sum(0).float(), rtol=1e-5, atol=1e-5 * rows ** 0.5)


@pytest.mark.parametrize("B,K", [(32768, 256), (10000, 256), (4096, 256), (100, 256), (37, 21), (32768, 21),
                                 (4096, 1), (5, 1)])
def test_dgrad_mask_matches_torch(B, K):
    """hs_dgrad_mask (ppo.hip dgrad_mask_*: the input gradient of a Linear fed by a ReLU, masked,
    with per-row-block column sums) == (g @ w) * (x > 0) and its fp64 column sums, fp32 tolerance:
    the MFMA instance with one / two / four row blocks (4096 / 10000 / 32768 rows), a partial last
    tile (100, 10000), the
    VALU instance for the heads (21 actions, 1 value) with ragged rows (37, 5)."""
    from mujocoposelearning_amd.ppo_ops import colsum_pair, dgrad_mask
    gen = torch.Generator(device="cuda").manual_seed(B + K)
    g = torch.randn(B, K, device="cuda", generator=gen)
    w = torch.randn(K, 256, device="cuda", generator=gen) * 0.06
    x = torch.relu(torch.randn(B, 256, device="cuda", generator=gen))
    gx, part = dgrad_mask(g, w, x)
    ref = (g.double() @ w.double()) * (x > 0)
    tol = 1e-5 * (1 + float(ref.abs().max()))
    assert float((gx.double() - ref).abs().max()) < tol
    assert torch.all(gx[x <= 0] == 0)
    _, s1 = colsum_pair(torch.zeros(1, 1, device="cuda"), part)
    assert torch.allclose(s1.double(), ref.sum(0), rtol=1e-5, atol=tol * B ** 0.5)


@pytest.mark.parametrize("K", [256, 21])
def test_dgrad_mask_unaligned_operands(K):
    """hs_dgrad_mask on operands whose rows are not 16-byte aligned (X and W views one float into
    wider rows): the element-load instances, same results as the aligned ones."""
    from mujocoposelearning_amd.ppo_ops import colsum_pair, dgrad_mask
    gen = torch.Generator(device="cuda").manual_seed(K)
    B = 3000
    g = torch.randn(B, K, device="cuda", generator=gen)
    w = (torch.randn(K, 261, device="cuda", generator=gen) * 0.06)[:, 1:257]
    x = torch.relu(torch.randn(B, 259, device="cuda", generator=gen))[:, 3:259]
    gx, part = dgrad_mask(g, w, x)
    ga, pa = dgrad_mask(g, w.contiguous(), x.contiguous())
    ref = (g.double() @ w.double()) * (x > 0)
    assert float((gx.double() - ref).abs().max()) < 1e-5 * (1 + float(ref.abs().max()))
    assert torch.equal(gx, ga) and torch.equal(part, pa)


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_mlp_chain_node_gradients_match_autograd(depth):
    """_MLPChainFn (a whole pi / vf net as one autograd node, ppo_ops.py) == module-by-module torch
    autograd of the same nn.Linear / ReLU net: outputs and every parameter gradient, fp32
    tolerance, for 1-3 hidden layers of 256, the pi head (21 actions) and the value head (rank-1
    weight gradient), with and without an input gradient."""
    from mujocoposelearning_amd import ppo_ops as O
    F = torch.nn.functional
    torch.manual_seed(3 + depth)
    B, D = 32768, 352
    for A, need_gx in ((21, False), (1, True)):
        mods = []
        for li in range(depth):
            mods += [O.Linear(D if li == 0 else 256, 256), torch.nn.ReLU()]
        seq = torch.nn.Sequential(*mods).cuda()
        head = O.Linear(256, A).cuda()
        params = list(seq.parameters()) + list(head.parameters())
        x = torch.randn(B, D, device="cuda", requires_grad=need_gx)
        gout = torch.randn(B, A, device="cuda")
        res = {}
        for fused in (True, False):
            O.FUSED_CHAIN = fused
            try:
                for p in params:
                    p.grad = None
                x.grad = None
                with torch.enable_grad():
                    if fused:
                        out = O.mlp_head_forward(seq, head, x)
                    else:   # plain torch: F.linear / relu on the same parameters
                        h = x
                        for m in seq[0::2]:
                            h = torch.relu(F.linear(h, m.weight, m.bias))
                        out = F.linear(h, head.weight, head.bias)
                    out.backward(gout)
                res[fused] = [out.detach()] + [p.grad.clone() for p in params]
                if need_gx:
                    res[fused].append(x.grad.clone())
            finally:
                O.FUSED_CHAIN = True
        for a, b in zip(res[True], res[False]):
            assert a.shape == b.shape
            assert torch.allclose(a, b, rtol=1e-4, atol=1e-4 * (1 + float(b.abs().max()))), float((a - b).abs().max())


def test_chain_node_in_a_real_ppo_minibatch():
    """In context: after a real fused rollout of 4096 fp64 envs (bench train config), one 32 768-
    sample minibatch's loss gradient for every policy parameter (log_std included) with the nets'
    backward as _MLPChainFn nodes == the module-by-module backward, fp32 tolerance; and so does the
    gradient norm clip_grad_norm_ sees."""
    from mujocoposelearning_amd import ppo_ops as O
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.ppo import PPO
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "frame_skip": 3, "reward_config": {"type": "stand"}},
                         n_envs=4096, model=HsModel(XML), seed=0, precision="fp64")
    ppo = PPO(env, n_steps=32, batch_size=32768, n_epochs=1, seed=0, stagger_episodes=True,
              policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [256, 256], "vf": [256, 256]}})
    adv, ret = ppo.collect_rollouts()
    b = ppo.buf
    M = 32 * 4096
    obs, act, old_logp = b["obs"].reshape(M, -1), b["act"].reshape(M, -1), b["logp"].reshape(-1)
    adv, ret = adv.reshape(-1).float().contiguous(), ret.reshape(-1).float().contiguous()
    idx = torch.randperm(M, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))[:32768]
    params = list(ppo.policy.parameters())
    grads = {}
    for fused in (True, False):
        O.FUSED_CHAIN = fused
        try:
            for p in params:
                p.grad = None
            with torch.enable_grad():
                loss, _, _ = ppo._minibatch_loss(obs, act, old_logp, adv, ret, idx)
                loss.backward()
            grads[fused] = [p.grad.clone() for p in params]
        finally:
            O.FUSED_CHAIN = True
    for a, c in zip(grads[True], grads[False]):
        assert torch.allclose(a, c, rtol=1e-3, atol=1e-4 * (1 + float(c.abs().max()))), float((a - c).abs().max())
    n1 = torch.sqrt(sum((g.double() ** 2).sum() for g in grads[True]))
    n0 = torch.sqrt(sum((g.double() ** 2).sum() for g in grads[False]))
    assert abs(float(n1 / n0) - 1) < 1e-4, (float(n1), float(n0))
    env.close()


def test_ppo_deep_net_arch_trains_on_gpu():
    """net_arch lists of any depth (main.py --net_arch_pi/--net_arch_vf): 3 + 3 hidden
    layers are 17 parameter tensors (> one 16-tensor Adam chunk); graphed training runs and
    changes every parameter."""
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.ppo import PPO
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3},
                         n_envs=256, model=HsModel(XML), seed=0)
    ppo = PPO(env, n_steps=8, batch_size=512, n_epochs=2, seed=0,
              policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [64, 64, 64], "vf": [64, 64, 64]}})
    params = [p for p in ppo.policy.parameters()]
    assert len(params) == 17
    before = [p.detach().clone() for p in params]
    ppo.learn(2 * 8 * 256)
    torch.cuda.synchronize()
    assert all(not torch.equal(a, p.detach()) for a, p in zip(before, params))
    assert all(torch.isfinite(p).all() for p in params)
    env.close()


@pytest.mark.parametrize("N,D", [(4096, 352), (1000, 350), (33, 7), (257, 100), (20000, 352), (9001, 350)])
def test_fused_mlp_forward_matches_gemm_chain(N, D):
    """hs_mlp2_forward (ppo.hip mlp2_fwd_kernel: MFMA f32 tiles, one launch, the nn.Linear weights
    read in place) == the packed GEMM chain of ActorCritic.net_forward (torch fp32) for the pi mean
    and the vf value, within 1e-4 relative; odd row counts and input widths: the 16-row tile, a
    partial last k-group (350, 7, 100), element loads for rows that are not 16-byte aligned (350, 7)
    and no full k-group at all (7); above 8192 rows the two-row-block instance (20000, 9001)."""
    from mujocoposelearning_amd import ppo as P
    torch.manual_seed(0)
    pol = P.ActorCritic(D, 21, [256, 256], [256, 256], torch.nn.ReLU).cuda()
    with torch.no_grad():
        for p in pol.parameters():
            p.add_(0.05 * torch.randn_like(p))
    pol.pack_heads()
    obs = torch.randn(N, D, device="cuda") * 2
    outs = {}
    for fused in (True, False):
        P.FUSED_MLP = fused
        try:
            outs[fused] = [pol.net_forward(obs, 0).clone(), pol.net_forward(obs, 1).clone()]
        finally:
            P.FUSED_MLP = True
    for a, b in zip(outs[True], outs[False]):
        assert a.shape == b.shape
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-4 * (1 + float(b.abs().max()))), float((a - b).abs().max())


def test_fused_mlp_abi_with_padded_strides():
    """hs_mlp2_forward through the C ABI on strided operands: input rows of 400 floats holding 352
    features, weight rows padded (ld1 = 360, ld2 = ld3 = 264), an output of stride 32 holding 21
    columns (the padding untouched) -- against the fp32 torch chain on the same values."""
    import torch
    from mujocoposelearning_amd import _lib
    torch.manual_seed(1)
    N, D, H, A = 1000, 352, 256, 21
    xs = torch.randn(N, 400, device="cuda")
    w1s, w2s, w3s = (torch.randn(H, 360, device="cuda") * 0.05, torch.randn(H, 264, device="cuda") * 0.05,
                     torch.randn(A, 264, device="cuda") * 0.05)
    b1, b2, b3 = (torch.randn(H, device="cuda") * 0.1, torch.randn(H, device="cuda") * 0.1,
                  torch.randn(A, device="cuda") * 0.1)
    out = torch.full((N, 32), 7.0, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    assert _lib.lib().hs_mlp2_forward(xs.data_ptr(), 400, D, N, w1s.data_ptr(), 360, b1.data_ptr(), w2s.data_ptr(),
                                      264, b2.data_ptr(), w3s.data_ptr(), 264, b3.data_ptr(), A, out.data_ptr(), 32,
                                      st) == 0
    x, w1, w2, w3 = xs[:, :D], w1s[:, :D], w2s[:, :H], w3s[:, :H]
    ref = torch.relu(torch.relu(x @ w1.t() + b1) @ w2.t() + b2) @ w3.t() + b3
    torch.cuda.synchronize()
    assert torch.allclose(out[:, :A], ref, rtol=1e-4, atol=1e-4 * (1 + float(ref.abs().max())))
    assert torch.all(out[:, A:] == 7.0)


def test_learn_raises_on_a_lost_handoff_and_warns_on_bad_states():
    """PPO.learn reduces the env's warning counters once per rollout (include/hsim.h HS_WARN_*): a
    lost chunk-queue hand-off (forced with the hs_debug_lose_handoff hook on a queued 4096-env fp64
    batch) raises, because it is a scheduling failure, not physics; before it, a bad-state reset is
    reported as MuJoCo reports it (a warning) and training goes on."""
    import warnings
    from mujocoposelearning_amd._lib import HsimError
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.ppo import PPO
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "frame_skip": 3, "reward_config": {"type": "stand"}},
                         n_envs=4096, model=HsModel(XML), seed=0, precision="fp64")
    ppo = PPO(env, n_steps=4, batch_size=4096, n_epochs=1, seed=0,
              policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [256, 256], "vf": [256, 256]}})
    assert env.batch.queued()
    ppo.learn(4 * 4096)                                          # clean: no warning, counts logged
    assert ppo.logger["env_warnings"] == [0, 0, 0, 0, 0]
    q = env.batch.qpos
    q[5, 2] = float("nan")                                       # a bad state: mj_checkPos resets it
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        ppo.learn(8 * 4096)
    assert ppo.logger["env_warnings"][0] == 1
    assert any("QPOS" in str(w.message) for w in rec)
    env.batch.debug_lose_handoff(1234)
    with pytest.raises(HsimError, match="hand-off lost"):
        ppo.learn(12 * 4096)
    env.batch.debug_lose_handoff(None)
    env.close()


@pytest.mark.slow
def test_trainer_still_learns_the_stand_task():
    """Learning regression (README.md:160-164 is the reference's one training outcome): bench.py's
    train config -- 4096 fp64 envs, fused hs_rollout rollouts, n_steps 32, batch 32768, 4 epochs,
    lr 3e-4, ent_coef 0, MLP[256,256] ReLU, staggered episode clocks -- seed 0 for 40 M env steps
    (~11 s).  A humanoid that falls at once scores ~18; with staggered clocks this config reaches
    52-54 by 39 M on seeds 0-2 and stands (return > 500, torso ~1.1 m) by 200-280 M
    (profiles/learning_curve_r5.md, r5u); its log_std falls (exploitation: -0.15 by 39 M).  Guards
    the fused rollout's sampling and bookkeeping and the graphed update against silent breaks the
    bitwise replay tests would not see."""
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.ppo import PPO
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "frame_skip": 3, "reward_config": {"type": "stand"}},
                         n_envs=4096, model=HsModel(XML), seed=0, precision="fp64")
    ppo = PPO(env, n_steps=32, batch_size=32768, n_epochs=4, learning_rate=3e-4, seed=0, stagger_episodes=True,
              policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [256, 256], "vf": [256, 256]}})
    ppo.policy.pack_heads()
    assert ppo._fused_rollout_args() is not None
    ppo.learn(40_000_000)
    ret = float(np.mean(ppo.ep_returns[-200:]))
    log_std = float(ppo.policy.log_std.mean())
    print(f"40 M env steps: return {ret:.2f}, log_std {log_std:.3f}, fallbacks {getattr(ppo, 'fused_fallbacks', 0)}")
    assert getattr(ppo, "fused_fallbacks", 0) == 0 and ppo.logger["env_warnings"][4] == 0
    assert ret >= 45.0, ret
    assert log_std < -0.05, log_std
    env.close()


def test_staggered_episode_clocks_spread_the_resets():
    """HumanoidVecEnv.stagger_episode_clocks: env i behaves as floor(i L / N) of the L = 667 env steps
    into its episode, so its first episode ends after L - floor(i L / N) steps and the next one after
    L more; nothing else about the state changes."""
    import torch
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    n = 64
    env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "frame_skip": 3, "reward_config": {"type": "stand"}},
                         n_envs=n, model=HsModel(XML), seed=0, precision="fp64")
    env.reset_tensors()
    q0 = env.batch.qpos.clone()
    L = env.episode_length()
    assert L == 667
    env.stagger_episode_clocks()
    assert torch.equal(env.batch.qpos, q0)
    k = np.floor(np.arange(n) * L / n).astype(int)
    first = np.full(n, -1)
    second = np.full(n, -1)
    zero = torch.zeros(n, 21, device="cuda")
    for t in range(1, 2 * L + 1):
        _, _, term, trunc = env.step_tensors(zero)[:4]
        done = (term | trunc).cpu().numpy().astype(bool)
        for i in np.nonzero(done)[0]:
            if first[i] < 0:
                first[i] = t
            elif second[i] < 0:
                second[i] = t
    assert np.array_equal(first, L - k), (first[:8], (L - k)[:8])
    assert np.array_equal(second[first <= L], first[first <= L] + L)
    env.close()
