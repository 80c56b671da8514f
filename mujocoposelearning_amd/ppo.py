"""On-device PPO (PyTorch-ROCm) restating SB3 2.3.2's PPO/MlpPolicy semantics (the reference's
trainer, train_sb3.py:208-231) so rollouts never leave HBM.

* ActorCritic: separate pi / vf MLPs (net_arch dict, ReLU -- main.py:16,100), diagonal Gaussian
  with state-independent log_std (init 0), orthogonal init (gain sqrt(2) hidden, 0.01 action
  head, 1 value head) -- SB3 ActorCriticPolicy defaults.
* Rollout: n_steps x n_envs on device; actions clipped to the action space before stepping
  (SB3 collect_rollouts); time-limit truncation bootstraps r += gamma V(terminal_obs).
* GAE(gamma, lambda) reverse scan; per-minibatch advantage normalisation; clipped surrogate,
  value MSE (vf_coef 0.5), entropy bonus, clip_grad_norm(max_grad_norm 0.5), Adam(eps 1e-5).
* Multi-GPU: envs are sharded per rank; each optimizer step all-reduces the flattened gradient
  bucket ONCE (RCCL over xGMI, ~1.27 MB at [256,256]) -- no other collective on the data path
  (SURVEY.md 8e).  Ranks stay in lockstep for ANY shard sizes (train_sb3.py:203 accepts any
  n_envs): at construction the ranks agree once on every rank's env count, so all of them run the
  same number of rollout timesteps, minibatches per epoch and all-reduces; each rank's gradient is
  weighted by its share of the rollout samples before the sum.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch
import torch.nn as nn


from . import batch as _batch_mod
from .ppo_ops import (Linear, _GaussLogpFn, _PPOLossFn, _SplitKLinearFn, _SplitKLinearReLUFn,  # noqa: F401
                      _SPLITK_ROWS, adam_clip_step, colsum, gae_device, mlp2_forward, mlp_forward,
                      mlp_head_forward, ppo_act, ppo_loss, ppo_post)

FUSED_MLP = True      # rollout forward through the fused hs_mlp2_forward kernel where it applies
FUSED_MLP_MAX_ROWS = None   # ... up to this many rows (None: any)
FUSED_ROLLOUT = True  # whole rollouts as hs_rollout launches (policy inside the env kernel) where they apply


def _flat_packed(pk):
    w1, b1, mid, w3, b3 = pk
    return [w1, b1] + [t for wb in mid for t in wb] + [w3, b3]


def _mlp(inp, sizes, act=nn.ReLU):
    layers, d = [], inp
    for s in sizes:
        layers += [Linear(d, s), act()]
        d = s
    return nn.Sequential(*layers), d


class ActorCritic(nn.Module):
    def __init__(self, obs_dim, act_dim, pi=(64, 64), vf=None, activation=nn.ReLU, log_std_init=0.0):
        super().__init__()
        vf = pi if vf is None else vf
        self.pi_net, dp = _mlp(obs_dim, pi, activation)
        self.vf_net, dv = _mlp(obs_dim, vf, activation)
        self.action_net = Linear(dp, act_dim)
        self.value_net = Linear(dv, 1)
        self.log_std = nn.Parameter(torch.full((act_dim,), float(log_std_init)))
        self._packed = None      # pack_heads() cache, rebuilt at the start of every rollout
        for mod, gain in ((self.pi_net, math.sqrt(2)), (self.vf_net, math.sqrt(2)), (self.action_net, 0.01),
                          (self.value_net, 1.0)):
            for m in mod.modules() if isinstance(mod, nn.Sequential) else [mod]:
                if isinstance(m, nn.Linear):
                    nn.init.orthogonal_(m.weight, gain=gain)
                    nn.init.zeros_(m.bias)

    def forward(self, obs):
        return (mlp_head_forward(self.pi_net, self.action_net, obs),
                mlp_head_forward(self.vf_net, self.value_net, obs).squeeze(-1))

    def _logp(self, mean, actions):
        """DiagGaussian log_prob; on a device through hs_gauss_logp (+ its HIP backward)."""
        if mean.is_cuda and mean.shape[-1] <= 32:
            return _GaussLogpFn.apply(mean, actions, self.log_std)
        return self._logp_torch(mean, actions)

    def _logp_torch(self, mean, actions):
        std = self.log_std.exp()
        z = (actions - mean) / std
        return (-0.5 * z * z - self.log_std - 0.5 * math.log(2 * math.pi)).sum(-1)

    def entropy(self):
        """DiagGaussian entropy (state-independent std, so the same for every sample)."""
        return (0.5 + 0.5 * math.log(2 * math.pi) + self.log_std).sum()

    @torch.no_grad()
    def act(self, obs, deterministic=False):
        mean, value = self(obs)
        a = mean if deterministic else mean + self.log_std.exp() * torch.randn_like(mean)
        return a, self._logp(mean, a), value

    def evaluate(self, obs, actions):
        mean, value = self(obs)
        ent = (0.5 + 0.5 * math.log(2 * math.pi) + self.log_std).sum().expand(obs.shape[0])
        return self._logp(mean, actions), ent, value

    @torch.no_grad()
    def value(self, obs):
        return self.value_net(self.vf_net(obs)).squeeze(-1)

    # -- rollout-time forward (no autograd) -------------------------------------------------------
    def _hidden(self, net):
        return [m for m in net if isinstance(m, nn.Linear)]

    @torch.no_grad()
    def pack_heads(self):
        """Stack the pi and vf MLPs into one chain of batched GEMMs for the rollout forward
        (weights are constant over a rollout, so this runs once per collect_rollouts): layer 1 is
        one [obs_dim x (h_pi + h_vf)] GEMM (both nets read the same obs), deeper layers one
        2-batch GEMM each, and the heads one 2-batch GEMM whose vf half carries the value column
        in column 0 of an A-wide block.  Needs equal pi/vf widths and ReLU; otherwise None and
        heads() runs the two nets."""
        lp, lv = self._hidden(self.pi_net), self._hidden(self.vf_net)
        acts = {type(m) for m in list(self.pi_net) + list(self.vf_net) if not isinstance(m, nn.Linear)}
        same = len(lp) == len(lv) >= 1 and all(a.weight.shape == b.weight.shape for a, b in zip(lp, lv))
        if not same or acts != {nn.ReLU}:
            self._packed = None
            return None
        A, H = self.action_net.out_features, lp[-1].out_features
        w1 = torch.cat([lp[0].weight, lv[0].weight]).t().contiguous()
        b1 = torch.cat([lp[0].bias, lv[0].bias])
        mid = [(torch.stack([a.weight.t(), b.weight.t()]).contiguous(), torch.stack([a.bias, b.bias])[:, None, :])
               for a, b in zip(lp[1:], lv[1:])]
        w3 = torch.zeros(2, H, A, device=w1.device, dtype=w1.dtype)
        w3[0] = self.action_net.weight.t()
        w3[1, :, 0] = self.value_net.weight[0]
        b3 = torch.zeros(2, 1, A, device=w1.device, dtype=w1.dtype)
        b3[0, 0] = self.action_net.bias
        b3[1, 0, 0] = self.value_net.bias[0]
        new = (w1, b1, mid, w3, b3)
        old = self._packed
        if old is not None and all(a.shape == b.shape for a, b in zip(_flat_packed(old), _flat_packed(new))):
            for a, b in zip(_flat_packed(old), _flat_packed(new)):    # in place: captured graphs stay valid
                a.copy_(b)
            return old
        self._packed = new
        return self._packed

    @torch.no_grad()
    def heads(self, obs):
        """Rollout forward: (mean [N, A] view, value [N] strided view) from the packed GEMM chain
        (pack_heads) or, for unequal pi/vf nets, the two MLPs."""
        pk = getattr(self, "_packed", None)
        if pk is None:
            mean, value = self(obs)
            return mean, value
        if self._fused_mlp_ok(obs):                               # two fused launches beat the chain here
            return self.net_forward(obs, 0), self.net_forward(obs, 1)
        w1, b1, mid, w3, b3 = pk
        n = obs.shape[0]
        # [N, 2H]: layer 1 of both nets, ReLU in the GEMM epilogue on a device
        h = torch._addmm_activation(b1, obs, w1) if obs.is_cuda else torch.addmm(b1, obs, w1).relu_()
        h = h.view(n, 2, -1).transpose(0, 1)                      # [2, N, H] (strided)
        for w, b in mid:
            h = torch.baddbmm(b, h, w).relu_()
        out = torch.baddbmm(b3, h, w3)                            # [2, N, A]
        return out[0], out[1, :, 0]

    def _fused_mlp_ok(self, obs):
        """The fused hs_mlp2_forward kernel applies: packed equal pi / vf nets of two hidden layers of
        256 (ReLU), <= 512 inputs and <= 32 actions, fp32 rows with unit stride on a device, and at
        most FUSED_MLP_MAX_ROWS rows (above, the library GEMM chain is faster)."""
        pk = getattr(self, "_packed", None)
        if pk is None or not FUSED_MLP or not obs.is_cuda:
            return False
        w1, _, mid, w3, _ = pk
        return (len(mid) == 1 and w1.shape[1] == 512 and obs.shape[1] <= 512 and w3.shape[2] <= 32
                and obs.dtype == torch.float32 and obs.stride(1) == 1
                and (FUSED_MLP_MAX_ROWS is None or obs.shape[0] <= FUSED_MLP_MAX_ROWS))

    @torch.no_grad()
    def net_forward(self, obs, which):
        """One of the two nets on its own from the packed weights (which = 0: pi -> mean [N, A],
        1: vf -> value [N]); hidden layers with the ReLU in the GEMM epilogue on a device.  The
        device rollout samples with the pi net per step and evaluates the vf net once per rollout
        over the whole [T*N] buffer (the policy is fixed during a rollout)."""
        pk = getattr(self, "_packed", None)
        if pk is None:
            return self(obs)[which]
        w1, b1, mid, w3, b3 = pk
        H = w1.shape[1] // 2
        if self._fused_mlp_ok(obs):
            # one fused MFMA launch (ppo.hip mlp2_fwd_kernel) instead of three GEMMs, reading the
            # nn.Linear weights as they are ([out][in]: the reduction index contiguous)
            net, head = (self.pi_net, self.action_net) if which == 0 else (self.vf_net, self.value_net)
            l1, l2 = self._hidden(net)
            out = mlp2_forward(obs, l1.weight, l1.bias, l2.weight, l2.bias, head.weight, head.bias)
            return out if which == 0 else out[:, 0]
        act = (lambda b, x, w: torch._addmm_activation(b, x, w)) if obs.is_cuda else (  # noqa: E731
            lambda b, x, w: torch.addmm(b, x, w).relu_())
        h = act(b1[which * H:(which + 1) * H], obs, w1[:, which * H:(which + 1) * H])
        for w, b in mid:
            h = act(b[which, 0], h, w[which])
        out = torch.addmm(b3[which, 0], h, w3[which])
        return out if which == 0 else out[:, 0]


def gae(rewards, values, dones, last_values, last_dones, gamma, lam):
    """SB3 RolloutBuffer.compute_returns_and_advantage (stable_baselines3 2.3.2 common/buffers.py):
    reverse scan over time, vectorised over envs.  rewards/values/dones: [T, N] (dones[t] = the
    episode_start flag of step t, as SB3 stores it).  Returns (advantages, returns).

    On a GPU the scan is the HIP kernel ``hs_gae`` (gae.hip, one launch per rollout); on the CPU
    (tests, toy envs) it is this torch loop."""
    if rewards.is_cuda:
        return gae_device(rewards, values, dones, last_values, last_dones, gamma, lam)
    T = rewards.shape[0]
    adv = torch.zeros_like(rewards)
    last = torch.zeros_like(last_values)
    for t in range(T - 1, -1, -1):
        if t == T - 1:
            nonterm = 1.0 - last_dones
            nv = last_values
        else:
            nonterm = 1.0 - dones[t + 1]
            nv = values[t + 1]
        delta = rewards[t] + gamma * nv * nonterm - values[t]
        last = delta + gamma * lam * nonterm * last
        adv[t] = last
    return adv, adv + values


def minibatch_weights(counts, rank, n_steps, n_minibatches):
    """Gradient weight of each of rank ``rank``'s minibatches in the world-plan of
    PPO._plan_minibatches: rank r splits its n_steps * counts[r] samples into n_minibatches
    chunks at (j * M_r) // n_minibatches, and minibatch j's weight is its chunk's share of the
    global minibatch j (the sum over ranks), so the all-reduced sum is the global mean."""
    nmb = n_minibatches
    def size(c, j):
        m = n_steps * c
        return ((j + 1) * m) // nmb - (j * m) // nmb
    return [size(counts[rank], j) / sum(size(c, j) for c in counts) for j in range(nmb)]


class PPO:
    """PPO over a device vec-env (HumanoidVecEnv's fast path).

    The env protocol: ``num_envs``, ``obs_dim``, ``act_dim``, ``device``, ``reset_tensors()``,
    ``step_tensors(actions) -> (obs, reward, terminated, truncated)`` on device, and
    ``terminal_obs`` (pre-reset obs of envs that just finished).  ``world_size``/``rank``
    default to the initialised torch.distributed group (one process per GPU, envs sharded).
    """

    def __init__(self, env, learning_rate=3e-4, n_steps=2048, batch_size=64, n_epochs=10, gamma=0.99,
                 gae_lambda=0.95, clip_range=0.2, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5,
                 policy_kwargs=None, seed=0, world_size=None, rank=None, sync_grads=None, stagger_episodes=False,
                 normalize_advantage=True):
        import torch.distributed as dist
        if world_size is None:
            world_size = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        if rank is None:
            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        # sync_grads: all-reduce the gradient bucket every optimizer step (default: world > 1; True
        # with a world-1 group runs the collective anyway -- the RCCL smoke test of tests/)
        self.sync_grads = world_size > 1 if sync_grads is None else bool(sync_grads)
        if self.sync_grads and not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("PPO: gradient sync needs an initialised torch.distributed process group "
                               f"(world_size={world_size}); see train.init_distributed")
        pk = dict(policy_kwargs or {})
        net = pk.get("net_arch", {"pi": [64, 64], "vf": [64, 64]})
        if isinstance(net, (list, tuple)):
            net = {"pi": list(net), "vf": list(net)}
        act = pk.get("activation_fn", nn.Tanh)
        if isinstance(act, str):
            act = getattr(nn, act)
        self.env = env
        self.policy_kwargs, self.net_arch, self.learning_rate = pk, net, learning_rate
        self.device = torch.device(env.device)
        torch.manual_seed(seed)          # identical initial weights on every rank
        self.policy = ActorCritic(env.obs_dim, env.act_dim, net["pi"], net["vf"], act,
                                  pk.get("log_std_init", 0.0)).to(self.device)
        torch.manual_seed(seed + 7919 * rank)   # per-rank exploration noise / minibatch order
        # fused (single-kernel) Adam on a device; the same update rule and state_dict as foreach Adam
        cuda = self.device.type == "cuda"
        self.opt = torch.optim.Adam(self.policy.parameters(), lr=learning_rate, eps=1e-5,
                                    fused=True if cuda else None, capturable=cuda)
        # on a device the minibatch step replays as HIP graphs (see _build_graphs); the update is
        # launch-bound without them (~1.3 ms of kernels per 32768-sample step, ~1.7 ms eager)
        self.graphs = cuda
        self._graphs = None
        self.n_steps, self.batch_size, self.n_epochs = n_steps, batch_size, n_epochs
        self.gamma, self.gae_lambda, self.clip_range = gamma, gae_lambda, clip_range
        self.ent_coef, self.vf_coef, self.max_grad_norm = ent_coef, vf_coef, max_grad_norm
        # SB3 PPO's normalize_advantage (default True): per-minibatch mean / std; with world > 1 each
        # rank normalises its own chunk of the global minibatch (tests/test_ppo.py equal-result test)
        self.normalize_advantage = bool(normalize_advantage)
        self.world_size, self.rank = world_size, rank
        N, T, D, A = env.num_envs, n_steps, env.obs_dim, env.act_dim
        self._plan_minibatches(N)
        f, dev = torch.float32, self.device
        self.buf = dict(obs=torch.zeros(T, N, D, dtype=f, device=dev), act=torch.zeros(T, N, A, dtype=f, device=dev),
                        rew=torch.zeros(T, N, dtype=f, device=dev), start=torch.zeros(T, N, dtype=f, device=dev),
                        val=torch.zeros(T, N, dtype=f, device=dev), logp=torch.zeros(T, N, dtype=f, device=dev),
                        done=torch.zeros(T, N, dtype=torch.bool, device=dev),
                        epret=torch.zeros(T, N, dtype=torch.float64, device=dev))
        if dev.type == "cuda":   # device rollout: deferred TimeLimit bootstrap (flags + terminal obs rows)
            self.buf.update(boot=torch.zeros(T, N, dtype=torch.bool, device=dev),
                            tobs=torch.zeros(T, N, D, dtype=f, device=dev))
        self.obs = env.reset_tensors().float().clone()
        # stagger_episodes: spread the envs' episode clocks after this first reset (not an SB3 option;
        # HumanoidVecEnv.stagger_episode_clocks) so that short rollouts see every episode phase
        if stagger_episodes:
            if not hasattr(env, "stagger_episode_clocks"):
                raise ValueError("stagger_episodes=True needs an env with stagger_episode_clocks() (HumanoidVecEnv)")
            env.stagger_episode_clocks()
        elif hasattr(env, "episode_length") and N > 1 and 2 * n_steps < env.episode_length():
            import warnings
            warnings.warn(f"PPO: rollouts of n_steps={n_steps} cover a small part of the {env.episode_length()}-step "
                          "episode and every env resets together, so each rollout sees one phase of it; "
                          "stagger_episodes=True spreads the envs' episode clocks (profiles/learning_curve_r5.md)",
                          RuntimeWarning, stacklevel=2)
        self.episode_start = torch.ones(N, dtype=f, device=dev)
        self.num_timesteps = 0
        self.ep_returns = []
        self.ep_acc = torch.zeros(N, dtype=torch.float64, device=dev)
        self.flat = [p for p in self.policy.parameters()]
        # device rollout: the clipped actions the env steps with, and the Philox noise stream
        self._act_clip = torch.zeros(N, A, dtype=f, device=dev)
        self._zero_n = torch.zeros(N, dtype=f, device=dev)        # value input of hs_ppo_act (values are
        self._val_scratch = torch.zeros(N, dtype=f, device=dev)   # filled once per rollout, see below)
        self._noise_seed = (int(seed) + 7919 * rank) * 0x9E3779B97F4A7C15 % 2 ** 64
        self._noise_ctr = torch.zeros(1, dtype=torch.int64, device=dev)    # Philox step counter (device)
        self._rollout_graph = None
        self.logger = {}

    def collect_rollouts(self):
        if self.device.type == "cuda":
            return self._collect_rollouts_device()
        return self._collect_rollouts_torch()

    def _collect_rollouts_device(self):
        """collect_rollouts on the GPU: per env step the packed policy GEMM chain, one hs_ppo_act
        launch (sample, log-prob, clip, buffer writes), the env kernel and one hs_ppo_post launch
        (dones, returns, obs -> slot t+1, and the TimeLimit.truncated envs' flags and terminal obs).
        No host synchronisation inside the loop.  The bootstrap r += gamma V(terminal obs) of the
        truncated envs is applied once after the loop, with one value forward over just those rows
        (the policy is fixed during the rollout, so this equals SB3's per-step evaluation)."""
        b, env, pol = self.buf, self.env, self.policy
        T, N = self.n_steps, env.num_envs
        pol.pack_heads()
        if self._fused_rollout_args() is not None:
            self._rollout_fused()
        else:
            if self.graphs and self._rollout_graph is None and getattr(env, "graph_safe", False):
                self._capture_rollout()                   # on failure: graphs off, eager body below
            if self._rollout_graph is not None:
                self._rollout_graph.replay()
            else:
                self._rollout_body()
        self.ep_returns += b["epret"][b["done"]].tolist()      # one device -> host transfer per rollout
        boot = b["boot"].view(-1).nonzero().squeeze(1)
        if boot.numel():                                        # deferred TimeLimit bootstrap
            b["rew"].view(-1)[boot] += self.gamma * pol.value(b["tobs"].view(T * N, -1)[boot])
        self.num_timesteps += T * self.n_envs_global
        last_v = pol.value(self.obs)
        return gae(b["rew"], b["val"], b["start"], last_v, self.episode_start, self.gamma, self.gae_lambda)

    def _fused_rollout_args(self):
        """(batch handle, hs_policy) when the whole rollout can run as hs_rollout launches -- the env's
        fp64 engine with the device reward (HumanoidVecEnv.rollout_handle) and a pi net of two ReLU
        layers of 256 (the reference's net_arch, README.md:44-50) -- else None."""
        if not FUSED_ROLLOUT or self.device.type != "cuda":
            return None
        handle = self.env.rollout_handle() if hasattr(self.env, "rollout_handle") else None
        pk = self.policy._packed
        if handle is None or pk is None:
            return None
        w1, b1, mid, w3, b3 = pk
        D, A = w1.shape[0], w3.shape[2]
        if (len(mid) != 1 or w1.shape[1] != 512 or D != self.env.obs_dim or D % 4 or D > 512 or A > 32
                or A != self.env.act_dim):
            return None
        from . import _lib
        ls = self.policy.log_std.detach()
        keep = (w1, b1, mid[0][0][0], mid[0][1][0, 0], w3[0], b3[0, 0], ls)
        if not all(t.is_contiguous() for t in keep):
            return None
        pol = _lib.hs_policy(*[t.data_ptr() for t in keep], w1.shape[1], D, A)
        return handle, pol, keep

    def _rollout_fused(self):
        """collect_rollouts as hs_rollout launches: this method samples step 0's action on the first obs
        (the per-step sampler, as _rollout_body), then each launch runs up to hs_rollout_max_steps env
        steps with the policy forward, sampling and buffer bookkeeping inside the env kernel
        (hs_kernels.hip step_pair), each env pair's step t + 1 starting when its own step t is done.
        The noise is hs_ppo_act's Philox stream, so the draws are those of the per-step path; the
        policy means agree with the GEMM chain to fp32 rounding (tests/test_gpu_ppo.py).  A launch
        that hits a resident-tier contact overflow is undone by the library, and the rest of the
        rollout runs step by step."""
        import ctypes as C

        from . import _lib
        b, env, pol = self.buf, self.env, self.policy
        T = self.n_steps
        handle, cpol, keep = self._fused_rollout_args()
        b["obs"][0].copy_(self.obs)
        mean = pol.net_forward(b["obs"][0], 0)
        ppo_act(mean, self._zero_n, pol.log_std.detach(), self.episode_start, self._noise_seed, 0, False,
                b["act"][0], self._act_clip, b["logp"][0], self._val_scratch, b["start"][0],
                counter_base=self._noise_ctr)
        rb = _lib.hs_rollout_bufs(b["obs"].data_ptr(), self.obs.data_ptr(), b["act"].data_ptr(), b["logp"].data_ptr(),
                                  b["start"].data_ptr(), b["rew"].data_ptr(), b["done"].data_ptr(),
                                  b["epret"].data_ptr(), b["boot"].data_ptr(), b["tobs"].data_ptr(),
                                  self.ep_acc.data_ptr(), self.episode_start.data_ptr(), self._act_clip.data_ptr(),
                                  self._noise_ctr.data_ptr(), self._noise_seed, 0)
        L = _lib.check(_lib.lib().hs_rollout_max_steps(handle))
        stream = torch.cuda.current_stream(self.device).cuda_stream
        t0 = 0
        while t0 < T:
            k = min(L, T - t0)
            rc = _lib.check(_lib.lib().hs_rollout(handle, C.byref(cpol), C.byref(rb), t0, k, T, stream))
            if rc == 0:                       # (env steps, kernel ms by HIP events) of the last launches
                ms = C.c_double(0)
                _lib.check(_lib.lib().hs_last_tape_ms(handle, C.byref(ms)))
                self.rollout_launches = (getattr(self, "rollout_launches", []) + [(k * self.env.num_envs, ms.value)])[-64:]
            if rc == 1:                       # resident-tier overflow: state restored, step by step from t0
                self.fused_fallbacks = getattr(self, "fused_fallbacks", 0) + 1
                self._rollout_body(t_from=t0)
                return
            t0 += k
        del keep
        self._rollout_tail()

    def _rollout_body(self, t_from=0):
        """The T env steps of a device rollout (what the rollout graph captures); t_from > 0: the
        rest of a rollout whose steps [0, t_from) are in the buffers (the fused path's fallback)."""
        b, env, pol = self.buf, self.env, self.policy
        T, N = self.n_steps, env.num_envs
        gamma = float(self.gamma)
        if t_from == 0:
            b["obs"][0].copy_(self.obs)
        for t in range(t_from, T):
            mean = pol.net_forward(b["obs"][t], 0) if pol._packed is not None else pol.heads(b["obs"][t])[0]
            ppo_act(mean, self._zero_n, pol.log_std.detach(), self.episode_start, self._noise_seed, t, False,
                    b["act"][t], self._act_clip, b["logp"][t], self._val_scratch, b["start"][t],
                    counter_base=self._noise_ctr)
            obs, rew, term, trunc = env.step_tensors(self._act_clip)
            nxt = b["obs"][t + 1] if t + 1 < T else self.obs
            ppo_post(rew.float(), term.to(torch.uint8), trunc.to(torch.uint8), None, gamma, obs.float(), nxt,
                     b["rew"][t], b["done"][t], self.ep_acc, b["epret"][t], self.episode_start,
                     terminal_obs=env.terminal_obs.float(), boot_obs_out=b["tobs"][t], boot_out=b["boot"][t])
        self._rollout_tail()

    def _rollout_tail(self):
        b, pol = self.buf, self.policy
        T, N = self.n_steps, self.env.num_envs
        self._noise_ctr.add_(T)
        # values of every buffered obs in one batched vf forward (SB3 stores V(obs_t) per step;
        # the policy does not change inside a rollout, so this is the same quantity)
        b["val"].view(-1).copy_(pol.net_forward(b["obs"].view(T * N, -1), 1) if pol._packed is not None
                                else pol.value(b["obs"].view(T * N, -1)))

    def _capture_rollout(self):
        """Capture the whole T-step device rollout as one HIP graph (policy GEMMs, hs_ppo_act, the
        env kernel, hs_ppo_post per step): one host call per rollout.  Every pointer it uses is
        persistent (rollout buffers, the env batch's buffers, pack_heads' weight copies) and the
        noise counter lives in device memory, so replays are exactly the eager loop.  Only the
        side-effect-free policy forward is warmed up (GEMM library handles); the env steps are
        recorded, not executed, during capture."""
        pol, b, dev = self.policy, self.buf, self.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side), torch.no_grad():
            for _ in range(2):
                pol.heads(b["obs"][0])
                pol.value(self.obs)
        torch.cuda.current_stream(dev).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._rollout_body()
            self._rollout_graph = g
        except RuntimeError as e:                  # nothing ran during capture: stay eager
            import warnings
            warnings.warn(f"rollout graph capture failed ({e}); collecting rollouts eagerly")
            self.graphs = False

    def _collect_rollouts_torch(self):
        """SB3 PPO.collect_rollouts on device.  No host synchronisation inside the loop: the
        timeout bootstrap r += gamma V(terminal_obs) is evaluated for every env and masked, and
        finished-episode returns are recorded in device buffers and read back once at the end."""
        b, env, pol = self.buf, self.env, self.policy
        for t in range(self.n_steps):
            a, logp, v = pol.act(self.obs)
            b["obs"][t] = self.obs
            b["act"][t] = a
            b["val"][t] = v
            b["logp"][t] = logp
            b["start"][t] = self.episode_start
            obs, rew, term, trunc = env.step_tensors(a.clamp(-1.0, 1.0))
            term, trunc = term.bool(), trunc.bool()
            boot = (trunc & ~term).float()          # TimeLimit.truncated: bootstrap from V(terminal obs)
            tv = pol.value(env.terminal_obs.float())
            b["rew"][t] = rew.float() + self.gamma * torch.where(boot > 0, tv, torch.zeros_like(tv))
            done = term | trunc
            self.ep_acc += rew.double()
            b["done"][t] = done
            b["epret"][t] = self.ep_acc
            self.ep_acc.masked_fill_(done, 0.0)
            self.obs = obs.float().clone()
            self.episode_start = done.float()
        self.ep_returns += b["epret"][b["done"]].tolist()      # one device -> host transfer per rollout
        self.num_timesteps += self.n_steps * self.n_envs_global
        last_v = pol.value(self.obs)
        return gae(b["rew"], b["val"], b["start"], last_v, self.episode_start, self.gamma, self.gae_lambda)

    # -- multi-rank lockstep ---------------------------------------------------------------------
    def _comm_device(self):
        import torch.distributed as dist
        return self.device if dist.get_backend() == "nccl" else torch.device("cpu")

    def _plan_minibatches(self, n_local):
        """Agree (one all-reduce at construction) on every rank's env count, then fix the per-epoch
        minibatch plan so that every rank issues the same number of gradient all-reduces:

        * world 1: SB3's plan -- ceil(M / batch_size) minibatches of batch_size, the last one short;
        * world > 1: n_mb = max over ranks of ceil(M_r / batch_size) minibatches per epoch on EVERY
          rank, each rank splitting its own permutation of M_r = n_steps * N_r samples into n_mb
          near-equal chunks (sizes differ by at most one; equal to batch_size for even shards whose
          M_r is a multiple of it, i.e. the usual case).  Gradients are weighted by the rank's share
          M_r / M_total before the sum, so uneven shards count per sample.
        """
        world, T, bs = self.world_size, self.n_steps, self.batch_size
        if self.sync_grads:      # independent trainers (sync_grads=False) plan locally, no collective
            import torch.distributed as dist
            counts = torch.zeros(world, dtype=torch.int64, device=self._comm_device())
            counts[self.rank] = n_local
            dist.all_reduce(counts)
            counts = [int(c) for c in counts.cpu()]
            if counts[self.rank] != n_local or min(counts) <= 0:
                raise RuntimeError(f"PPO: inconsistent env counts across ranks: {counts}")
        else:
            counts = [n_local]
        self.env_counts = counts
        self.n_envs_global = sum(counts)
        M = T * n_local
        if world == 1 or not self.sync_grads:
            self.n_minibatches = -(-M // bs)
            self._mb_bounds = [min(s, M) for s in range(0, M + bs, bs)][: self.n_minibatches + 1]
            self._mb_bounds[-1] = M
        else:
            self.n_minibatches = max(-(-(T * c) // bs) for c in counts)
            if T * min(counts) < self.n_minibatches:
                raise ValueError(f"batch_size={bs} is too small for env shards {counts} x n_steps={T}: "
                                 "a rank would get an empty minibatch")
            self._mb_bounds = [(j * M) // self.n_minibatches for j in range(self.n_minibatches + 1)]
        sizes = {b - a for a, b in zip(self._mb_bounds, self._mb_bounds[1:])}
        self._chunk = sizes.pop() if len(sizes) == 1 else None     # uniform minibatch size (graphable)
        # minibatch j's gradient is weighted by this rank's share of the global minibatch j,
        # s_r(j) / sum_r' s_r'(j) (every rank's chunk sizes follow from the agreed counts), so the
        # summed bucket is the mean over the global minibatch for even and uneven shards alike
        self._mb_weight = (minibatch_weights(counts, self.rank, T, self.n_minibatches)
                           if self.sync_grads and world > 1 else [1.0] * self.n_minibatches)
        self.grad_weight = self._mb_weight[0]

    def _agree_stop(self, stop):
        """Every rank leaves learn() at the same iteration (a callback may stop one rank only)."""
        if self.world_size == 1:
            return stop
        import torch.distributed as dist
        f = torch.tensor([1 if stop else 0], dtype=torch.int32, device=self._comm_device())
        dist.all_reduce(f, op=dist.ReduceOp.MAX)
        return bool(f.item())

    def _allreduce_flat(self, flat):
        import torch.distributed as dist
        if flat.is_cuda and dist.get_backend() == "gloo":     # multi-rank rehearsal without RCCL
            host = flat.cpu()
            dist.all_reduce(host)
            flat.copy_(host)
        else:
            dist.all_reduce(flat)        # ONE RCCL all-reduce per optimizer step (xGMI ring)

    def _allreduce_grads(self):
        if not self.sync_grads:
            return
        grads = [p.grad for p in self.flat]
        flat = torch.cat([g.reshape(-1) for g in grads])
        flat.mul_(self.grad_weight)      # this rank's share of the samples (1/world for even shards)
        self._allreduce_flat(flat)
        o = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[o:o + n].view_as(g))
            o += n

    def _minibatch_loss(self, obs, act, old_logp, adv, ret, idx):
        """SB3 PPO.train's per-minibatch loss (clipped surrogate + vf_coef MSE - ent_coef entropy)."""
        mean, v = self.policy(obs[idx])
        logp = self.policy._logp(mean, act[idx])
        if logp.is_cuda:                            # fused HIP loss (same formulas as below)
            pg, vf = ppo_loss(logp, v, idx, adv, ret, old_logp, self.clip_range, self.normalize_advantage)
            loss = torch.add(pg, vf, alpha=self.vf_coef)
            if self.ent_coef:                       # SB3's default ent_coef 0: no term, no launches
                loss = loss - self.ent_coef * self.policy.entropy()
            return loss, pg, vf
        ent_mean = self.policy.entropy()            # = evaluate()'s per-sample entropy, averaged
        a = adv[idx]
        if self.normalize_advantage and a.numel() > 1:
            a = (a - a.mean()) / (a.std() + 1e-8)
        ratio = torch.exp(logp - old_logp[idx])
        pg = -torch.min(a * ratio, a * ratio.clamp(1 - self.clip_range, 1 + self.clip_range)).mean()
        vf = torch.nn.functional.mse_loss(ret[idx], v)
        return pg + self.ent_coef * (-ent_mean) + self.vf_coef * vf, pg, vf

    def train(self, adv, ret):
        b = self.buf
        T, N = self.n_steps, self.env.num_envs
        M = T * N
        if self.device.type == "cuda" and self.graphs and self._chunk is not None:
            return self._train_graphed(adv, ret)
        obs = b["obs"].reshape(M, -1)
        act = b["act"].reshape(M, -1)
        old_logp = b["logp"].reshape(-1)
        adv, ret = adv.reshape(-1), ret.reshape(-1)
        stats = []
        for epoch in range(self.n_epochs):
            perm = torch.randperm(M, device=self.device)
            for j, (s, e) in enumerate(zip(self._mb_bounds, self._mb_bounds[1:])):
                self.grad_weight = self._mb_weight[j]
                loss, pg, vf = self._minibatch_loss(obs, act, old_logp, adv, ret, perm[s:e])
                self.opt.zero_grad(set_to_none=True)
                loss.backward()
                self._allreduce_grads()
                self._clip_and_step()
                stats.append((pg.detach(), vf.detach()))
        pg = torch.stack([s[0] for s in stats]).mean().item()
        vf = torch.stack([s[1] for s in stats]).mean().item()
        return dict(policy_loss=pg, value_loss=vf)

    def _clip_and_step(self):
        """clip_grad_norm_(max_grad_norm) + Adam step: hs_adam_clip on a device, torch on the CPU."""
        params = self.flat
        if params[0].is_cuda:
            self._adam_ws = adam_clip_step(self.opt, params, self.max_grad_norm, getattr(self, "_adam_ws", None))
        else:
            torch.nn.utils.clip_grad_norm_(params, self.max_grad_norm)
            self.opt.step()

    # -- HIP-graph update ----------------------------------------------------------------------
    def _build_graphs(self):
        """Capture one minibatch step as two HIP graphs over static buffers: G1 = gather by the
        static index buffer + forward + loss + backward (gradients land in graph-owned .grad
        tensors and, for world > 1, are packed into one flat bucket), G2 = unpack/average the
        bucket + clip_grad_norm + capturable fused Adam.  The per-step RCCL all-reduce of the
        bucket (world > 1) is the one eager call between the two replays.  The warm-up steps
        capture needs are undone (parameters and Adam state restored in place), so graphed
        training takes exactly the eager path's optimizer steps."""
        b, M, bs = self.buf, self.n_steps * self.env.num_envs, self._chunk
        dev = self.device
        self._g_idx = torch.zeros(bs, dtype=torch.long, device=dev)
        self._g_adv = torch.zeros(M, dtype=torch.float32, device=dev)
        self._g_ret = torch.zeros(M, dtype=torch.float32, device=dev)
        self._g_stats = torch.zeros(2, dtype=torch.float32, device=dev)
        src = (b["obs"].view(M, -1), b["act"].view(M, -1), b["logp"].view(-1), self._g_adv, self._g_ret)
        params = list(self.policy.parameters())

        sync = self.sync_grads
        self._g_flat = torch.zeros(sum(p.numel() for p in params), dtype=torch.float32, device=dev) if sync else None
        self._g_w = torch.full((1,), float(self._mb_weight[0]), dtype=torch.float32, device=dev)

        def g1_body():
            loss, pg, vf = self._minibatch_loss(*src, self._g_idx)
            loss.backward()
            self._g_stats.add_(torch.stack([pg.detach(), vf.detach()]))
            if sync:                     # the weighted gradient bucket the eager all-reduce sends
                torch.cat([p.grad.reshape(-1) for p in params], out=self._g_flat)
                self._g_flat.mul_(self._g_w)     # minibatch weight, refreshed before each replay

        def g2_body():
            if sync:                     # summed bucket back into the .grad tensors
                o = 0
                for p in params:
                    n = p.numel()
                    p.grad.copy_(self._g_flat[o:o + n].view_as(p.grad))
                    o += n
            self._clip_and_step()

        saved_p = [p.detach().clone() for p in params]
        saved_s = {id(p): {k: v.clone() for k, v in self.opt.state[p].items()} for p in params if p in self.opt.state}
        self._g_idx.copy_(torch.arange(bs, device=dev))
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):
                self.opt.zero_grad(set_to_none=True)
                g1_body()
                g2_body()
        torch.cuda.current_stream(dev).wait_stream(side)
        self.opt.zero_grad(set_to_none=True)
        pool = torch.cuda.graph_pool_handle()
        g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        try:
            # thread_local: RCCL's proxy threads (world > 1) may touch the runtime meanwhile
            with torch.cuda.graph(g1, pool=pool, capture_error_mode="thread_local"):
                g1_body()
            with torch.cuda.graph(g2, pool=pool, capture_error_mode="thread_local"):
                g2_body()
            self._graphs = (g1, g2)
            if not sync:
                # world 1: the whole epoch -- every minibatch's gather, forward, loss, backward, clip and
                # Adam, indices read from slices of one static permutation buffer -- as ONE graph, so
                # small minibatches (README.md:23-53: batch 128, 128 steps per epoch) cost one replay
                # per epoch instead of two per minibatch.  Each step starts from .grad = None, so its
                # backward writes fresh gradients exactly as G1 does.
                self._g_perm = torch.zeros(M, dtype=torch.long, device=dev)
                ge = torch.cuda.CUDAGraph()
                with torch.cuda.graph(ge, pool=pool, capture_error_mode="thread_local"):
                    for s0, e0 in zip(self._mb_bounds, self._mb_bounds[1:]):
                        self.opt.zero_grad(set_to_none=True)
                        loss, pg, vf = self._minibatch_loss(*src, self._g_perm[s0:e0])
                        loss.backward()
                        self._g_stats.add_(torch.stack([pg.detach(), vf.detach()]))
                        self._clip_and_step()
                self._epoch_graph = ge
        except RuntimeError as e:                  # capture refused: train eagerly from here on
            import warnings
            warnings.warn(f"PPO update graph capture failed ({e}); falling back to the eager update")
            self.graphs = False
            self._graphs = None
            self.opt.zero_grad(set_to_none=True)
        finally:
            with torch.no_grad():                  # undo the warm-up steps in place
                for p, q in zip(params, saved_p):
                    p.copy_(q)
                for p in params:
                    st, old = self.opt.state.get(p, {}), saved_s.get(id(p))
                    for k, v in st.items():
                        if old is not None and k in old:
                            v.copy_(old[k])
                        elif torch.is_tensor(v):
                            v.zero_()

    def _train_graphed(self, adv, ret):
        if self._graphs is None:
            self._build_graphs()
            if self._graphs is None:
                return self.train(adv, ret)       # capture failed: self.graphs is now False
        g1, g2 = self._graphs
        M = self.n_steps * self.env.num_envs
        self._g_adv.copy_(adv.reshape(-1))
        self._g_ret.copy_(ret.reshape(-1))
        self._g_stats.zero_()
        n = 0
        ge = getattr(self, "_epoch_graph", None)
        for epoch in range(self.n_epochs):
            perm = torch.randperm(M, device=self.device)
            if ge is not None:                    # world 1: one replay per epoch
                self._g_perm.copy_(perm)
                ge.replay()
                n += len(self._mb_bounds) - 1
                continue
            for j, (s, e) in enumerate(zip(self._mb_bounds, self._mb_bounds[1:])):
                self._g_idx.copy_(perm[s:e])
                if self.sync_grads:
                    self._g_w.fill_(self._mb_weight[j])
                g1.replay()
                if self.sync_grads:
                    self._allreduce_flat(self._g_flat)
                g2.replay()
                n += 1
        pg, vf = (self._g_stats / n).tolist()
        return dict(policy_loss=pg, value_loss=vf)

    WARN_KINDS = _batch_mod.WARN_KINDS

    def _check_env_warnings(self):
        """Once per rollout: the env's warning counters (include/hsim.h HS_WARN_*) since the last
        check, summed over ranks.  Bad-state resets are reported the way MuJoCo's mj_step reports
        them (mju_warning: the state was reset with mj_resetData and the run goes on; custom_env.py:160);
        a lost chunk-queue hand-off is a scheduling failure, not physics, so it raises on every
        rank (batch.report_warnings).  Returns the new counts (also in ``logger["env_warnings"]``)."""
        fn = getattr(self.env, "warning_counts", None)
        if fn is None:
            return None
        tot = np.asarray(fn(), dtype=np.int64)
        prev = getattr(self, "_warn_seen", None)
        new = np.maximum(tot - prev, 0) if prev is not None and prev.shape == tot.shape else tot
        self._warn_seen = tot
        if self.world_size > 1:
            import torch.distributed as dist
            t = torch.as_tensor(new, dtype=torch.int64, device=self._comm_device())
            dist.all_reduce(t)
            new = t.cpu().numpy()
        self._warn_new = new
        _batch_mod.report_warnings(new, "rollout")
        return new

    def learn(self, total_timesteps, callback=None, log_interval=1):
        it = 0
        while self.num_timesteps < total_timesteps:
            t0 = time.perf_counter()
            adv, ret = self.collect_rollouts()
            warn = self._check_env_warnings()
            t1 = time.perf_counter()
            st = self.train(adv, ret)
            t2 = time.perf_counter()
            it += 1
            mean_ret = float(np.mean(self.ep_returns[-100:])) if self.ep_returns else float("nan")
            self.logger = dict(iteration=it, timesteps=self.num_timesteps, rollout_s=t1 - t0, train_s=t2 - t1,
                               ep_rew_mean=mean_ret, **st)
            if warn is not None:
                self.logger["env_warnings"] = [int(x) for x in warn]
            if self._agree_stop(callback is not None and callback(self) is False):
                break
        return self

    @torch.no_grad()
    def predict(self, observation, state=None, episode_start=None, deterministic=False):
        """SB3 BaseAlgorithm.predict (render_policy.py:30): obs (obs_dim,) or (n, obs_dim) ->
        (actions clipped to [-1, 1] as numpy, None)."""
        obs = torch.as_tensor(np.asarray(observation), dtype=torch.float32, device=self.device)
        single = obs.dim() == 1
        a, _, _ = self.policy.act(obs[None] if single else obs, deterministic=deterministic)
        a = a.clamp(-1.0, 1.0).cpu().numpy()
        return (a[0] if single else a), None

    def _data(self):
        act = self.policy_kwargs.get("activation_fn", nn.Tanh)
        return {"n_steps": self.n_steps, "batch_size": self.batch_size, "n_epochs": self.n_epochs,
                "gamma": self.gamma, "gae_lambda": self.gae_lambda, "clip_range": self.clip_range,
                "ent_coef": self.ent_coef, "vf_coef": self.vf_coef, "max_grad_norm": self.max_grad_norm,
                "learning_rate": self.learning_rate, "num_timesteps": self.num_timesteps,
                "n_envs": self.n_envs_global,
                "policy_kwargs": {"net_arch": self.net_arch,
                                  "activation_fn": act if isinstance(act, str) else act.__name__}}

    def save(self, path):
        """SB3 checkpoint layout (train_sb3.py:234 ``model.save``): writes ``path``.zip."""
        from .sb3_format import save_sb3_zip
        return save_sb3_zip(path, self.policy, self.opt, self._data())

    def load(self, path):
        """Load weights + optimizer state from an SB3-layout zip (ours or SB3's own)."""
        from .sb3_format import load_sb3_zip
        data = load_sb3_zip(path, self.policy, self.opt, map_location=self.device)
        self._graphs = None          # optimizer state tensors were replaced: recapture
        self.num_timesteps = int(data.get("num_timesteps", 0))
        return self
