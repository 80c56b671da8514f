"""Device operators of the on-device PPO (ppo.py): thin torch wrappers over the HIP kernels of
csrc/ppo.hip and csrc/gae.hip (through the C ABI, include/hsim.h) plus the autograd functions that
use them in the update.  Every operator here runs on a GPU only; ppo.py keeps the torch
restatement for CPU tensors (toy envs, tests).

* rollout: ppo_act (Gaussian sample + log-prob + clip + buffer writes), ppo_post (bootstrap,
  dones, returns, next obs), gae_device (GAE reverse scan)
* update: _GaussLogpFn (log-prob fwd/bwd), _PPOLossFn / ppo_loss (clipped surrogate + value MSE
  fwd/bwd), _SplitKLinearFn / _SplitKLinearReLUFn / Linear / mlp_forward (split-K weight
  gradients, ReLU in the GEMM epilogue), _MLPChainFn / mlp_head_forward (a whole net as one node:
  input gradient + ReLU mask + bias sum fused, hs_dgrad_mask), colsum (deterministic column sums), adam_clip_step
  (clip_grad_norm_ + Adam on a torch Adam's own state)
"""
from __future__ import annotations

import torch
import torch.nn as nn

_SPLITK_ROWS = 2048      # rows per split-K slice of a weight gradient
SPLIT_K = True           # module switch (A/B probes)


class _SplitKLinearFn(torch.autograd.Function):
    """y = x W^T + b whose weight gradient is computed as S batched [out x rows] x [rows x in]
    products summed over S, instead of one GEMM with a K = batch-size reduction.  The library's
    kernel for a 256 x 32768 x 352 weight gradient runs at a few TFLOP/s (one long reduction on few
    tiles); split into 16 slices it fills the chip (tools/probes/gpu_mlp_probe.py: minibatch fwd+bwd
    1.45 -> 0.97 ms at 32768 samples)."""

    @staticmethod
    def forward(ctx, x, w, b, s):
        ctx.save_for_backward(x, w)
        ctx.s = s
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        s = ctx.s
        g = g.contiguous()
        if g.shape[1] == 1:      # value head: rank-1 gradients without a K = 1 / N = 1 GEMM
            gx = g * w if ctx.needs_input_grad[0] else None
            return gx, colsum(x, g.view(-1)).view_as(w), g.sum(0), None
        gx = g @ w if ctx.needs_input_grad[0] else None
        part = torch.bmm(g.view(s, -1, g.shape[1]).transpose(1, 2), x.view(s, -1, x.shape[1]))   # [S, out, in]
        gw = colsum(part.view(s, -1)).view_as(w)
        return gx, gw, colsum(g), None


class _GaussLogpFn(torch.autograd.Function):
    """DiagGaussianDistribution.log_prob(actions) for mean [N, A] (A <= 32) on a device: one
    hs_gauss_logp launch forward; backward one hs_gauss_logp_grad launch (dL/dmean and the
    per-row dL/dlog_std terms) + hs_colsum over the rows."""

    @staticmethod
    def forward(ctx, mean, actions, log_std):
        from . import _lib
        if mean.stride(1) != 1:
            mean = mean.contiguous()
        actions = actions.contiguous()
        N, A = mean.shape
        logp = torch.empty(N, dtype=torch.float32, device=mean.device)
        st = torch.cuda.current_stream(mean.device).cuda_stream
        _lib.check(_lib.lib().hs_gauss_logp(mean.data_ptr(), mean.stride(0), actions.data_ptr(), log_std.data_ptr(),
                                            logp.data_ptr(), N, A, st))
        ctx.save_for_backward(mean, actions, log_std)
        return logp

    @staticmethod
    def backward(ctx, g):
        from . import _lib
        mean, actions, log_std = ctx.saved_tensors
        N, A = mean.shape
        g = g.contiguous()
        g_mean = torch.empty(N, A, dtype=torch.float32, device=mean.device)
        rows = torch.empty(N, A, dtype=torch.float32, device=mean.device)
        st = torch.cuda.current_stream(mean.device).cuda_stream
        _lib.check(_lib.lib().hs_gauss_logp_grad(mean.data_ptr(), mean.stride(0), actions.data_ptr(),
                                                 log_std.data_ptr(), g.data_ptr(), g_mean.data_ptr(), rows.data_ptr(),
                                                 N, A, st))
        return g_mean, None, colsum(rows)


class _PPOLossFn(torch.autograd.Function):
    """SB3 PPO.train's minibatch policy/value loss (advantage normalisation, clipped surrogate,
    value MSE) over indices idx into the rollout arrays: one hs_ppo_loss launch forward, one
    hs_ppo_loss_grad launch backward (dL/dlog_prob, dL/dvalues)."""

    @staticmethod
    def forward(ctx, logp, v, idx, adv, ret, old_logp, clip, normalize=True):
        from . import _lib
        logp, v = logp.contiguous(), v.contiguous()
        B = logp.shape[0]
        dev = logp.device
        L = _lib.lib()
        pg = torch.empty((), dtype=torch.float32, device=dev)
        vf = torch.empty((), dtype=torch.float32, device=dev)
        ws = torch.empty(int(L.hs_ppo_loss_workspace(B)), dtype=torch.float32, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(L.hs_ppo_loss(logp.data_ptr(), v.data_ptr(), idx.data_ptr(), adv.data_ptr(), ret.data_ptr(),
                                 old_logp.data_ptr(), B, float(clip), 1 if normalize else 0, pg.data_ptr(), vf.data_ptr(),
                                 ws.data_ptr(), st))
        ctx.save_for_backward(logp, v, ws)
        ctx.clip = float(clip)
        return pg, vf

    @staticmethod
    def backward(ctx, g_pg, g_vf):
        from . import _lib
        logp, v, ws = ctx.saved_tensors
        B = logp.shape[0]
        dev = logp.device
        z = torch.zeros((), dtype=torch.float32, device=dev)
        g_pg = z if g_pg is None else g_pg.to(torch.float32).contiguous()
        g_vf = z if g_vf is None else g_vf.to(torch.float32).contiguous()
        g_logp = torch.empty(B, dtype=torch.float32, device=dev)
        g_v = torch.empty(B, dtype=torch.float32, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(_lib.lib().hs_ppo_loss_grad(logp.data_ptr(), v.data_ptr(), B, ctx.clip, ws.data_ptr(),
                                               g_pg.data_ptr(), g_vf.data_ptr(), g_logp.data_ptr(), g_v.data_ptr(),
                                               st))
        return g_logp, g_v, None, None, None, None, None, None


def ppo_loss(logp, v, idx, adv, ret, old_logp, clip, normalize=True):
    """(policy_loss, value_loss) of one minibatch on a device (hs_ppo_loss / hs_ppo_loss_grad);
    ``normalize``: SB3's normalize_advantage."""
    for t in (adv, ret, old_logp):
        assert t.dtype == torch.float32 and t.is_contiguous() and t.dim() == 1
    assert idx.dtype == torch.int64 and idx.is_contiguous()
    return _PPOLossFn.apply(logp, v, idx, adv, ret, old_logp, clip, normalize)


def adam_clip_step(opt, params, max_norm, workspace=None):
    """clip_grad_norm_(params, max_norm) + opt.step() for a single-group torch Adam on a device in
    three HIP launches (hs_adam_clip).  Reads and updates the optimizer's own state tensors
    (exp_avg, exp_avg_sq, capturable float32 step), so torch's state_dict / SB3 checkpoints see
    the same state; initialises it the way torch's Adam does on its first step.  Returns the
    workspace (reuse it: a persistent buffer keeps graph captures valid)."""
    import ctypes as C
    from . import _lib
    grp = opt.param_groups[0]
    assert len(opt.param_groups) == 1 and not grp.get("amsgrad") and not grp.get("weight_decay")
    assert not grp.get("maximize") and len(params) <= 1024
    dev = params[0].device
    for p in params:
        st = opt.state[p]
        if len(st) == 0:
            st["step"] = torch.zeros((), dtype=torch.float32, device=dev)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
    L = _lib.lib()
    total = sum(p.numel() for p in params)
    if workspace is None:
        workspace = torch.empty(max(1, int(L.hs_adam_workspace(total))), dtype=torch.float32, device=dev)
    nt = len(params)
    arr = lambda xs: (C.c_void_p * nt)(*[x.data_ptr() for x in xs])   # noqa: E731
    sts = [opt.state[p] for p in params]
    b1, b2 = grp["betas"]
    _lib.check(L.hs_adam_clip(nt, arr(params), arr([p.grad for p in params]), arr([s["exp_avg"] for s in sts]),
                              arr([s["exp_avg_sq"] for s in sts]), arr([s["step"] for s in sts]),
                              (C.c_int64 * nt)(*[p.numel() for p in params]), workspace.data_ptr(),
                              float(max_norm), float(grp["lr"]), float(b1), float(b2), float(grp["eps"]),
                              torch.cuda.current_stream(dev).cuda_stream))
    return workspace


def relu_grad_colsum(g, y):
    """(g masked by y > 0, per-chunk column sums of it) through hs_relu_grad_colsum."""
    from . import _lib
    assert g.is_contiguous() and y.is_contiguous() and g.shape == y.shape and g.dim() == 2
    rows, cols = g.shape
    L = _lib.lib()
    gm = torch.empty_like(g)
    part = torch.empty(int(L.hs_colsum_partial_rows(rows, cols)), cols, dtype=torch.float32, device=g.device)
    _lib.check(L.hs_relu_grad_colsum(g.data_ptr(), y.data_ptr(), rows, cols, gm.data_ptr(), part.data_ptr(),
                                     torch.cuda.current_stream(g.device).cuda_stream))
    return gm, part


def dgrad_mask(g, w, x):
    """(g @ w masked by x > 0, per-row-block column sums of it) through hs_dgrad_mask: the input
    gradient of a Linear layer (weight w [K, 256], output gradient g [B, K]) whose input x [B, 256]
    is a ReLU output, fused with that ReLU's backward and its bias sum's first pass."""
    from . import _lib
    B, K = g.shape
    assert w.shape == (K, 256) and x.shape == (B, 256) and g.stride(1) == 1 and w.stride(1) == 1 and x.stride(1) == 1
    L = _lib.lib()
    gx = torch.empty(B, 256, dtype=torch.float32, device=g.device)
    part = torch.empty(int(L.hs_dgrad_mask_partial_rows(B, K)), 256, dtype=torch.float32, device=g.device)
    nws = int(L.hs_dgrad_mask_workspace(K))
    ws = torch.empty(nws, dtype=torch.float32, device=g.device) if nws else None
    _lib.check(L.hs_dgrad_mask(g.data_ptr(), g.stride(0), K, w.data_ptr(), w.stride(0), x.data_ptr(), x.stride(0), B,
                               256, gx.data_ptr(), part.data_ptr(), None if ws is None else ws.data_ptr(),
                               torch.cuda.current_stream(g.device).cuda_stream))
    return gx, part


def colsum_pair(x0, x1):
    """(column sums of x0, column sums of x1) for two short contiguous matrices, one launch."""
    from . import _lib
    assert x0.is_contiguous() and x1.is_contiguous() and x0.dim() == 2 and x1.dim() == 2
    o0 = torch.empty(x0.shape[1], dtype=torch.float32, device=x0.device)
    o1 = torch.empty(x1.shape[1], dtype=torch.float32, device=x1.device)
    _lib.check(_lib.lib().hs_colsum_pair(x0.data_ptr(), x0.shape[0], x0.shape[1], o0.data_ptr(), x1.data_ptr(),
                                         x1.shape[0], x1.shape[1], o1.data_ptr(),
                                         torch.cuda.current_stream(x0.device).cuda_stream))
    return o0, o1


def colsum(x, row_weight=None):
    """Column sums of a contiguous [rows, cols] float32 device matrix through hs_colsum
    (ppo.hip): deterministic, and 3-5x faster than torch's dim-0 reduction at the PPO update's
    shapes ([32768, 256] bias gradients, [16, 90112] split-K finishes)."""
    from . import _lib
    assert x.dim() == 2 and x.is_contiguous() and x.dtype == torch.float32 and x.is_cuda
    rows, cols = x.shape
    L = _lib.lib()
    ws_n = int(L.hs_colsum_workspace(rows, cols))
    ws = torch.empty(ws_n, dtype=torch.float32, device=x.device) if ws_n else None
    out = torch.empty(cols, dtype=torch.float32, device=x.device)
    if row_weight is not None:
        assert row_weight.is_contiguous() and row_weight.numel() == rows and row_weight.dtype == torch.float32
    _lib.check(L.hs_colsum(x.data_ptr(), rows, cols, None if row_weight is None else row_weight.data_ptr(),
                           ws.data_ptr() if ws is not None else None, out.data_ptr(),
                           torch.cuda.current_stream(x.device).cuda_stream))
    return out


class _SplitKLinearReLUFn(torch.autograd.Function):
    """relu(x W^T + b) with the ReLU in the GEMM's epilogue (hipBLASLt bias+ReLU through
    torch._addmm_activation: no separate activation pass over [B, out]); backward masks the
    upstream gradient with y > 0, then takes _SplitKLinearFn's split-K gradients."""

    @staticmethod
    def forward(ctx, x, w, b, s):
        y = torch._addmm_activation(b, x, w.t())
        ctx.save_for_backward(x, w, y)
        ctx.s = s
        return y

    @staticmethod
    def backward(ctx, g):
        x, w, y = ctx.saved_tensors
        s = ctx.s
        g, bias_part = relu_grad_colsum(g.contiguous(), y)  # ReLU mask + the bias sum's first pass
        gx = g @ w if ctx.needs_input_grad[0] else None
        part = torch.bmm(g.view(s, -1, g.shape[1]).transpose(1, 2), x.view(s, -1, x.shape[1]))
        gw, gb = colsum_pair(part.view(s, -1), bias_part)    # both finishes in one launch
        return gx, gw.view_as(w), gb, None


class _MLPChainFn(torch.autograd.Function):
    """head(relu(... relu(x W1^T + b1) ...)) for one SB3 MlpPolicy net (mlp_extractor's pi or vf
    half + action_net / value_net, policies.py, SB3 2.3.2) with hidden widths 256, as one autograd
    node.  Forward: each hidden layer one GEMM with the ReLU in its epilogue, the head one GEMM.
    Backward by hand, so that a layer's input gradient, the ReLU mask of the layer below and that
    layer's bias sum come out of one hs_dgrad_mask pass (autograd would write g @ w, read it back
    with the ReLU output for the mask and again for the bias sum); weight gradients split-K as
    _SplitKLinearFn, each layer's weight and bias finishes in one colsum_pair launch."""

    @staticmethod
    def forward(ctx, x, s, *params):
        ws, bs = params[0::2], params[1::2]
        ys, h = [], x
        for w, b in zip(ws[:-1], bs[:-1]):
            h = torch._addmm_activation(b, h, w.t())
            ys.append(h)
        out = torch.addmm(bs[-1], h, ws[-1].t())
        ctx.save_for_backward(x, *ys, *ws)
        ctx.s, ctx.nl = s, len(ws)
        return out

    @staticmethod
    def backward(ctx, g):
        s, nl = ctx.s, ctx.nl
        saved = ctx.saved_tensors
        x, ys, ws = saved[0], saved[1:nl], saved[nl:]
        g = g.contiguous()
        A, yl = g.shape[1], ys[-1]
        grads = [None] * (2 * nl)
        if A == 1:       # value head: a rank-1 weight gradient
            grads[-2] = colsum(yl, g.view(-1)).view_as(ws[-1])
        else:
            part = torch.bmm(g.view(s, -1, A).transpose(1, 2), yl.view(s, -1, yl.shape[1]))
            grads[-2] = colsum(part.view(s, -1)).view_as(ws[-1])
        grads[-1] = colsum(g)
        g, bias_part = dgrad_mask(g, ws[-1], yl)
        gx = None
        for li in range(nl - 2, -1, -1):
            xin = ys[li - 1] if li else x
            part = torch.bmm(g.view(s, -1, g.shape[1]).transpose(1, 2), xin.view(s, -1, xin.shape[1]))
            gw, grads[2 * li + 1] = colsum_pair(part.view(s, -1), bias_part)
            grads[2 * li] = gw.view_as(ws[li])
            if li:
                g, bias_part = dgrad_mask(g, ws[li], ys[li - 1])
            elif ctx.needs_input_grad[0]:
                gx = g @ ws[0]
        return (gx, None, *grads)


FUSED_CHAIN = True       # module switch (A/B probes)


def mlp_head_forward(seq, head, x):
    """head(seq(x)) for an MlpPolicy net (seq = [Linear, ReLU] * L, head a Linear); a large device
    minibatch with hidden widths 256 and a head of <= 32 outputs runs as one _MLPChainFn node, the
    rest through mlp_forward."""
    mods = list(seq)
    s = _splitk_rows(x)
    if (FUSED_CHAIN and s and x.dtype == torch.float32 and len(mods) >= 2 and len(mods) % 2 == 0
            and all(isinstance(m, nn.Linear) and m.out_features == 256 for m in mods[0::2])
            and all(type(m) is nn.ReLU for m in mods[1::2]) and isinstance(head, nn.Linear)
            and head.out_features <= 32 and x.stride(1) == 1):
        params = [t for m in mods[0::2] + [head] for t in (m.weight, m.bias)]
        return _MLPChainFn.apply(x, s, *params)
    return head(mlp_forward(seq, x))


def _splitk_rows(x):
    n = x.shape[0] if x.dim() == 2 else 0
    if SPLIT_K and x.is_cuda and torch.is_grad_enabled() and n >= 2 * _SPLITK_ROWS and n % _SPLITK_ROWS == 0:
        return n // _SPLITK_ROWS
    return 0


class Linear(nn.Linear):
    """nn.Linear (same parameters and state_dict keys, so SB3 checkpoints map 1:1) with split-K
    weight gradients for large device minibatches; small or CPU batches take nn.Linear's path."""

    def forward(self, x):
        s = _splitk_rows(x)
        if s:
            return _SplitKLinearFn.apply(x, self.weight, self.bias, s)
        return super().forward(x)


def mlp_forward(seq, x):
    """nn.Sequential forward that runs each (Linear, ReLU) pair of a large device minibatch as one
    fused GEMM + epilogue (_SplitKLinearReLUFn); everything else module by module."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        if (isinstance(m, Linear) and i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
                and _splitk_rows(x)):
            x = _SplitKLinearReLUFn.apply(x, m.weight, m.bias, _splitk_rows(x))
            i += 2
            continue
        x = m(x)
        i += 1
    return x


def mlp2_forward(x, w1, b1, w2, b2, w3, b3):
    """Fused forward of one 2-hidden-layer (256) ReLU MLP through hs_mlp2_forward (ppo.hip: MFMA
    tiles, one launch): x [N, D] (row stride >= D); w1 [256, D], w2 [256, 256], w3 [A, 256] in
    nn.Linear's [out][in] layout (unit column stride), b1 / b2 [256], b3 [A] contiguous; returns
    out [N, A] float32."""
    from . import _lib
    N, D = x.shape
    A = w3.shape[0]
    assert x.stride(1) == 1 and w1.stride(1) == 1 and w2.stride(1) == 1 and w3.stride(1) == 1
    assert w1.shape == (256, D) and w2.shape == (256, 256) and w3.shape[1] == 256
    out = torch.empty(N, A, dtype=torch.float32, device=x.device)
    _lib.check(_lib.lib().hs_mlp2_forward(x.data_ptr(), x.stride(0), D, N, w1.data_ptr(), w1.stride(0), b1.data_ptr(),
                                          w2.data_ptr(), w2.stride(0), b2.data_ptr(), w3.data_ptr(), w3.stride(0),
                                          b3.data_ptr(), A, out.data_ptr(), A,
                                          torch.cuda.current_stream(x.device).cuda_stream))
    return out


def gae_device(rewards, values, dones, last_values, last_dones, gamma, lam):
    """GAE through the C ABI (hs_gae) on the tensors' device and current stream; float32."""
    from . import _lib
    T, N = rewards.shape
    f32 = lambda x: x.to(torch.float32).contiguous()   # noqa: E731
    r, v, st, lv, ld = f32(rewards), f32(values), f32(dones), f32(last_values), f32(last_dones)
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    with torch.cuda.device(r.device):
        stream = torch.cuda.current_stream(r.device).cuda_stream
        _lib.check(_lib.lib().hs_gae(r.data_ptr(), v.data_ptr(), st.data_ptr(), lv.data_ptr(), ld.data_ptr(),
                                     adv.data_ptr(), ret.data_ptr(), T, N, float(gamma), float(lam), stream))
    return adv, ret


def ppo_act(mean, value, log_std, episode_start, seed, counter, deterministic, act_out, act_clip_out, logp_out,
            val_out, start_out, stream=None, counter_base=None):
    """hs_ppo_act on device tensors (ppo.hip): Gaussian sample + log-prob + clip + buffer writes.
    The Philox counter is ``counter`` plus, if given, the int64 device scalar ``counter_base``
    (read by the kernel, so a captured graph draws fresh noise on every replay)."""
    from . import _lib
    N, A = act_out.shape
    assert mean.stride(1) == 1 and mean.shape == (N, A) and value.shape == (N,), (mean.shape, value.shape)
    for t in (log_std, episode_start, act_out, act_clip_out, logp_out, val_out, start_out):
        assert t.dtype == torch.float32 and t.is_contiguous()
    st = torch.cuda.current_stream(mean.device).cuda_stream if stream is None else stream
    _lib.check(_lib.lib().hs_ppo_act(mean.data_ptr(), mean.stride(0), value.data_ptr(), value.stride(0),
                                     log_std.data_ptr(), episode_start.data_ptr(), int(seed) & (2 ** 64 - 1),
                                     int(counter), None if counter_base is None else counter_base.data_ptr(),
                                     int(bool(deterministic)), act_out.data_ptr(),
                                     act_clip_out.data_ptr(), logp_out.data_ptr(), val_out.data_ptr(),
                                     start_out.data_ptr(), N, A, st))


def ppo_post(reward, terminated, truncated, terminal_value, gamma, obs, obs_out, reward_out, done_out, ep_acc,
             ep_return_out, episode_start, terminal_obs=None, boot_obs_out=None, boot_out=None, stream=None):
    """hs_ppo_post on device tensors (ppo.hip): reward bootstrap, dones, returns, next obs copy.
    terminal_value None = deferred bootstrap: boot flags -> boot_out, terminal-obs rows of the
    boot envs -> boot_obs_out (the caller adds gamma V(row) at the end of the rollout)."""
    from . import _lib
    N = reward.shape[0]
    assert terminated.dtype == torch.uint8 and truncated.dtype == torch.uint8 and done_out.dtype == torch.bool
    assert ep_acc.dtype == torch.float64 and ep_return_out.dtype == torch.float64
    assert obs.is_contiguous() and obs_out.is_contiguous() and obs.numel() == obs_out.numel()
    ptr = lambda t: None if t is None else t.data_ptr()     # noqa: E731
    D = 0
    if terminal_value is None:
        assert terminal_obs.is_contiguous() and boot_obs_out.is_contiguous() and boot_out.dtype in (torch.bool,
                                                                                                torch.uint8)
        D = terminal_obs.shape[1]
        assert boot_obs_out.shape == terminal_obs.shape == (N, D)
    st = torch.cuda.current_stream(reward.device).cuda_stream if stream is None else stream
    _lib.check(_lib.lib().hs_ppo_post(reward.data_ptr(), terminated.data_ptr(), truncated.data_ptr(),
                                      ptr(terminal_value), ptr(terminal_obs), ptr(boot_obs_out), ptr(boot_out), D,
                                      float(gamma), obs.data_ptr(), obs_out.data_ptr(), obs.numel(),
                                      reward_out.data_ptr(), done_out.data_ptr(), ep_acc.data_ptr(),
                                      ep_return_out.data_ptr(), episode_start.data_ptr(), N, st))
