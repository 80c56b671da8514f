"""PPO minibatch fwd+bwd timing probe: autograd nn.Linear vs split-K weight gradients (and the
pi/vf first layers fused into one GEMM).  python tools/probes/gpu_mlp_probe.py"""
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


class SplitK(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, s):
        ctx.save_for_backward(x, w)
        ctx.s = s
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        s = ctx.s
        B = x.shape[0]
        gx = g @ w if ctx.needs_input_grad[0] else None
        gw = torch.bmm(g.view(s, B // s, -1).transpose(1, 2), x.view(s, B // s, -1)).sum(0)
        gb = g.sum(0)
        return gx, gw, gb, None


def mlp(x, layers, s, fused_first=None):
    for i, (w, b) in enumerate(layers):
        x = SplitK.apply(x, w, b, s) if s else torch.nn.functional.linear(x, w, b)
        if i < len(layers) - 1:
            x = torch.relu(x)
    return x


def run(B=32768, reps=30):
    dev = "cuda"
    torch.manual_seed(0)
    mk = lambda o, i: (torch.randn(o, i, device=dev, requires_grad=True) * 0.05).detach().requires_grad_()  # noqa
    pi = [(mk(256, 352), torch.zeros(256, device=dev, requires_grad=True)),
          (mk(256, 256), torch.zeros(256, device=dev, requires_grad=True)),
          (mk(21, 256), torch.zeros(21, device=dev, requires_grad=True))]
    vf = [(mk(256, 352), torch.zeros(256, device=dev, requires_grad=True)),
          (mk(256, 256), torch.zeros(256, device=dev, requires_grad=True)),
          (mk(1, 256), torch.zeros(1, device=dev, requires_grad=True))]
    obs = torch.randn(B, 352, device=dev)

    def step(s, fuse):
        if fuse:
            w1 = torch.cat([pi[0][0], vf[0][0]])
            b1 = torch.cat([pi[0][1], vf[0][1]])
            h = torch.relu(SplitK.apply(obs, w1, b1, s) if s else torch.nn.functional.linear(obs, w1, b1))
            hp, hv = h[:, :256], h[:, 256:]
            m = mlp(hp, pi[1:], s)
            v = mlp(hv, vf[1:], s)
        else:
            m = mlp(obs, pi, s)
            v = mlp(obs, vf, s)
        loss = (m * m).sum() + (v * v).sum()
        loss.backward()

    for s, fuse in [(0, False), (0, True), (4, False), (8, False), (16, False), (8, True), (16, True), (32, True)]:
        for _ in range(3):
            step(s, fuse)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            step(s, fuse)
        torch.cuda.synchronize()
        print(f"split={s:2d} fuse_first={fuse}: {1e3 * (time.perf_counter() - t) / reps:.3f} ms fwd+bwd", flush=True)


if __name__ == "__main__":
    run()
