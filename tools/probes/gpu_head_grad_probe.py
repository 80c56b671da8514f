"""Value-head (out = 1) / action-head (out = 21) gradient variants at the PPO minibatch size.
python tools/probes/gpu_head_grad_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mujocoposelearning_amd.ppo_ops import colsum  # noqa: E402


def t(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / reps


def main(B=32768, S=16, inp=256):
    for out in (1, 21):
        x = torch.randn(B, inp, device="cuda")
        g = torch.randn(B, out, device="cuda")
        w = torch.randn(out, inp, device="cuda")
        ref = g.t() @ x
        res = {
            "bmm gT x + colsum": t(lambda: colsum(torch.bmm(g.view(S, -1, out).transpose(1, 2),
                                                           x.view(S, -1, inp)).view(S, -1))),
            "bmm xT g + colsum": t(lambda: colsum(torch.bmm(x.view(S, -1, inp).transpose(1, 2),
                                                           g.view(S, -1, out)).view(S, -1))),
            "dense gT x": t(lambda: g.t() @ x),
            "dx g @ w": t(lambda: g @ w),
        }
        if out == 1:
            res["mv xT g"] = t(lambda: torch.mv(x.t(), g.view(-1)))
            res["colsum(x*g)"] = t(lambda: colsum(x * g))
            res["dx g*w bcast"] = t(lambda: g * w)
            assert torch.allclose(colsum(x * g).view(1, -1), ref, rtol=1e-3, atol=1e-2)
        b2 = colsum(torch.bmm(x.view(S, -1, inp).transpose(1, 2), g.view(S, -1, out)).view(S, -1)).view(inp, out)
        assert torch.allclose(b2.t(), ref, rtol=1e-3, atol=1e-2)
        print(f"out={out}:", {k: round(v, 1) for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
