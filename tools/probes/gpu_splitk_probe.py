"""Split-K weight-gradient reduction variants (ppo.Linear backward).  python tools/probes/gpu_splitk_probe.py"""
import time

import torch


def t(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / reps


def main():
    dev = "cuda"
    B = 32768
    for (i, o) in ((352, 256), (256, 256), (256, 21), (256, 1)):
        x = torch.randn(B, i, device=dev)
        g = torch.randn(B, o, device=dev)
        ref = g.t() @ x
        res = {"dense": t(lambda: g.t() @ x)}
        for s in (8, 16, 32):
            gv, xv = g.view(s, -1, o), x.view(s, -1, i)
            ones = torch.ones(1, s, device=dev)
            P = torch.bmm(gv.transpose(1, 2), xv)
            res[f"bmm{s}"] = t(lambda: torch.bmm(gv.transpose(1, 2), xv))
            res[f"sum0_{s}"] = t(lambda: P.sum(0))
            res[f"gemv_{s}"] = t(lambda: (ones @ P.view(s, -1)).view(o, i))
            out = (ones @ P.view(s, -1)).view(o, i)
            assert torch.allclose(out, ref, rtol=1e-3, atol=1e-2), float((out - ref).abs().max())
        res["bias_sum0"] = t(lambda: g.sum(0))
        bref = g.sum(0)
        for s in (16, 64, 256):
            gv = g.view(s, -1, o)
            res[f"bias_sum1_{s}"] = t(lambda: gv.sum(1).sum(0))
            ones3 = torch.ones(s, 1, B // s, device=dev)
            res[f"bias_bmm_{s}"] = t(lambda: torch.bmm(ones3, gv).sum(0))
            assert torch.allclose(torch.bmm(ones3, gv).sum(0).view(-1), bref, rtol=1e-3, atol=1e-2)
        gt = g.t().contiguous()
        res["bias_rowsum_T"] = t(lambda: gt.sum(1))
        print(f"{o}x{i}:", {k: round(v, 1) for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
