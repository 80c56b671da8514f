"""Timing of the fused policy-MLP forward (ppo.hip mlp2_fwd_kernel) against the torch GEMM chain
(addmm + ReLU epilogues) at the rollout's two shapes: the pi net per env step (4096 rows) and the
vf net over a rollout buffer (32 x 4096 rows).  HIP events on the current stream; FLOP/s counts the
three layers' 2 N (D H + H H + H A) multiply-adds.   python tools/probes/gpu_mlp2_fwd.py
(profiles/r5i/mlp2_probe_rb{1,2}.log were taken with a build that let HSIM_MLP_RB force the row
blocks per wave; the launcher now picks them by row count, ppo.hip MLP_RB2_ROWS)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mujocoposelearning_amd.ppo_ops import mlp2_forward  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    torch.manual_seed(0)
    D, H = 352, 256
    out = {}
    for N, A, reps in ((4096, 21, 200), (8192, 21, 100), (16384, 21, 50), (32768, 1, 40), (131072, 1, 20),
                       (131072, 21, 20)):
        x = torch.randn(N, D, device="cuda")
        w1, b1 = torch.randn(H, D, device="cuda") * 0.05, torch.randn(H, device="cuda") * 0.1
        w2, b2 = torch.randn(H, H, device="cuda") * 0.05, torch.randn(H, device="cuda") * 0.1
        w3, b3 = torch.randn(A, H, device="cuda") * 0.05, torch.randn(A, device="cuda") * 0.1
        w1t, w2t, w3t = w1.t().contiguous(), w2.t().contiguous(), w3.t().contiguous()

        def fused():
            return mlp2_forward(x, w1, b1, w2, b2, w3, b3)

        def chain():
            h = torch._addmm_activation(b1, x, w1t)
            h = torch._addmm_activation(b2, h, w2t)
            return torch.addmm(b3, h, w3t)

        err = float((fused() - chain()).abs().max())
        flop = 2.0 * N * (D * H + H * H + H * A)
        tf, tc = timed(fused, reps), timed(chain, reps)
        out[f"N{N}_A{A}"] = {"fused_ms": tf, "chain_ms": tc, "fused_tflops": flop / tf / 1e9,
                             "chain_tflops": flop / tc / 1e9, "max_abs_diff": err}
        print(json.dumps({f"N{N}_A{A}": out[f"N{N}_A{A}"]}), flush=True)


def heads():
    """ActorCritic.heads at 4096 rows: the packed pi+vf GEMM chain against two fused launches."""
    from mujocoposelearning_amd import ppo as P
    torch.manual_seed(0)
    pol = P.ActorCritic(352, 21, [256, 256], [256, 256], torch.nn.ReLU).cuda()
    pol.pack_heads()
    obs = torch.randn(4096, 352, device="cuda")
    res = {}
    with torch.no_grad():
        chain = lambda: pol.heads(obs) if not P.FUSED_MLP else None  # noqa: E731
        P.FUSED_MLP = False
        res["packed_chain_ms"] = timed(lambda: pol.heads(obs), 200)
        res["net_forward_chain_ms"] = timed(lambda: (pol.net_forward(obs, 0), pol.net_forward(obs, 1)), 200)
        P.FUSED_MLP = True
        res["net_forward_fused_ms"] = timed(lambda: (pol.net_forward(obs, 0), pol.net_forward(obs, 1)), 200)
        del chain
    print(json.dumps({"heads_4096": res}), flush=True)


if __name__ == "__main__":
    heads()
    main()
