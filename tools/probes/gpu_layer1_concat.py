"""Would one layer-1 GEMM for both nets beat two?  The pi and vf nets read the same minibatch obs
[32768, 352]; per minibatch the update runs layer 1 forward twice ([352 -> 256], ReLU epilogue) and
its split-K weight gradient twice.  Times (median of 50, HIP events) both shapes of both GEMMs.
    python tools/probes/gpu_layer1_concat.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def timed(fn, n=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(n):
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[n // 2]


def main():
    B, D, S = 32768, 352, 16
    x = torch.randn(B, D, device="cuda")
    res = {}
    for H in (256, 512):
        w = torch.randn(H, D, device="cuda") * 0.05
        b = torch.randn(H, device="cuda")
        g = torch.randn(B, H, device="cuda")
        res[f"fwd_{H}"] = timed(lambda: torch._addmm_activation(b, x, w.t()))
        res[f"wgrad_{H}"] = timed(lambda: torch.bmm(g.view(S, -1, H).transpose(1, 2), x.view(S, -1, D)))
    res["fwd_two_256_vs_one_512"] = [2 * res["fwd_256"], res["fwd_512"]]
    res["wgrad_two_256_vs_one_512"] = [2 * res["wgrad_256"], res["wgrad_512"]]
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else [round(t, 1) for t in v]) for k, v in res.items()}))


if __name__ == "__main__":
    main()
