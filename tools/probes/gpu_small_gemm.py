"""The reference config's minibatch GEMMs (256 rows, MLP[64,64] on 352 obs): which formulation of
layer 1's forward and weight gradient gets the library onto more than one tile?  Median of 200
HIP-event-timed calls each (~5 us of that is the event pair's own overhead).
    python tools/probes/gpu_small_gemm.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def timed(fn, n=200):
    for _ in range(10):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(n):
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return round(sorted(ts)[n // 2], 1)


def main():
    torch.manual_seed(0)
    out = {}
    for B, D, H in ((256, 352, 64), (256, 64, 64), (1024, 352, 64), (256, 352, 256)):
        x = torch.randn(B, D, device="cuda")
        w = torch.randn(H, D, device="cuda")
        wt = w.t().contiguous()
        b = torch.randn(H, device="cuda")
        g = torch.randn(B, H, device="cuda")
        r = {
            "fwd_addmm_relu": timed(lambda: torch._addmm_activation(b, x, w.t())),
            "fwd_addmm": timed(lambda: torch.addmm(b, x, w.t())),
            "fwd_addmm_wt": timed(lambda: torch.addmm(b, x, wt)),
            "fwd_linear": timed(lambda: torch.nn.functional.linear(x, w, b)),
            "fwd_mm_T": timed(lambda: torch.mm(w, x.t())),
            "wgrad_gT_x": timed(lambda: g.t() @ x),
            "wgrad_xT_g": timed(lambda: x.t() @ g),
            "wgrad_bmm_s4": timed(lambda: torch.bmm(g.view(4, -1, H).transpose(1, 2), x.view(4, -1, D)).sum(0)),
            "dgrad_g_w": timed(lambda: g @ w),
            "empty_event": timed(lambda: None),
        }
        out[f"{B}x{D}->{H}"] = r
        print(json.dumps({f"{B}x{D}->{H}": r}), flush=True)


if __name__ == "__main__":
    main()
