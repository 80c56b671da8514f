"""hs_dgrad_mask against the module-by-module path it replaces, per call at the PPO update's shapes
(32768-row minibatch, hidden 256): the input gradient g @ w (library GEMM, or the broadcast product
for the value head) + hs_relu_grad_colsum (mask + first bias pass).  Median of 50 HIP-event-timed
calls each.
    python tools/probes/gpu_dgrad_mask.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mujocoposelearning_amd.ppo_ops import dgrad_mask, relu_grad_colsum  # noqa: E402


def timed(fn, n=50):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[n // 2]


def main():
    B = 32768
    for K in (256, 21, 1):
        g = torch.randn(B, K, device="cuda")
        w = torch.randn(K, 256, device="cuda") * 0.06
        x = torch.relu(torch.randn(B, 256, device="cuda"))
        fused = timed(lambda: dgrad_mask(g, w, x))
        mm = (lambda: g * w) if K == 1 else (lambda: g @ w)
        gemm = timed(mm)
        gx = mm()
        mask = timed(lambda: relu_grad_colsum(gx, x))
        print(json.dumps({"B": B, "K": K, "dgrad_mask_us": round(fused, 1), "mm_us": round(gemm, 1),
                          "relu_colsum_us": round(mask, 1), "unfused_us": round(gemm + mask, 1)}), flush=True)


if __name__ == "__main__":
    main()
