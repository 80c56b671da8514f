"""What the device reward costs inside the fp64 step launch: the same staggered 4096-env batch
stepped with reward_id stand (0) and none (-1), alternating, HIP-event time per launch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mujocoposelearning_amd.batch import HsBatch  # noqa: E402
from mujocoposelearning_amd.model import HsModel  # noqa: E402


def main(prec="fp64", n=4096):
    model = HsModel(os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml"))
    b = HsBatch(model, n, precision=prec, seed=1)
    b.configure(frame_skip=3, duration=10.0, reward_id=0, aux=False, ctrl=False)
    b.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    tape = torch.rand(64, n, 21, device="cuda", generator=g) * 2 - 1
    b.set_state(time=np.floor(np.arange(n) * 667 / n) * 0.015 + 0.005)
    for k in range(667):
        b.step(tape[k % 64])
    res = {0: [], -1: []}
    for rep in range(6):
        for rid in (0, -1):
            b.configure(reward_id=rid)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for k in range(20):
                b.step(tape[k % 64])
            e1.record()
            torch.cuda.synchronize()
            res[rid].append(e0.elapsed_time(e1) / 20)
    print(f"[{prec}] ms per launch: stand reward {np.median(res[0]):.4f}, no reward {np.median(res[-1]):.4f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "fp64")
