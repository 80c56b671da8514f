"""Hash of the state after K env steps of a fixed workload (A/B builds that must be bitwise equal:
run once per HSIM_LIB and compare the printed digests)."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mujocoposelearning_amd.batch import HsBatch  # noqa: E402
from mujocoposelearning_amd.model import HsModel  # noqa: E402


def main(n=4096, k=60, prec="fp64"):
    m = HsModel(os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml"))
    b = HsBatch(m, n, precision=prec, seed=7)
    b.configure(frame_skip=3, duration=10.0, reward_id=0, autoreset=1)
    b.reset()
    g = torch.Generator(device="cuda").manual_seed(3)
    for _ in range(k):
        b.step(torch.rand(n, 21, device="cuda", generator=g) * 2 - 1)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for key in ("qpos", "qvel", "qacc_warmstart", "obs", "reward"):
        h.update(b.t[key].cpu().numpy().tobytes())
    print(os.path.basename(os.environ.get("HSIM_LIB", "libhsim.so")), prec, n, k, h.hexdigest())


if __name__ == "__main__":
    main(prec=sys.argv[1] if len(sys.argv) > 1 else "fp64")
