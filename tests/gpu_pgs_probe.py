"""Throughput of the <option solver="PGS"> kernel instance vs the default Newton instance
(4096 envs, fp32, stand, frame_skip 3, U(-1,1) tape).  python tests/gpu_pgs_probe.py"""
import os
import re
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mujocoposelearning_amd.model import HsModel  # noqa: E402
from mujocoposelearning_amd.vec_env import HumanoidVecEnv  # noqa: E402

XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")


def rate(xml, n=4096, steps=40):
    env = HumanoidVecEnv({"model_path": xml, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3},
                         n_envs=n, model=HsModel(xml), seed=0)
    env.reset_tensors()
    g = torch.Generator(device="cuda").manual_seed(0)
    tape = torch.rand(steps + 10, n, 21, device="cuda", generator=g) * 2 - 1
    for k in range(10):
        env.step_tensors(tape[k])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(steps):
        env.step_tensors(tape[10 + k])
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    it = float(env.batch.aux[:, 37].float().mean())
    w = env.batch.warning.sum(0).tolist()
    env.close()
    return n / ms * 1e3, ms, it, w


def main():
    src = open(XML).read()
    d = tempfile.mkdtemp()
    for name, opt in (("Newton", None), ("PGS 100/1e-8", '<option timestep="0.005" solver="PGS"/>')):
        xml = XML
        if opt:
            xml = os.path.join(d, "pgs.xml")
            open(xml, "w").write(re.sub(r"<option[^>]*/>", opt, src, count=1))
        r, ms, it, w = rate(xml)
        print(f"{name:14s} {r / 1e6:6.2f} M env steps/s  {ms:.3f} ms/step  mean iterations/substep {it:.1f}  "
              f"warnings {w}", flush=True)


if __name__ == "__main__":
    main()
