"""Throughput of the <option solver="PGS"> kernel instance vs the default Newton instance: 4096 envs,
stand, frame_skip 3, U(-1,1) tape, bench.py's staggered-episode window (env i starts i/N into its
episode, one untimed full episode first, so the timed steps average standing, falling and lying
humanoids); warnings (bad qpos / qvel / qacc resets, contact overflow) are counted over the whole
run.  python tools/probes/gpu_pgs_probe.py [fp64|fp32 ...]"""
import os
import re
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mujocoposelearning_amd.model import HsModel  # noqa: E402
from mujocoposelearning_amd.vec_env import HumanoidVecEnv  # noqa: E402

XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")
EPISODE = 667


def rate(xml, prec, n=4096, steps=40):
    env = HumanoidVecEnv({"model_path": xml, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3},
                         n_envs=n, model=HsModel(xml), seed=0, precision=prec)
    env.reset_tensors()
    g = torch.Generator(device="cuda").manual_seed(0)
    tape = torch.rand(256, n, 21, device="cuda", generator=g) * 2 - 1
    env.batch.set_state(time=np.floor(np.arange(n) * EPISODE / n) * 0.015 + 0.005)
    for k in range(EPISODE):
        env.step_tensors(tape[k % 256])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(steps):
        env.step_tensors(tape[(EPISODE + k) % 256])
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    it = float(env.batch.aux[:, 37].float().mean())
    rows = float(env.batch.aux[:, 36].float().mean())
    w = env.batch.warning.sum(0).tolist()
    env.close()
    return n / ms * 1e3, ms, it, rows, w


def main(precs):
    src = open(XML).read()
    d = tempfile.mkdtemp()
    for prec in precs:
        for name, opt in (("Newton", None), ("PGS 100/1e-8", '<option timestep="0.005" solver="PGS"/>')):
            xml = XML
            if opt:
                xml = os.path.join(d, "pgs.xml")
                open(xml, "w").write(re.sub(r"<option[^>]*/>", opt, src, count=1))
            r, ms, it, rows, w = rate(xml, prec)
            print(f"[{prec}] {name:14s} {r / 1e6:6.2f} M env steps/s  {ms:.3f} ms/step  mean iterations/substep "
                  f"{it:.1f}  mean rows {rows:.1f}  warnings over {EPISODE + 40} steps x 4096 envs {w}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["fp64", "fp32"])
