"""Where PGS launch time goes: kernel time vs the sweep cap, and the per-env sweep x row work of the
last substep (aux row) -- max vs mean (the launch waits for its slowest env pair)."""
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


def run(xml, prec, n=4096, steps=30):
    env = HumanoidVecEnv({"model_path": xml, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3},
                         n_envs=n, model=HsModel(xml), seed=0, precision=prec)
    env.reset_tensors()
    g = torch.Generator(device="cuda").manual_seed(0)
    tape = torch.rand(256, n, 21, device="cuda", generator=g) * 2 - 1
    env.batch.set_state(time=np.floor(np.arange(n) * 667 / n) * 0.015 + 0.005)
    for k in range(300):
        env.step_tensors(tape[k % 256])
    ms, work = [], []
    for k in range(steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        env.step_tensors(tape[k % 256])
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
        a = env.batch.aux.double().cpu().numpy()
        w = a[:, 37] * np.maximum(a[:, 36], 1)
        work.append((w.max(), w.mean(), a[:, 37].max(), a[:, 36].max(), (a[:, 37] >= 100).sum()))
    warn = env.batch.warning.sum(0).tolist()
    print(f"    schedule: {'chunk queue' if env.batch.queued() else 'one wave per pair'} (resident waves "
          f"{env.batch.resident_waves}); warnings over {300 + steps} staggered steps [badqpos, badqvel, badqacc "
          f"(mj_checkAcc resets), overflow] = {warn}", flush=True)
    env.close()
    ms = np.array(ms)
    work = np.array(work)
    c = np.corrcoef(ms, work[:, 0])[0, 1]
    return ms.mean(), work.mean(0), c


def main():
    src = open(XML).read()
    d = tempfile.mkdtemp()
    for prec in ("fp64", "fp32"):
        for it in ((100,) if "defaults" in sys.argv else (100, 50, 25)):
            xml = os.path.join(d, f"pgs{it}.xml")
            open(xml, "w").write(re.sub(r"<option[^>]*/>", f'<option timestep="0.005" solver="PGS" iterations="{it}"/>',
                                        src, count=1))
            ms, w, c = run(xml, prec)
            print(f"[{prec}] PGS iterations={it:3d}: {ms:.3f} ms/step ({4096 / ms / 1e3:.2f} M/s); last substep "
                  f"sweeps x rows max {w[0]:.0f} mean {w[1]:.0f}; max sweeps {w[2]:.0f} max rows {w[3]:.0f}; "
                  f"envs at the cap {w[4]:.1f}; corr(ms, max work) {c:.2f}", flush=True)


if __name__ == "__main__":
    main()
