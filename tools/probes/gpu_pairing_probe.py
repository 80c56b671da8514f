"""Is an env's step independent of its wave partner?  Runs the same staggered fp64 batch (777 envs,
stand) under the single-env schedule (twice), the paired schedule (twice) and the paired schedule with
the envs' order reversed (new partners), and reports, per comparison, the first step where any env's
(qpos, qvel) differs and the size of that first difference (round-off vs a discrete event).
python tools/probes/gpu_pairing_probe.py [n] [steps] [full_state 0/1] [reward_id]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mujocoposelearning_amd.batch import HsBatch  # noqa: E402
from mujocoposelearning_amd.model import HUMANOID_XML, HsModel  # noqa: E402


def run(model, n, acts, t0, sched, perm, full, rid):
    b = HsBatch(model, n, precision="fp64", seed=3, full_state=full)
    b.configure(frame_skip=3, duration=10.0, reward_id=rid, autoreset=1, max_steps=750, schedule=sched)
    b.reset()
    st = b.get_state()
    for k in st:
        st[k] = st[k][perm]
    b.set_state(**st)
    b.set_state(time=t0[perm])
    traj, aux = [], []
    for k in range(acts.shape[0]):
        b.step(acts[k][perm])
        inv = np.argsort(perm)
        traj.append(torch.cat([b.qpos, b.qvel], 1)[inv].clone())
        aux.append(b.aux[inv].clone())
    name = b.schedule_name()
    b.close()
    return torch.stack(traj), torch.stack(aux), name


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 777
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    full = bool(int(sys.argv[3])) if len(sys.argv) > 3 else False
    rid = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    model = HsModel(HUMANOID_XML)
    g = torch.Generator(device="cuda").manual_seed(21)
    acts = torch.rand(K, n, 21, device="cuda", generator=g) * 2 - 1
    t0 = np.floor(np.arange(n) * 667 / n) * 0.015 + 0.005
    ident, rev = np.arange(n), np.arange(n)[::-1].copy()
    runs = {}
    for key, sched, perm in [("single", "auto", ident), ("single2", "auto", ident), ("paired", "direct", ident),
                             ("paired2", "direct", ident), ("paired_rev", "direct", rev), ("single_rev", "auto", rev)]:
        runs[key] = run(model, n, acts, t0, sched, perm, full, rid)
        print(f"{key}: schedule {runs[key][2]}", flush=True)
    for a, b in [("single", "single2"), ("paired", "paired2"), ("single", "paired"), ("paired", "paired_rev"),
                 ("single", "single_rev"), ("single", "paired_rev")]:
        x, y = runs[a][0], runs[b][0]
        d = (x - y).abs().amax(2)            # [K, n]
        bad = torch.nonzero(d > 0)
        if bad.numel() == 0:
            print(f"{a} vs {b}: bitwise equal over {K} steps", flush=True)
            continue
        t = int(bad[0, 0])
        envs = torch.nonzero(d[t] > 0).flatten().tolist()
        ax, ay = runs[a][1][t, envs[0]], runs[b][1][t, envs[0]]
        print(f"{a} vs {b}: first diff at step {t}, envs {envs[:10]} (total {int((d.amax(0) > 0).sum())} envs by the end), "
              f"first |diff| {float(d[t].max()):.3e}; env {envs[0]} ncon/nefc/iters {ax[35:38].tolist()} vs {ay[35:38].tolist()}",
              flush=True)


if __name__ == "__main__":
    main()
