"""Quick GPU probe: env-step throughput at N envs and trajectory divergence vs the oracle."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mujocoposelearning_amd.batch import HsBatch  # noqa: E402
from mujocoposelearning_amd.model import HsModel  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")


def throughput(n, steps=50, prec="fp32"):
    model = HsModel(XML)
    b = HsBatch(model, n, precision=prec, seed=1)
    b.configure(frame_skip=3, duration=10.0, reward_id=0)
    b.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = torch.rand(steps + 5, n, model.nu, device="cuda", generator=g) * 2 - 1
    for k in range(5):
        b.step(acts[k])
    torch.cuda.synchronize()
    t = time.perf_counter()
    for k in range(steps):
        b.step(acts[5 + k])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"[{prec}] N={n}: {dt / steps * 1e3:.3f} ms/step  -> {n * steps / dt:,.0f} env-steps/s ; "
          f"mean ncon {b.aux[:, 35].float().mean().item():.1f} nefc {b.aux[:, 36].float().mean().item():.1f} "
          f"newton {b.aux[:, 37].float().mean().item():.2f}  warnings {b.warning.sum(0).tolist()}")


def divergence(prec, tape, nsub=1000, seed=0):
    model = HsModel(XML)
    o = Oracle(XML)
    rng = np.random.default_rng(seed)
    qpos = o.M["qpos0"].copy()
    qpos += rng.uniform(-0.01, 0.01, 28) * np.r_[1, 1, 0.1, 0, 0, 0, 0, np.ones(21)]
    qvel = rng.uniform(-0.01, 0.01, 27)
    b = HsBatch(model, 1, precision=prec)
    b.set_state(qpos=qpos, qvel=qvel, time=0.0, qacc_warmstart=0.0)
    o.qpos[:] = qpos
    o.qvel[:] = qvel
    if tape == "zeros":
        ctrl = np.zeros((nsub, 21), np.float32)
    else:
        ctrl = rng.uniform(-1, 1, (nsub, 21)).astype(np.float32)
    errs = []
    c = torch.tensor(ctrl, device="cuda")
    for s in range(nsub):
        b.physics_step(c[s:s + 1], 1)
        o.step(ctrl[s].astype(np.float64), 1)
        if s % 50 == 49 or s == nsub - 1:
            st = b.get_state()
            errs.append((s + 1, np.abs(st["qpos"][0] - o.qpos).max(), np.abs(st["qvel"][0] - o.qvel).max(), o.d.ncon))
    print(f"[{prec} tape={tape}] " + " ".join(f"{s}:{eq:.1e}/{ev:.1e}/c{nc}" for s, eq, ev, nc in errs))


def streams(n=4096, steps=100):
    """Same 4096 envs split into S independent groups, each stepped on its own HIP stream: one
    group's Newton-iteration tail overlaps the other groups' next launches."""
    model = HsModel(XML)
    for S in (1, 2, 4, 8):
        m = n // S
        bs = []
        for gi in range(S):
            b = HsBatch(model, m, precision="fp32", seed=1 + gi)
            b.configure(frame_skip=3, duration=10.0, reward_id=0)
            b.reset()
            bs.append(b)
        g = torch.Generator(device="cuda").manual_seed(0)
        tape = torch.rand(steps + 5, n, model.nu, device="cuda", generator=g) * 2 - 1
        torch.cuda.synchronize()
        sts = [torch.cuda.Stream() for _ in range(S)]

        def run(k0, k1):
            for k in range(k0, k1):
                for gi, (b, st) in enumerate(zip(bs, sts)):
                    with torch.cuda.stream(st):
                        b.step(tape[k, gi * m:(gi + 1) * m])
        run(0, 5)
        torch.cuda.synchronize()
        t = time.perf_counter()
        run(5, 5 + steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print(f"[fp32] N={n} as {S} groups x {m} on {S} streams: {dt / steps * 1e3:.3f} ms/step -> "
              f"{n * steps / dt:,.0f} env-steps/s")


def groups_api(n=4096, steps=100):
    """HsBatch(groups=G).step(join=False) vs separate batches stepped inside torch.cuda.stream()."""
    model = HsModel(XML)
    g = torch.Generator(device="cuda").manual_seed(0)
    tape = torch.rand(steps + 5, n, model.nu, device="cuda", generator=g) * 2 - 1
    for G in (1, 2, 4):
        b = HsBatch(model, n, precision="fp32", seed=1, groups=G)
        b.configure(frame_skip=3, duration=10.0, reward_id=0)
        b.reset()
        for k in range(5):
            b.step(tape[k], join=False)
        b.join()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(steps):
            b.step(tape[5 + k], join=False)
        b.join()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print(f"HsBatch(groups={G}) join=False: {dt / steps * 1e3:.3f} ms/step -> {n * steps / dt:,.0f} env-steps/s")


def tail(n=4096, steps=300, prec="fp32"):
    """Distribution of per-env Newton iterations / contacts over an episode, and the launch-time
    sensitivity to the Newton iteration cap (the launch ends with its slowest wave)."""
    model = HsModel(XML)
    for cap in (100, 30, 15):
        b = HsBatch(model, n, precision=prec, seed=1)
        b.configure(frame_skip=3, duration=10.0, reward_id=0, max_newton=cap)
        b.reset()
        g = torch.Generator(device="cuda").manual_seed(0)
        acts = torch.rand(steps, n, model.nu, device="cuda", generator=g) * 2 - 1
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ms = []
        rows = []
        for k in range(steps):
            e0.record()
            b.step(acts[k])
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
            if cap == 100 and k in (5, 30, 60, 100, 200, 299):
                it = b.aux[:, 37].float()
                nc = b.aux[:, 35].float()
                ne = b.aux[:, 36].float()
                q = torch.tensor([0.5, 0.9, 0.99, 1.0], device=it.device)
                rows.append(f"  step {k:3d}: newton p50/p90/p99/max {torch.quantile(it, q).tolist()}  "
                            f"ncon mean/max {nc.mean().item():.1f}/{nc.max().item():.0f}  "
                            f"nefc mean/max {ne.mean().item():.1f}/{ne.max().item():.0f}")
        ms = np.array(ms)
        print(f"[{prec}] N={n} max_newton={cap}: ms/step mean {ms.mean():.3f} (steps 0-99 {ms[:100].mean():.3f}, "
              f"100-299 {ms[100:].mean():.3f})  warnings {b.warning.sum(0).tolist()}")
        for r in rows:
            print(r)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "streams":
        streams()
        groups_api()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "tail":
        tail()
        sys.exit(0)
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("all", "tp"):
        for n in (1024, 4096, 16384):
            throughput(n)
        throughput(4096, prec="fp64")
    if which in ("all", "div"):
        divergence("fp64", "uniform")
        divergence("fp64", "zeros")
        divergence("fp32", "uniform")
        divergence("fp32", "zeros")
