"""Per-phase cycle breakdown of the step kernel (diagnostic build libhsim_timing.so)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["HSIM_LIB"] = os.environ.get("HSIM_TIMING_LIB",
                                        os.path.join(ROOT, "mujocoposelearning_amd", "libhsim_timing.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mujocoposelearning_amd.batch import HsBatch  # noqa: E402
from mujocoposelearning_amd.model import HsModel  # noqa: E402

NAMES = ["load", "kinematics", "mass_matrix", "vel+rne", "collision", "rows+aref", "newton:init Jx",
         "newton:rowf+aggr", "newton:gradient", "newton:hess dense rows", "newton:solve", "newton:ls loop",
         "newton:final frc", "euler:integrate", "obs+writeback", "newton:chol", "newton:ls J s rows",
         "euler:solve", "newton:ls M s", "newton:ls map_vx", "euler:pre", "euler:chol", "pre-obs (loop top)",
         "obs write", "step_count/energy sum", "reward", "newton:factor update", "newton:hess contacts", "newton:hess M+tree rows"]
NS = len(NAMES)


def main(n=4096, steps=20, prec="fp32", staggered=False):
    model = HsModel(os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml"))
    b = HsBatch(model, n, precision=prec, seed=1)
    b.configure(frame_skip=3, duration=10.0, reward_id=0)
    b.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    if staggered:
        # bench.py's window: env i starts i/N into the episode, then one full (667-step) episode
        t0 = np.floor(np.arange(n) * 667 / n) * 0.015 + 0.005
        b.set_state(time=t0)
        for k in range(667):
            b.step(torch.rand(n, 21, device="cuda", generator=g) * 2 - 1)
    for k in range(5):
        b.step(torch.rand(n, 21, device="cuda", generator=g) * 2 - 1)
    b.set_debug(True)
    b.t["aux"].zero_()
    torch.cuda.synchronize()
    dbg0 = b.get_debug()[8000:8031].copy()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for k in range(steps):
        b.step(torch.rand(n, 21, device="cuda", generator=g) * 2 - 1)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / steps
    d = b.get_debug()[8000:8031] - dbg0
    tot = d[:NS].sum()
    per = d[:NS] / (n * steps * 3)
    print(f"[{prec}{' staggered' if staggered else ''}] N={n}: {ms:.3f} ms/launch; cycles per env-substep (wave lifetime) {tot / (n * steps * 3):,.0f}; "
          f"newton iters/env step {d[30] / (n * steps):.2f}")
    for name, c, f in zip(NAMES, per, d[:NS] / tot):
        print(f"  {name:20s} {c:10,.0f} cyc  {100 * f:5.1f}%")
    life = b.get_debug()[9000:9000 + (n + 1) // 2]        # last launch, one value per wave
    q = np.percentile(life, [0, 10, 50, 90, 99, 100])
    print("  wave lifetime (last launch, cycles) min/p10/p50/p90/p99/max: " + " / ".join(f"{v:,.0f}" for v in q)
          + f"   mean {life.mean():,.0f}  (launch = max; mean/max = {life.mean() / life.max():.2f})")
    dbg = b.get_debug()
    st = dbg[16384:16384 + len(life)].astype(np.int64)      # s_memrealtime (100 MHz) at wave start / end
    en = dbg[18432:18432 + len(life)].astype(np.int64)
    base = st.min()
    st, en = (st - base) % (1 << 24), (en - base) % (1 << 24)
    span = en.max()
    ghz = life.mean() / max(1.0, (en - st).mean() * 10.0)   # shader cycles per ns
    print(f"  realtime: launch span {span * 10 / 1e3:.1f} us, mean wave {((en - st).mean()) * 10 / 1e3:.1f} us "
          f"(shader clock {ghz:.2f} GHz); wave start p10/p50/p90/max (us) " +
          " / ".join(f"{v * 10 / 1e3:.1f}" for v in np.percentile(st, [10, 50, 90, 100])))
    print("  wave end (fraction of span) p10/p50/p90/p99: " +
          " / ".join(f"{v:.2f}" for v in np.percentile(en / span, [10, 50, 90, 99])))
    late = st > 0.05 * span
    print(f"  waves starting in the first 5% of the span: {(~late).sum()}, later: {late.sum()}")
    busy = np.zeros(200)
    for a_, e_ in zip(st, en):
        busy[int(a_ / span * 199):int(e_ / span * 199) + 1] += 1
    print("  resident waves over the launch (20 bins): " + " ".join(f"{v:.0f}" for v in busy.reshape(20, 10).mean(1)))
    q0 = dbg[20480:20480 + 8192].reshape(-1, 2).astype(np.int64)
    qw = dbg[28672:28672 + 4096]
    if q0.any():    # chunk-queue schedule: per item realtime start / end and flag-wait cycles
        qs, qe = (q0[:, 0] - q0[:, 0].min()) % (1 << 24), (q0[:, 1] - q0[:, 0].min()) % (1 << 24)
        span = qe.max()
        npair = len(life)
        d0, d1 = (qe - qs)[:npair], (qe - qs)[npair:2 * npair]
        print(f"  queue: span {span * 10 / 1e3:.1f} us; chunk0 items mean {d0.mean() * 10 / 1e3:.1f} us, last-substep items "
              f"mean {d1.mean() * 10 / 1e3:.1f} us (p90 {np.percentile(d1, 90) * 10 / 1e3:.1f}, max {d1.max() * 10 / 1e3:.1f})")
        busy = np.zeros(200)
        for a_, e_ in zip(qs, qe):
            busy[int(a_ / span * 199):int(e_ / span * 199) + 1] += 1
        print("  busy waves over the launch (20 bins): " + " ".join(f"{v:.0f}" for v in busy.reshape(20, 10).mean(1)))
    np.savez(os.path.join(ROOT, "gpurun_out", f"timing_{prec}_{n}.npz"), life=life, st=st, en=en,
             it=dbg[11100:11100 + 2 * len(life)], q0=q0, qw=qw)
    it = b.get_debug()[11100:11100 + 2 * len(life)].reshape(-1, 2)
    wmax, wsum = it.max(1), it.sum(1)
    print(f"  newton iters per env per launch: mean {it.mean():.1f} max {it.max():.0f}; corr(lifetime, max-of-pair) "
          f"{np.corrcoef(life, wmax)[0, 1]:.2f}, corr(lifetime, sum-of-pair) {np.corrcoef(life, wsum)[0, 1]:.2f}")
    for lo, hi in ((0, 8), (8, 12), (12, 16), (16, 24), (24, 1000)):
        sel = (wmax >= lo) & (wmax < hi)
        if sel.any():
            print(f"    pair-max iters [{lo},{hi}): {sel.sum():5d} waves, lifetime mean {life[sel].mean():,.0f} "
                  f"max {life[sel].max():,.0f}")


def predict(n=4096, steps=60, prec="fp32"):
    """Is per-env Newton work predictable from the previous env step?  (timing build: dbg[11100+env]
    = Newton iterations of env summed over the launch's substeps)"""
    model = HsModel(os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml"))
    b = HsBatch(model, n, precision=prec, seed=1)
    b.configure(frame_skip=3, duration=10.0, reward_id=0)
    b.reset()
    b.set_debug(True)
    g = torch.Generator(device="cuda").manual_seed(0)
    hist = []
    for k in range(steps):
        b.step(torch.rand(n, 21, device="cuda", generator=g) * 2 - 1)
        hist.append(b.get_debug()[11100:11100 + n].copy())
    h = np.array(hist[10:])
    c1 = np.mean([np.corrcoef(h[i], h[i + 1])[0, 1] for i in range(len(h) - 1)])
    c5 = np.mean([np.corrcoef(h[i], h[i + 5])[0, 1] for i in range(len(h) - 5)])
    # wave cost model: max over the env pair; compare random pairing vs pairing sorted by the
    # previous step's count (what a predictor-driven permutation would achieve)
    rnd, srt = [], []
    for i in range(len(h) - 1):
        cur, prev = h[i + 1], h[i]
        rnd.append(np.maximum(cur[0::2], cur[1::2]).sum())
        o = np.argsort(prev)
        srt.append(np.maximum(cur[o][0::2], cur[o][1::2]).sum())
    print(f"[{prec}] N={n}: corr(iters_t, iters_t+1) {c1:.2f}, corr(t, t+5) {c5:.2f}; "
          f"sum over waves of max(pair): random pairing {np.mean(rnd):,.0f} vs sorted by previous step "
          f"{np.mean(srt):,.0f} ({np.mean(srt) / np.mean(rnd):.3f}); ideal {h[1:].sum(1).mean() / 2:,.0f}")


def predict_queue(n=4096, prec="fp64", steps=6):
    """Chunk-queue schedule: is a pair's item cost predictable from the previous env step's?
    (timing build: per-item realtime start / end of the last launch, staggered mix)"""
    model = HsModel(os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml"))
    b = HsBatch(model, n, precision=prec, seed=1)
    b.configure(frame_skip=3, duration=10.0, reward_id=0)
    b.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    b.set_state(time=np.floor(np.arange(n) * 667 / n) * 0.015 + 0.005)
    for k in range(667):
        b.step(torch.rand(n, 21, device="cuda", generator=g) * 2 - 1)
    b.set_debug(True)
    np_ = (n + 1) // 2
    hist = []
    for k in range(steps):
        b.step(torch.rand(n, 21, device="cuda", generator=g) * 2 - 1)
        q0 = b.get_debug()[20480:20480 + 4 * np_].reshape(-1, 2).astype(np.int64)
        d = ((q0[:, 1] - q0[:, 0]) % (1 << 24)) * 10 / 1e3
        hist.append((d[:np_], d[np_:2 * np_]))
    c0 = np.mean([np.corrcoef(hist[i][0], hist[i + 1][0])[0, 1] for i in range(steps - 1)])
    c1 = np.mean([np.corrcoef(hist[i][1], hist[i + 1][1])[0, 1] for i in range(steps - 1)])
    ct = np.mean([np.corrcoef(hist[i][0] + hist[i][1], hist[i + 1][1])[0, 1] for i in range(steps - 1)])
    cw = np.mean([np.corrcoef(hist[i][0], hist[i][1])[0, 1] for i in range(steps)])
    print(f"[{prec}] per-pair item durations, consecutive steps: corr(chunk0) {c0:.2f}, corr(last) {c1:.2f}, "
          f"corr(prev total, last) {ct:.2f}; within a step corr(chunk0, last) {cw:.2f}")
    np.savez(os.path.join(ROOT, "gpurun_out", f"predict_queue_{prec}.npz"), d0=np.array([h[0] for h in hist]),
             d1=np.array([h[1] for h in hist]))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "predict_queue":
        predict_queue(prec=sys.argv[1])
        sys.exit(0)
    if len(sys.argv) > 2 and sys.argv[2] == "predict":
        predict(prec=sys.argv[1])
        sys.exit(0)
    kw = dict(a.split("=", 1) for a in sys.argv[2:] if "=" in a)
    main(n=int(kw.get("n", 4096)), prec=sys.argv[1] if len(sys.argv) > 1 else "fp32",
         staggered="staggered" in sys.argv[2:])
