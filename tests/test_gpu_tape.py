"""Tape launches (hs_step_tape / HsBatch.step_tape): K consecutive env steps over a given action
tape in ONE launch of the chunk-queue kernel, whole env steps as items, each env pair's step t + 1
waiting only for its own step t (hs_kernels.hip step_kernel_queue).

The contract is bitwise equality with K ``step`` calls (custom_env.py:152-230 per step): states,
every step's obs / reward / terminated / truncated, auto-resets inside the tape with their
terminal obs and final-step info, warnings -- on the fp64 engine at configs[1] size (4096 envs,
more pairs than resident waves) and at a small odd count, on the fp32 engine, with full-state obs,
and through the overflow path (an env over the resident contact tier stops the launch and the tape
is replayed step by step, where the wide tier re-runs it).
"""
import numpy as np
import pytest

from conftest import XML

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model():
    from mujocoposelearning_amd.model import HsModel
    return HsModel(XML)


def _run(model, n, prec, acts, t0, tape, full_state=False, reward_id=0, lying=None, outputs=True, pre_step=True,
         duration=10.0, max_steps=750):
    import torch
    from mujocoposelearning_amd.batch import HsBatch
    b = HsBatch(model, n, precision=prec, seed=3, full_state=full_state)
    b.configure(frame_skip=3, duration=duration, reward_id=reward_id, autoreset=1, max_steps=max_steps)
    b.reset()
    b.set_state(time=t0)
    if lying is not None:
        idx, q = lying
        st = b.get_state()
        st["qpos"][idx] = q
        st["qvel"][idx] = 0.0
        st["qacc_warmstart"][idx] = 0.0
        b.set_state(**st)
    if pre_step:
        b.step(acts[0])                 # one ordinary step first (the queue's cost order is then set)
    K = acts.shape[0] - 2
    if tape:
        res = b.step_tape(acts[1:1 + K], outputs=outputs)
        if outputs:
            per = [x.clone() for x in res]
        else:
            per = None
    else:
        o, r, te, tr = [], [], [], []
        for k in range(K):
            b.step(acts[1 + k])
            o.append(b.obs.clone()); r.append(b.reward.clone()); te.append(b.terminated.clone())
            tr.append(b.truncated.clone())
        per = [torch.stack(o), torch.stack(r), torch.stack(te), torch.stack(tr)]
    fin = [b.qpos.clone(), b.qvel.clone(), b.qacc_warmstart.clone(), b.time.clone(), b.warning.clone(),
           b.step_count.clone(), b.episode.clone(), b.total_reward.clone(), b.obs.clone(), b.reward.clone(),
           b.terminated.clone(), b.truncated.clone(), b.terminal_obs.clone(), b.terminal_step_count.clone(),
           b.terminal_total_reward.clone()]
    if full_state:
        fin += [b.cfrc_ext.clone(), b.subtree_linvel.clone()]
    b.step(acts[-1])                    # an ordinary step after the tape: flags / epoch / order stay sound
    after = [b.qpos.clone(), b.obs.clone(), b.reward.clone()]
    info = dict(aborts=b.tape_aborts(), reruns=b.wide_reruns(), queued=b.queued())
    b.close()
    return per, fin, after, info


def _same(name, xs, ys):
    import torch
    for k, (x, y) in enumerate(zip(xs, ys)):
        if not torch.equal(x, y):
            d = (x.double() - y.double()).abs()
            raise AssertionError(f"{name}[{k}]: max |diff| {float(d.max()):.3e}, "
                                 f"{int((d.reshape(d.shape[0], -1).amax(1) > 0).sum())} rows differ")


CASES = [("fp64", 4096, False, 0), ("fp64", 777, False, 0), ("fp32", 4096, False, 0), ("fp64", 1024, True, 1)]


@pytest.mark.parametrize("prec,n,full,reward", CASES, ids=[f"{p}-{n}{'-full' if f else ''}" for p, n, f, _ in CASES])
def test_step_tape_bitwise_equals_step_loop(model, prec, n, full, reward):
    import torch
    K = 40
    g = torch.Generator(device="cuda").manual_seed(21)
    acts = torch.rand(K + 2, n, 21, device="cuda", generator=g) * 2 - 1
    t0 = np.floor(np.arange(n) * 667 / n) * 0.015 + 0.005      # staggered clocks: resets inside the tape
    per_a, fin_a, aft_a, info_a = _run(model, n, prec, acts, t0, True, full, reward)
    per_b, fin_b, aft_b, info_b = _run(model, n, prec, acts, t0, False, full, reward)
    assert info_a["aborts"] == 0 and info_a["reruns"] == info_b["reruns"]
    assert int(torch.stack([x for x in per_b[2]]).sum()) > 0     # episodes ended inside the tape
    _same("per-step", per_a, per_b)
    _same("final", fin_a, fin_b)
    _same("after", aft_a, aft_b)


@pytest.mark.parametrize("duration,max_steps", [(0.5, 750), (10.0, 20)], ids=["short-episodes", "truncation"])
def test_step_tape_longer_than_an_episode_is_split(model, duration, max_steps):
    """A tape longer than the shortest episode runs as several launches (the host splits it at
    hs_rollout_max_steps, so each env finishes at most one episode per launch): 0.5 s episodes
    (33 env steps, termination at duration) and max_steps 20 (TimeLimit truncation), 80 steps each,
    every env resetting two to four times inside the tape -- bitwise the step loop."""
    import torch
    n, K = 1024, 80
    g = torch.Generator(device="cuda").manual_seed(12)
    acts = torch.rand(K + 2, n, 21, device="cuda", generator=g) * 2 - 1
    L = min(max_steps, round(duration / 0.015))
    t0 = np.floor(np.arange(n) * L / n) * 0.015 + 0.005 if max_steps >= 750 else np.zeros(n) + 0.005
    kw = dict(duration=duration, max_steps=max_steps)
    per_a, fin_a, aft_a, info_a = _run(model, n, "fp64", acts, t0, True, **kw)
    per_b, fin_b, aft_b, info_b = _run(model, n, "fp64", acts, t0, False, **kw)
    assert info_a["aborts"] == 0
    ends = per_b[2].int() + per_b[3].int()
    assert int(ends.sum(0).min()) >= 2                               # every env reset at least twice
    if max_steps < 750:
        assert int(per_b[3].sum()) > 0                               # TimeLimit truncations inside the tape
    _same("per-step", per_a, per_b)
    _same("final", fin_a, fin_b)
    _same("after", aft_a, aft_b)


def test_step_tape_without_outputs_matches(model):
    import torch
    n, K = 4096, 12
    g = torch.Generator(device="cuda").manual_seed(4)
    acts = torch.rand(K + 2, n, 21, device="cuda", generator=g) * 2 - 1
    t0 = np.floor(np.arange(n) * 667 / n) * 0.015 + 0.005
    _, fin_a, aft_a, _ = _run(model, n, "fp64", acts, t0, True, outputs=False)
    _, fin_b, aft_b, _ = _run(model, n, "fp64", acts, t0, False)
    _same("final", fin_a, fin_b)
    _same("after", aft_a, aft_b)


def test_step_tape_overflow_replays_step_by_step(model):
    """16 envs lying pressed into the floor (over the resident tier's contacts / rows): the tape
    launch stops at the first overflow, the tape is replayed step by step from the saved state (the
    wide tier re-runs the overflowing steps), and the results are bitwise the step loop's."""
    import torch
    from oracle.oracle import Oracle
    from test_gpu_contacts import lying_states
    n, K = 4096, 6
    o = Oracle(XML)
    q = np.stack(lying_states(o, 16, seed=11))
    idx = np.arange(16) * 255 + 7
    g = torch.Generator(device="cuda").manual_seed(9)
    acts = torch.rand(K + 2, n, 21, device="cuda", generator=g) * 2 - 1
    t0 = np.zeros(n) + 0.005
    # lying when the tape starts: its first step overflows
    per_a, fin_a, aft_a, info_a = _run(model, n, "fp64", acts, t0, True, lying=(idx, q), pre_step=False)
    per_b, fin_b, aft_b, info_b = _run(model, n, "fp64", acts, t0, False, lying=(idx, q), pre_step=False)
    assert info_a["aborts"] == 1, info_a
    assert info_a["reruns"] == info_b["reruns"] >= len(idx), (info_a, info_b)
    _same("per-step", per_a, per_b)
    _same("final", fin_a, fin_b)
    _same("after", aft_a, aft_b)


def test_step_tape_pgs_instance_bitwise_equals_step_loop(tmp_path):
    """The <option solver="PGS"> kernel instance takes the same tape path (its own queue kernel):
    bitwise the step loop at 4096 fp64 envs (more pairs than the PGS instance's resident waves)."""
    import torch
    from mujocoposelearning_amd.batch import HsBatch
    from mujocoposelearning_amd.model import HsModel
    from test_gpu_pgs import _pgs_xml
    model = HsModel(_pgs_xml(tmp_path, 100, 1e-8))
    n, K = 4096, 8
    g = torch.Generator(device="cuda").manual_seed(31)
    acts = torch.rand(K, n, 21, device="cuda", generator=g) * 2 - 1
    t0 = np.floor(np.arange(n) * 667 / n) * 0.015 + 0.005
    outs = []
    for tape in (True, False):
        b = HsBatch(model, n, precision="fp64", seed=3)
        b.configure(frame_skip=3, duration=10.0, reward_id=0, autoreset=1, max_steps=750)
        b.reset()
        b.set_state(time=t0)
        if tape:
            obs = b.step_tape(acts)[0].clone()
        else:
            o = []
            for k in range(K):
                b.step(acts[k])
                o.append(b.obs.clone())
            obs = torch.stack(o)
        outs.append([obs, b.qpos.clone(), b.qvel.clone(), b.qacc_warmstart.clone(), b.warning.clone()])
        if tape:
            assert b.tape_aborts() == 0
        b.close()
    _same("pgs", outs[0], outs[1])


def test_step_tape_overflow_on_the_last_step_replays(model, tmp_path):
    """An env whose contacts overflow the resident tier only on the tape's LAST step (which hands
    nothing over) must still stop the launch: the tape is replayed step by step and the results are
    bitwise the step loop's.  Two lying humanoids under 100 g (a <option gravity> variant) land flat:
    their contacts stay inside the tier for two env steps and pass it in the third (found with the
    oracle; the step loop's wide-tier counter confirms it on the GPU)."""
    import re
    import torch
    from mujocoposelearning_amd.batch import HsBatch
    from mujocoposelearning_amd.model import HsModel
    from oracle.oracle import Oracle
    from test_gpu_contacts import lying_states
    src = re.sub(r"<option[^>]*/>", '<option timestep="0.005" gravity="0 0 -1000"/>', open(XML).read(), count=1)
    p = tmp_path / "heavy.xml"
    p.write_text(src)
    heavy, o = HsModel(str(p)), Oracle(str(p))
    qs = lying_states(Oracle(XML), 20, seed=11)
    q = []
    for i in (17, 18):            # lowest geom brought to the floor, then 2 mm up
        lo, hi = qs[i][2], qs[i][2] + 0.5
        for _ in range(30):
            z = 0.5 * (lo + hi)
            o.reset_data()
            o.qpos[:] = np.r_[qs[i][:2], z, qs[i][3:]]
            o.forward()
            lo, hi = (lo, z) if o.d.ncon == 0 else (z, hi)
        q.append(np.r_[qs[i][:2], hi + 0.002, qs[i][3:]])
    n, K = 2, 3
    acts = torch.zeros(K + 1, n, 21, device="cuda")
    outs, info = [], []
    for tape in (True, False):
        b = HsBatch(heavy, n, precision="fp64", seed=3)
        b.configure(frame_skip=3, duration=10.0, reward_id=0, autoreset=1, max_steps=750)
        b.reset()
        b.set_state(qpos=np.stack(q), qvel=0.0, qacc_warmstart=0.0, time=0.005)
        if tape:
            per = [x.clone() for x in b.step_tape(acts[:K])]
        else:
            o_, r_, te_, tr_, reruns = [], [], [], [], []
            for k in range(K):
                b.step(acts[k])
                o_.append(b.obs.clone()); r_.append(b.reward.clone()); te_.append(b.terminated.clone())
                tr_.append(b.truncated.clone())
                reruns.append(b.wide_reruns())
            per = [torch.stack(o_), torch.stack(r_), torch.stack(te_), torch.stack(tr_)]
            assert reruns[K - 2] == 0 and reruns[K - 1] >= 1, reruns     # overflow on the last step only
        fin = [b.qpos.clone(), b.qvel.clone(), b.qacc_warmstart.clone(), b.time.clone(), b.warning.clone(),
               b.step_count.clone(), b.total_reward.clone()]
        b.step(acts[K])
        outs.append((per, fin, [b.qpos.clone(), b.obs.clone()]))
        info.append(b.tape_aborts())
        b.close()
    assert info[0] == 1, info
    _same("per-step", outs[0][0], outs[1][0])
    _same("final", outs[0][1], outs[1][1])
    _same("after", outs[0][2], outs[1][2])


def test_step_tape_longer_than_511_steps(model):
    """A tape longer than QTAG_STEPS (511, the most steps one launch's hand-off tags can name) runs as
    several launches (hs_step_tape splits it), bitwise the step loop: 600 steps of 64 envs with
    episodes of 10 s (667 steps), so the 511-step limit is the one that splits it."""
    import torch
    n, K = 64, 600
    g = torch.Generator(device="cuda").manual_seed(5)
    acts = torch.rand(K + 2, n, 21, device="cuda", generator=g) * 2 - 1
    t0 = np.zeros(n) + 0.005
    _, fin_a, aft_a, info_a = _run(model, n, "fp64", acts, t0, True, outputs=False)
    _, fin_b, aft_b, _ = _run(model, n, "fp64", acts, t0, False)
    assert info_a["aborts"] == 0
    _same("final", fin_a, fin_b)
    _same("after", aft_a, aft_b)


def test_last_tape_ms_times_the_tape_launch(model):
    """hs_last_tape_ms (the bench's train-leg roofline reads it for hs_rollout): -1 before any tape
    launch, then the last tape kernel's duration from HIP events on its stream -- positive, and no
    longer than the host-timed call around it."""
    import time

    import torch
    from mujocoposelearning_amd.batch import HsBatch
    b = HsBatch(model, 256, precision="fp64", seed=2)
    b.configure(frame_skip=3, duration=10.0, reward_id=0, autoreset=1)
    b.reset()
    assert b.last_tape_ms() == -1.0
    acts = torch.zeros(8, 256, 21, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    b.step_tape(acts, outputs=False)
    host_ms = (time.perf_counter() - t0) * 1e3
    ms = b.last_tape_ms()
    assert 0.0 < ms <= host_ms, (ms, host_ms)
    b.close()
