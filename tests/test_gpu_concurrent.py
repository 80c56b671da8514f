"""Two processes, each stepping its own queued 4096-env fp64 batch, on ONE GPU at the same time (the
round-4 verdict's case: "a user who runs two 4096-env fp64 trainers on one GPU").  Each launch's
persistent chunk-queue grid is sized for the whole GPU, so the two kernels' waves are not all
co-resident; the schedule must still hand every pair over (a wave only waits for a first chunk that
a running wave has claimed).  Both processes must end with no lost hand-off and
states bitwise equal to the same batch stepped alone."""
import multiprocessing as mp

import numpy as np
import pytest

from conftest import XML

pytestmark = pytest.mark.gpu

N, STEPS = 4096, 200


def _run(seed, q, barrier=None):
    """Step a seeded queued batch STEPS times with a seeded action tape (after the barrier, so that
    concurrent runs overlap); report (qpos, qvel, warnings)."""
    try:
        import torch
        from mujocoposelearning_amd.batch import HsBatch
        from mujocoposelearning_amd.model import HsModel
        b = HsBatch(HsModel(XML), N, precision="fp64", seed=seed)
        b.configure(frame_skip=3, duration=10.0, reward_id=0, autoreset=1, max_steps=750)
        assert b.queued()
        b.reset()
        g = torch.Generator(device="cuda").manual_seed(seed)
        acts = torch.rand(STEPS, N, 21, device="cuda", generator=g) * 2 - 1
        torch.cuda.synchronize()
        if barrier is not None:
            barrier.wait(timeout=240)
        for k in range(STEPS):
            b.step(acts[k])
        torch.cuda.synchronize()
        q.put((seed, b.qpos.cpu().numpy(), b.qvel.cpu().numpy(), b.warning.sum(0).cpu().numpy()))
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        q.put((seed, repr(e), None, None))


def test_two_processes_step_queued_batches_on_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    bar = ctx.Barrier(2)
    procs = [ctx.Process(target=_run, args=(s, q, bar)) for s in (1, 2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        seed, qp, qv, w = q.get(timeout=240)
        assert not isinstance(qp, str), qp
        got[seed] = (qp, qv, w)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # each batch alone: one process at a time
    for seed in (1, 2):
        q2 = ctx.Queue()
        p = ctx.Process(target=_run, args=(seed, q2))
        p.start()
        s, qp, qv, w = q2.get(timeout=240)
        p.join(timeout=60)
        assert not isinstance(qp, str), qp
        cq, cv, cw = got[seed]
        assert cw[4] == 0 and w[4] == 0, (cw, w)        # HS_WARN_HANDOFF: no lost hand-off
        assert np.array_equal(cq, qp) and np.array_equal(cv, qv), seed
