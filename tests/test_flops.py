"""The algorithmic FLOP counter: oracle/flopcount.h turns the fp64
restatement into a per-stage counting build.  Checked here: it computes bitwise the same
trajectory as the plain oracle build (counting changes nothing), and profiles/flops_per_env_step.json
(what bench.py's VALU-FLOP fraction uses) is what oracle/flops.py computes."""
import json
import os

import numpy as np

from conftest import ROOT, XML


def test_counting_build_is_bitwise_the_oracle():
    from oracle import flops
    from oracle.oracle import Oracle
    a, b = Oracle(XML), Oracle(XML)
    b.lib = flops.load()
    rng = np.random.default_rng(3)
    for o in (a, b):
        o.reset_data()
        o.qpos[:] = a.M["qpos0"]
        o.qpos[2] = 1.25
    for _ in range(60):
        c = rng.uniform(-1, 1, 21)
        a.step(c, 3)
        b.step(c, 3)
    assert np.array_equal(a.qpos, b.qpos) and np.array_equal(a.qvel, b.qvel)
    cnt = flops.read(b.lib)
    assert cnt.sum() > 0 and cnt[len(flops.STAGES):].sum() == 0


def test_committed_flop_figure_reproduces():
    from oracle import flops
    ref = json.load(open(os.path.join(ROOT, "profiles", "flops_per_env_step.json")))
    got = flops.count(XML, "T1")
    assert got["total"] == ref["T1"]["total"]
    assert 1e5 < ref["mean_total"] < 1e6          # SURVEY 8d's O(3e5 - 6e5) per env step
    assert ref["T1"]["per_stage"]["solver"] > ref["T1"]["per_stage"]["kinematics"]
