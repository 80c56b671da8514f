"""HumanoidVecEnv.step_wait's infos (vec_env.StepInfos, built by the native csrc/hs_infos.c) against
the eager per-env Python construction SubprocVecEnv's info dicts follow (custom_env.py:216-230 keys,
SB3's terminal_observation / TimeLimit.truncated for finished envs; train_sb3.py:203).  CPU only: the
builder is host code."""
import time

import numpy as np


def _eager(obs, term, trunc, step_count, total, term_obs_full):
    dones = term | trunc
    out = []
    for i in range(len(term)):
        info = {"reward_components": {}, "height": None, "step_count": int(step_count[i]),   # custom_env.py:216-224 order
                "truncated": bool(trunc[i]), "truncation_info": {"reason": "timeout"} if trunc[i] else {},
                "terminated": bool(term[i]), "total_reward": float(total[i])}
        if dones[i]:
            info["terminal_observation"] = term_obs_full[i]
            info["TimeLimit.truncated"] = bool(trunc[i] and not term[i])
            info["height"] = float(term_obs_full[i][0])
        else:
            info["height"] = float(obs[i][0])
        out.append(info)
    return out


def _case(n, seed):
    rng = np.random.default_rng(seed)
    obs = rng.normal(size=(n, 352))
    term = rng.random(n) < 0.05
    trunc = (rng.random(n) < 0.05) & ~term
    trunc[:3] = True                       # truncated, and one env both terminated and truncated
    term[2 % n] = True
    sc = rng.integers(0, 751, n).astype(np.float64)
    tot = rng.normal(size=n)
    tobs_full = rng.normal(size=(n, 352))
    idx = np.flatnonzero(term | trunc)
    return obs, term, trunc, sc, tot, idx, tobs_full


import pytest


@pytest.mark.parametrize("builder", ["native", "python"])
def test_step_infos_equal_the_eager_dicts(builder, monkeypatch):
    """Both builders: the native one, and the Python fallback taken when the extension cannot be
    imported (not built, or built for another interpreter)."""
    import sys
    from mujocoposelearning_amd.vec_env import StepInfos
    if builder == "python":
        import mujocoposelearning_amd as pkg
        import mujocoposelearning_amd.vec_env as ve
        monkeypatch.setitem(sys.modules, "mujocoposelearning_amd._hsinfo", None)   # import -> ImportError
        monkeypatch.delattr(pkg, "_hsinfo", raising=False)
        calls = []
        real = ve._build_infos_py
        monkeypatch.setattr(ve, "_build_infos_py", lambda *a: calls.append(1) or real(*a))
    for n, seed in ((8, 0), (4096, 1), (1, 2)):
        obs, term, trunc, sc, tot, idx, tobs_full = _case(n, seed)
        infos = StepInfos(obs, term, trunc, sc, tot, idx, tobs_full[idx])
        ref = _eager(obs, term, trunc, sc, tot, tobs_full)
        assert len(infos) == n
        got = list(infos)
        for i in range(n):
            x, y = got[i], ref[i]
            assert list(x.keys()) == list(y.keys()), i
            for k in y:
                if k == "terminal_observation":
                    np.testing.assert_array_equal(x[k], y[k])
                else:
                    assert x[k] == y[k] and type(x[k]) is type(y[k]), (i, k, x[k], y[k])
        assert infos[-1] is got[-1] and infos[0:2] == got[0:2]
        infos[0]["episode"] = {"r": 1.0}               # annotations persist (SB3 VecMonitor)
        assert infos[0]["episode"] == {"r": 1.0}
        if n > 1:
            assert infos[0]["truncation_info"] is not infos[1]["truncation_info"]   # fresh dicts per env
    if builder == "python":
        assert len(calls) == 3


def test_step_infos_build_4096_in_about_a_millisecond():
    """The point of the native builder: all 4096 dicts well under the ~5 ms Python needs."""
    from mujocoposelearning_amd.vec_env import StepInfos
    obs, term, trunc, sc, tot, idx, tobs_full = _case(4096, 3)
    best = 1e9
    for _ in range(5):
        t0 = time.perf_counter()
        list(StepInfos(obs, term, trunc, sc, tot, idx, tobs_full[idx]))
        best = min(best, time.perf_counter() - t0)
    t0 = time.perf_counter()
    _eager(obs, term, trunc, sc, tot, tobs_full)
    eager = time.perf_counter() - t0
    assert best < 0.5 * eager, (best, eager)
