"""Failures surface on the SB3 drop-in path (train_sb3.py:203 -> HumanoidVecEnv, custom_env.py:160):
the warning counters (include/hsim.h HS_WARN_*) travel in step_wait's single packed copy, a bad-state
reset warns as MuJoCo's mj_step does (mju_warning + mj_resetData, the run goes on), and a lost
chunk-queue hand-off raises HsimError -- with only step_async / step_wait in the loop, as SB3's own
PPO drives a VecEnv."""
import warnings

import numpy as np
import pytest

from conftest import XML

pytestmark = pytest.mark.gpu


def _cfg():
    return {"model_path": XML, "duration": 10.0, "frame_skip": 3, "reward_config": {"type": "stand"}}


def test_step_wait_raises_on_a_lost_handoff_and_warns_on_bad_states():
    from mujocoposelearning_amd._lib import HsimError
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv(_cfg(), n_envs=4096, model=HsModel(XML), seed=0, precision="fp64")
    assert env.batch.queued()
    env.reset()
    rng = np.random.default_rng(0)
    act = lambda: rng.uniform(-1, 1, (4096, 21)).astype(np.float32)  # noqa: E731
    with warnings.catch_warnings():
        warnings.simplefilter("error")                     # a clean run warns about nothing
        for _ in range(3):
            env.step_async(act())
            env.step_wait()
    env.batch.qpos[5, 2] = float("nan")                    # mj_checkPos resets it in the next substep
    with pytest.warns(RuntimeWarning, match="QPOS in 1 env step"):
        env.step_async(act())
        env.step_wait()
    env.batch.debug_lose_handoff(1234)
    env.step_async(act())
    with pytest.raises(HsimError, match="hand-off lost"):
        env.step_wait()
    env.batch.debug_lose_handoff(None)
    with warnings.catch_warnings():
        warnings.simplefilter("error")                     # reported once, not again
        env.step_async(act())
        obs, rew, dones, infos = env.step_wait()
    assert np.isfinite(obs).all()
    assert env.warning_counts()[4] == 2                    # both envs of the pair (1234, 1235)
    env.close()


def test_gym_step_warns_on_a_bad_state_reset():
    from mujocoposelearning_amd.env import HumanoidEnv
    env = HumanoidEnv(_cfg())
    env.reset(seed=0)
    a = np.zeros(21, np.float32)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        env.step(a)
    env._batch.qvel[0, 7] = float("inf")
    with pytest.warns(RuntimeWarning, match="QVEL"):
        state, reward, terminated, truncated, info = env.step(a)
    assert np.isfinite(state).all()
