"""GPU side of the render path: hs_kinematics (the poses the renderer draws) against the fp64
oracle's mj_kinematics/mj_comPos, and HumanoidEnv(render_mode='rgb_array') frame capture and
save_video (custom_env.py:227-228, 273-321)."""
import os

import numpy as np
import pytest

from conftest import XML

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model():
    from mujocoposelearning_amd.model import HsModel
    return HsModel(XML)


def _oracle_states(n, seed=0):
    from oracle.oracle import Oracle
    o = Oracle(XML)
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        o.step(rng.uniform(-1, 1, 21), 7)
        out.append(o.qpos.copy())
    return o, out


@pytest.mark.parametrize("prec,tol", [("fp64", 1e-9), ("fp32", 2e-5)])
def test_kinematics_matches_oracle(model, prec, tol):
    from mujocoposelearning_amd.batch import HsBatch
    o, states = _oracle_states(12)
    n = len(states)
    b = HsBatch(model, n, precision=prec)
    b.set_state(qpos=np.array(states))
    for e, q in enumerate(states):
        k = b.kinematics(e)
        o.qpos[:] = q
        o.forward()
        gm = o.get("geom_xmat").reshape(-1, 3, 3)
        np.testing.assert_allclose(k["xpos"], o.get("xpos"), atol=tol)
        np.testing.assert_allclose(k["xmat"], o.get("xmat"), atol=tol)
        np.testing.assert_allclose(k["geom_xpos"], o.get("geom_xpos"), atol=tol)
        np.testing.assert_allclose(k["geom_zaxis"], gm[:, :, 2], atol=tol)
        np.testing.assert_allclose(k["com"], o.get("subtree_com")[0], atol=tol)
    # posing an explicit qpos does not touch the env's state
    k0 = b.kinematics(0, qpos=model.qpos0)
    o.qpos[:] = model.qpos0
    o.forward()
    np.testing.assert_allclose(k0["xpos"], o.get("xpos"), atol=tol)
    np.testing.assert_allclose(b.get_state()["qpos"][0], states[0], atol=tol)
    with pytest.raises(IndexError):
        b.kinematics(n)


def test_env_rgb_array_frames_and_video(tmp_path, monkeypatch):
    from PIL import Image

    from mujocoposelearning_amd.env import HumanoidEnv
    monkeypatch.chdir(tmp_path)
    env = HumanoidEnv({"model_path": XML, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3,
                       "render_mode": "rgb_array", "run_name": "t"})
    env.reset(seed=0)
    assert env.frames == [] and env.renderer is None
    rng = np.random.default_rng(0)
    expect = 0
    for k in range(30):
        env.step(rng.uniform(-1, 1, 21).astype(np.float32))
        # custom_env.py:283: a frame is appended while len(frames) < time * framerate
        if expect < env.data.time * env.framerate:
            expect += 1
        assert len(env.frames) == expect
    assert 20 <= expect < 30
    f0, f1 = env.frames[0], env.frames[-1]
    assert f0.shape == (480, 640, 3) and f0.dtype == np.uint8
    assert np.abs(f0.astype(int) - f1.astype(int)).sum() > 0      # the body moved
    n = len(env.frames)
    p = env.save_video(7)
    assert p == os.path.join("recordings", "t", "episode_7.gif") and os.path.exists(p)
    assert Image.open(p).n_frames == n
    assert env.frames == [] and env.renderer is None
    env.close()


def test_vecenv_get_images(model):
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3},
                         n_envs=4, model=model, seed=1)
    env.reset()
    rng = np.random.default_rng(1)
    for _ in range(20):
        env.step_async(rng.uniform(-1, 1, (4, 21)).astype(np.float32))
        env.step_wait()
    imgs = env.get_images(indices=[0, 3], height=96, width=128)
    assert len(imgs) == 2 and imgs[0].shape == (96, 128, 3) and imgs[0].dtype == np.uint8
    assert np.abs(imgs[0].astype(int) - imgs[1].astype(int)).sum() > 0     # different envs, different poses
    env.close()
