"""Full-state option (HS_FULL_STATE / env_config['full_state_obs']) on the GPU vs the oracle.

The reference leaves cfrc_ext / subtree_linvel at zero (custom_env.py never requests them; its
cfrc_ext obs line is commented out, :247,255).  With the option on, both are computed as
MuJoCo's mj_rnePostConstraint (contact part) / mj_subtreeVel define them -- restated in the
oracle and pinned there by the power identity against the efc path -- and the obs gains
cfrc_ext[1:] (448 floats).  fp64 parity bar: 1e-8 relative.
"""
import numpy as np
import pytest

from conftest import XML

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model():
    from mujocoposelearning_amd.model import HsModel
    return HsModel(XML)


@pytest.mark.parametrize("key", ["prone", "squat", "supine"])
def test_cfrc_ext_and_subtree_linvel_match_oracle_fp64(model, key):
    import torch
    from mujocoposelearning_amd.batch import HsBatch
    from oracle.oracle import Oracle
    o = Oracle(XML)
    q = o.M["keyframes"][key].copy()
    q[2] -= 0.004
    v = np.random.default_rng(5).normal(0, 0.3, 27)
    c = np.random.default_rng(6).uniform(-1, 1, 21)
    b = HsBatch(model, 1, precision="fp64", full_state=True)
    assert b.obs_dim == 352 + 6 * 16
    b.set_state(qpos=q, qvel=v, time=0.0, qacc_warmstart=0.0)
    b.physics_step(torch.tensor(c[None], dtype=torch.float32, device=b.device), 1)
    o.qpos[:] = q
    o.qvel[:] = v
    o.step(c.astype(np.float32).astype(np.float64), 1, full=True)
    cf, lv = b.cfrc_ext[0].cpu().numpy(), b.subtree_linvel[0].cpu().numpy()
    rc, rl = o.get("cfrc_ext"), o.get("subtree_linvel")
    assert o.d.ncon > 0 and np.abs(rc).max() > 1.0
    assert np.abs(cf - rc).max() <= 1e-8 * (1 + np.abs(rc).max())
    assert np.abs(lv - rl).max() <= 1e-8 * (1 + np.abs(rl).max())
    obs = b.obs[0].cpu().numpy()
    assert np.abs(obs[352:] - rc[1:].reshape(-1)).max() <= 1e-8 * (1 + np.abs(rc).max())


@pytest.mark.parametrize("reward", ["stand", "kneeling"])
def test_full_state_env_obs_and_reward_match_oracle_env(reward):
    """HumanoidEnv(full_state_obs=True) vs the oracle env over 40 env steps (same seeded reset
    noise): 448-dim obs and rewards whose foot / com-velocity terms now see real values."""
    from mujocoposelearning_amd.env import HumanoidEnv
    from oracle.env import OracleHumanoidEnv
    cfg = {"model_path": XML, "duration": 10.0, "reward_config": {"type": reward}, "frame_skip": 3,
           "full_state_obs": True, "precision": "fp64"}
    env, ref = HumanoidEnv(cfg), OracleHumanoidEnv(cfg)
    assert env.observation_space.shape == (448,)
    obs, _ = env.reset(seed=7)        # both draw the reset noise from numpy's legacy global RNG
    robs, _ = ref.reset(seed=7)
    rng = np.random.default_rng(2)
    assert np.abs(obs - robs).max() <= 1e-8 * (1 + np.abs(robs).max())
    foot_seen = False
    for k in range(40):
        a = rng.uniform(-1, 1, 21).astype(np.float32)
        obs, r, *_ = env.step(a)
        robs, rr, *_ = ref.step(a)
        scale = 1 + np.abs(robs).max()
        assert np.abs(obs - robs).max() <= 1e-7 * scale, k
        assert abs(r - rr) <= 1e-7 * (1 + abs(rr)), k
        foot_seen |= bool(np.abs(robs[352:]).max() > 1.0)   # some body (the feet) carries contact force
    assert foot_seen


def test_default_keeps_reference_zeros(model):
    import torch
    from mujocoposelearning_amd.batch import HsBatch
    b = HsBatch(model, 64, precision="fp32")
    b.configure(frame_skip=3, duration=10.0, reward_id=0)
    b.reset()
    for _ in range(20):
        b.step(torch.rand(64, 21, device=b.device) * 2 - 1)
    assert b.obs_dim == 352 and b.obs.shape[1] == 352
    assert not b.cfrc_ext.any() and not b.subtree_linvel.any()


def test_full_state_fp32_batch_is_finite_and_carries_the_weight(model):
    """configs[4]-style batch (full-state obs) in fp32: finite outputs, and once the passive
    humanoids lie on the floor, the time-averaged vertical contact force equals the weight
    (impulse balance: the average vertical acceleration of a lying body is ~0)."""
    import torch
    from mujocoposelearning_amd.batch import HsBatch
    n = 1024
    b = HsBatch(model, n, precision="fp32", full_state=True)
    b.configure(frame_skip=3, duration=1000.0, reward_id=1, max_steps=10 ** 6)
    b.reset()
    z = torch.zeros(n, 21, device=b.device)
    for _ in range(600):          # 9 s of passive collapse: everyone ends up lying on the floor
        obs, rew, *_ = b.step(z)
    acc = torch.zeros(n, device=b.device, dtype=torch.float64)
    for _ in range(200):
        obs, rew, *_ = b.step(z)
        acc += b.cfrc_ext[:, 1:, 5].sum(1).double()               # vertical force on all bodies
    torch.cuda.synchronize()
    assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
    mg = 40.84402122162132 * 9.81
    fz = acc / 200
    assert ((fz - mg).abs() < 0.05 * mg).float().mean() > 0.9
