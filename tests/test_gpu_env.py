"""GPU env semantics and full-size properties (BASELINE.json configs[1]: 4096 envs, stand,
frame_skip 3, duration 10) through the C ABI."""
import numpy as np
import pytest

from conftest import XML

pytestmark = pytest.mark.gpu
CFG = {"model_path": XML, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3}


@pytest.fixture(scope="module")
def model():
    from mujocoposelearning_amd.model import HsModel
    return HsModel(XML)


def _batch(model, n, prec="fp32", seed=0, reward=0, autoreset=1):
    from mujocoposelearning_amd.batch import HsBatch
    b = HsBatch(model, n, precision=prec, seed=seed)
    b.configure(frame_skip=3, duration=10.0, reward_id=reward, autoreset=autoreset, max_steps=750)
    return b


def test_termination_at_667_and_autoreset(model):
    import torch
    n = 64
    b = _batch(model, n)
    b.reset()
    # fast-forward every env's clock to just before the end (physics state unchanged)
    st = b.get_state()
    b.set_state(time=st["time"] + 0.015 * 665)
    b.step_count.fill_(665)
    a = torch.zeros(n, 21, device=b.device)
    obs, rew, term, trunc = b.step(a)
    assert not term.any() and not trunc.any()
    obs, rew, term, trunc = b.step(a)
    assert term.all() and not trunc.any()
    # auto-reset: fresh episode (time = one reset substep, step_count 0), terminal obs kept
    st = b.get_state()
    assert np.allclose(st["time"], 0.005)
    assert (b.step_count == 0).all() and (b.episode == 2).all()
    assert not torch.equal(b.terminal_obs, b.obs)
    assert torch.isfinite(b.obs).all()


def test_truncation_reward_zero(model):
    import torch
    b = _batch(model, 8)
    b.configure(duration=1e9)
    b.reset()
    b.step_count.fill_(749)
    _, rew, term, trunc = b.step(torch.zeros(8, 21, device=b.device))
    assert trunc.all() and not term.any() and (rew == 0).all()


def test_vecenv_sb3_surface(model):
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv(CFG, n_envs=8, model=model, seed=4)
    obs = env.reset()
    assert obs.shape == (8, 352) and obs.dtype == np.float64
    a = np.random.default_rng(0).uniform(-1, 1, (8, 21)).astype(np.float32)
    obs, rew, dones, infos = env.step(a)
    assert obs.shape == (8, 352) and rew.shape == (8,) and dones.shape == (8,) and len(infos) == 8
    assert not dones.any() and infos[0]["step_count"] == 1
    env.batch.set_state(time=np.full(8, 9.999))
    obs, rew, dones, infos = env.step(a)
    assert dones.all()
    for i in range(8):
        assert "terminal_observation" in infos[i] and infos[i]["TimeLimit.truncated"] is False
        assert infos[i]["terminal_observation"].shape == (352,)
    assert env.get_attr("frame_skip") == [3] * 8
    assert env.env_is_wrapped(object) == [False] * 8
    assert env.seed(7) == list(range(7, 15))
    env.close()


def test_full_size_determinism_and_batch_invariance(model):
    """configs[1] size: 4096 envs.  Bitwise-identical reruns; an env's trajectory does not depend
    on its neighbours (same state in a 1-env batch and at index 17 of the 4096-env batch)."""
    import torch
    n = 4096
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = torch.rand(20, n, 21, device="cuda", generator=g) * 2 - 1
    outs = []
    for rep in range(2):
        b = _batch(model, n, seed=9)
        b.reset()
        for k in range(20):
            b.step(acts[k])
        outs.append((b.qpos.clone(), b.qvel.clone(), b.obs.clone(), b.reward.clone()))
        st0 = b.get_state()
        warn = b.warning.sum(0).tolist()
        aux = b.aux.clone()
    for x, y in zip(*outs):
        assert torch.equal(x, y)
    assert torch.isfinite(outs[0][2]).all()
    assert warn == [0, 0, 0, 0, 0]
    assert int(aux[:, 35].max()) >= 1 and int(aux[:, 36].max()) >= 4      # contacts are being solved
    # batch-composition invariance
    b1 = _batch(model, 1, seed=9)
    b1.reset()
    idx = 17
    b1.set_state(qpos=st0["qpos"][idx], qvel=st0["qvel"][idx], qacc_warmstart=st0["qacc_warmstart"][idx],
                 time=st0["time"][idx], ctrl=st0["ctrl"][idx])
    bN = _batch(model, n, seed=9)
    bN.set_state(**{k: v for k, v in st0.items()})
    a = acts[0]
    b1.step(a[idx:idx + 1])
    bN.step(a)
    assert torch.equal(b1.qpos[0], bN.qpos[idx]) and torch.equal(b1.obs[0], bN.obs[idx])


def test_chunk_queue_schedule_bitwise_equals_direct(model):
    """The fp64 engine at configs[1] size runs on the chunk-queue schedule (2048 env pairs > 1024
    resident waves: each env step as two items, the state handed over through uncached memory,
    DESIGN.md 3.1).  It must give bitwise the states, obs, rewards, done flags, auto-reset info and
    warnings of one wave per pair -- through falls, contacts and auto-resets (staggered clocks: some
    envs terminate at every step), including odd batch sizes (a ghost half-wave)."""
    import torch
    for n in (4096, 3001):
        g = torch.Generator(device="cuda").manual_seed(4)
        acts = torch.rand(40, n, 21, device="cuda", generator=g) * 2 - 1
        t0 = np.floor(np.arange(n) * 667 / n) * 0.015 + 0.005
        outs = []
        for sched in ("auto", "direct"):
            b = _batch(model, n, prec="fp64", seed=3)
            b.configure(schedule=sched)
            b.reset()
            b.set_state(time=t0)
            tr = []
            for k in range(40):
                b.step(acts[k])
                if k % 10 == 9:
                    tr += [b.obs.clone(), b.reward.clone(), b.terminated.clone(), b.truncated.clone()]
            tr += [b.qpos.clone(), b.qvel.clone(), b.qacc_warmstart.clone(), b.time.clone(), b.warning.clone(),
                   b.terminal_obs.clone(), b.terminal_step_count.clone(), b.terminal_total_reward.clone(),
                   b.episode.clone(), b.aux.clone()]
            outs.append(tr)
        assert int(outs[0][-2].min()) >= 1 and int(outs[0][-2].max()) >= 2      # auto-resets happened
        for x, y in zip(*outs):
            assert torch.equal(x, y)


def test_reset_distribution_device_rng(model):
    """On-device reset noise: U(-.01, .01) per coordinate, z noise x0.1, quaternion exact; the
    reset then runs exactly one substep (time 0.005)."""
    n = 4096
    b = _batch(model, n, seed=123)
    b.configure(max_newton=100)
    b.reset()
    st = b.get_state()
    assert np.allclose(st["time"], 0.005)
    # root x, y move only h * |v| ~ 5e-5 in the one reset substep: they carry the raw noise
    xy = st["qpos"][:, :2].ravel()
    assert np.abs(xy).max() < 0.0101
    hist, _ = np.histogram(xy, bins=10, range=(-0.01, 0.01))
    assert np.all(np.abs(hist / xy.size - 0.1) < 0.02)
    assert abs(xy.mean()) < 5e-4 and abs(xy.std() - 0.02 / np.sqrt(12)) < 5e-4
    # root z: init height 1.282 + 0.1 * noise, then one substep of settling
    assert np.abs(st["qpos"][:, 2] - 1.282).max() < 0.0015
    quat = st["qpos"][:, 3:7]
    assert np.allclose(np.linalg.norm(quat, axis=1), 1, atol=1e-6)
    assert np.abs(quat[:, 0] - 1).max() < 1e-3
    # different seeds -> different states, same seed -> identical
    b2 = _batch(model, n, seed=123)
    b2.reset()
    assert np.array_equal(b2.get_state()["qpos"], st["qpos"])
    b3 = _batch(model, n, seed=124)
    b3.reset()
    assert not np.array_equal(b3.get_state()["qpos"], st["qpos"])


def test_bad_state_autoreset_warning(model):
    """mj_checkPos semantics: a NaN qpos resets that env to qpos0 / time 0 and bumps a warning."""
    import torch
    b = _batch(model, 4)
    b.reset()
    st = b.get_state()
    q = st["qpos"].copy()
    q[2, 10] = np.nan
    b.set_state(qpos=q)
    b.physics_step(torch.zeros(4, 21, device=b.device), 1)
    w = b.warning.cpu().numpy()
    assert w[2, 0] == 1 and w[[0, 1, 3], 0].sum() == 0
    st2 = b.get_state()
    assert st2["time"][2] == pytest.approx(0.005, abs=1e-7)
    assert np.all(np.isfinite(st2["qpos"]))


def test_action_clamp_and_reward_reads_raw_ctrl(model):
    """Force uses clamp(ctrl, -1, 1) (motor ctrlrange), the stand reward reads the raw ctrl."""
    import torch
    b = _batch(model, 2, prec="fp64")
    b.configure(autoreset=0)
    b.reset()
    st = b.get_state()
    b2 = _batch(model, 2, prec="fp64")
    b2.configure(autoreset=0)
    b2.set_state(**st)
    big = torch.full((2, 21), 3.0, device=b.device)
    one = torch.full((2, 21), 1.0, device=b.device)
    _, r_big, *_ = b.step(big)
    _, r_one, *_ = b2.step(one)
    assert torch.equal(b.qpos, b2.qpos)            # identical physics
    s = b.get_state()
    if s["qpos"][0, 2] >= 0.8:
        assert (r_big < r_one).all()                # torque penalty sees 3.0, not 1.0


def test_integration_md_ctypes_stub_runs():
    """The C-ABI binding stub of INTEGRATION.md section 2, executed as written (model path
    pointed at the fixture), then checked against the Python layer's view of the same step."""
    import os
    import re
    import torch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = open(os.path.join(root, "INTEGRATION.md")).read()
    code = re.findall(r"```python\n(# hsim_binding.py.*?)```", text, re.S)[0]
    code = code.replace('b"XML/humanoid.xml"', repr(XML.encode())).replace(
        '"mujocoposelearning_amd/libhsim.so"', repr(os.path.join(root, "mujocoposelearning_amd", "libhsim.so")))
    ns = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    lib, batch = ns["lib"], ns["batch"]
    from mujocoposelearning_amd import _lib
    bi = _lib.hs_batch_info()
    lib.hs_batch_get_info.argtypes = [_lib.C.c_void_p, _lib.C.c_void_p]
    assert lib.hs_batch_get_info(_lib.C.c_void_p(batch), _lib.C.byref(bi)) == 0
    assert (bi.n_envs, bi.obs_dim, bi.nu) == (4096, 352, 21)
    torch.cuda.synchronize()
    lib.hs_batch_destroy.argtypes = [_lib.C.c_void_p]
    lib.hs_model_free.argtypes = [_lib.C.c_void_p]
    lib.hs_batch_destroy(_lib.C.c_void_p(batch))
    lib.hs_model_free(_lib.C.c_void_p(ns["model"]))


def test_train_humanoid_short_run(tmp_path):
    """train_sb3.py:170-240 mirror: a short on-device PPO run through train_humanoid."""
    from mujocoposelearning_amd.train import train_humanoid
    env_kwargs = {"n_envs": 64, "reward_function": "stand", "frame_skip": 3, "total_timesteps": 64 * 16 * 2}
    ppo_kwargs = {"n_steps": 16, "batch_size": 256, "n_epochs": 2,
                  "policy_kwargs": {"activation_fn": "ReLU", "net_arch": {"pi": [256, 256], "vf": [256, 256]}}}
    m = train_humanoid(env_kwargs, ppo_kwargs, xml_path=XML, storage_path=str(tmp_path))
    assert m.num_timesteps == 64 * 16 * 2
    assert np.isfinite(m.logger["policy_loss"]) and np.isfinite(m.logger["value_loss"])
    assert (tmp_path / "final_model.zip").exists()


def test_generate_trajectory_xml_with_saved_policy(tmp_path):
    """generate_trajectories.py mirror end to end on the GPU engine: a PPO checkpoint saved in the
    SB3 layout is reloaded and rolled out; the keyframes follow the reference file's layout."""
    import xml.etree.ElementTree as ET
    from mujocoposelearning_amd.ppo import ActorCritic
    from mujocoposelearning_amd.sb3_format import save_sb3_zip
    from mujocoposelearning_amd.trajectories import generate_trajectory_xml
    pol = ActorCritic(352, 21, [64, 64], [64, 64])
    zp = save_sb3_zip(tmp_path / "final_model", pol, None, {"policy_kwargs": {"net_arch": [64, 64],
                                                                              "activation_fn": "Tanh"}})
    out = generate_trajectory_xml(zp, XML, tmp_path / "traj.xml", num_steps=40, step_interval=5)
    keys = ET.parse(out).getroot().find("keyframe").findall("key")
    assert keys[4].get("name") == "initial_pose" and len(keys) == 4 + 1 + 8
    assert [k.get("time") for k in keys[5:]] == [f"{s * 0.005:.3f}" for s in range(0, 40, 5)]
    q = np.array(keys[4].get("qpos").split(), float)
    assert abs(q[2] - 1.282) < 0.002 and np.isfinite(q).all()


def test_stream_groups_are_bitwise_identical_to_one_batch(model):
    """HsBatch(groups=4) (4 native sub-batches on 4 HIP streams over slices of the same tensors)
    steps every env exactly like one batch."""
    import torch
    from mujocoposelearning_amd.batch import HsBatch
    n = 1000                                   # ragged: 250 per group
    rng = np.random.default_rng(0)
    q0 = np.tile(model.qpos0, (n, 1))
    q0[:, 2] = 1.282
    q0[:, 3:7] = [1, 0, 0, 0]
    q0 += rng.uniform(-0.01, 0.01, q0.shape) * np.r_[1, 1, 0.1, 0, 0, 0, 0, np.ones(21)]
    v0 = rng.uniform(-0.01, 0.01, (n, 27))
    tape = torch.tensor(rng.uniform(-1, 1, (30, n, 21)), dtype=torch.float32, device="cuda")
    outs = []
    for G in (1, 4):
        b = HsBatch(model, n, precision="fp32", groups=G)
        assert len(b._groups) == G
        b.configure(frame_skip=3, duration=10.0, reward_id=0)
        b.set_state(qpos=q0, qvel=v0, time=0.005, qacc_warmstart=0.0)
        for k in range(30):
            obs, rew, term, trunc = b.step(tape[k], join=(k % 2 == 0))   # free-running half the time
        b.join()
        torch.cuda.synchronize()
        outs.append((obs.clone(), rew.clone(), b.get_state()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    for k in ("qpos", "qvel", "qacc_warmstart", "time"):
        assert np.array_equal(outs[0][2][k], outs[1][2][k]), k


def test_grouped_vecenv_episode_semantics():
    """2048 envs in 4 stream groups: every env terminates at step 667 and auto-resets."""
    import torch
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv(CFG, n_envs=2048, groups=4)
    assert len(env.batch._groups) == 4
    env.reset_tensors()
    a = torch.zeros(2048, 21, device=env.device)
    for k in range(667):
        obs, rew, term, trunc = env.step_tensors(a)
        if k < 666:
            assert not term.any()
    torch.cuda.synchronize()
    assert term.all() and not trunc.any()
    assert (env.batch.step_count == 0).all() and torch.isfinite(obs).all()
    assert (env.batch.terminal_obs[:, 0] != obs[:, 0]).any()


def test_vecenv_host_reward_callable_matches_device_reward(model):
    """Reward plug-in surface (custom_env.py:263-271) for the batched env: a user-registered
    callable runs on the host over per-env data views.  Registered as a copy of stand_reward it
    must reproduce the device 'stand' rewards, and finished envs still auto-reset SB3-style."""
    import torch

    from mujocoposelearning_amd import reward_functions as rf
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv

    def stand_copy(data, params=None):
        return rf.stand_reward(data, params)

    rf.REWARD_FUNCTIONS["stand_host"] = stand_copy
    try:
        n = 16
        dev = HumanoidVecEnv(CFG, n_envs=n, model=model, seed=3)
        host = HumanoidVecEnv(dict(CFG, reward_config={"type": "stand_host", "params": {}}), n_envs=n, model=model,
                              seed=3)
        assert host._host_reward is stand_copy and host._host_params[0] is not host._host_params[1]
        o1, o2 = dev.reset(), host.reset()
        np.testing.assert_array_equal(o1, o2)
        rng = np.random.default_rng(0)
        for k in range(12):
            a = rng.uniform(-1, 1, (n, 21)).astype(np.float32)
            dev.step_async(a)
            host.step_async(a)
            od, rd, dd, _ = dev.step_wait()
            oh, rh, dh, ih = host.step_wait()
            np.testing.assert_allclose(oh, od, rtol=0, atol=0)
            np.testing.assert_allclose(rh, rd, atol=2e-6)
            assert not dh.any()
        # stand_reward's side effect lands in each env's own params (reward_functions.py:208-209)
        np.testing.assert_allclose(host._host_params[5]["previous_qpos"], host.batch.get_state()["qpos"][5])
        # episode end: reward on the pre-reset state, terminal_observation, fresh episode
        for env in (dev, host):
            st = env.batch.get_state()
            env.batch.set_state(time=st["time"] + 0.015 * (666 - 12))
            env.batch.step_count.fill_(666)
        a = np.zeros((n, 21), np.float32)
        dev.step_async(a)
        host.step_async(a)
        od, rd, dd, idv = dev.step_wait()
        oh, rh, dh, ih = host.step_wait()
        assert dd.all() and dh.all()
        np.testing.assert_allclose(rh, rd, atol=2e-6)
        for i in range(n):
            np.testing.assert_allclose(ih[i]["terminal_observation"], idv[i]["terminal_observation"], atol=0)
            # SubprocVecEnv returns the finished episode's last info: step_count 667, its return
            assert ih[i]["TimeLimit.truncated"] is False and ih[i]["step_count"] == 667
            assert idv[i]["step_count"] == 667
            assert ih[i]["total_reward"] == pytest.approx(idv[i]["total_reward"], abs=1e-4)
        assert int(host.batch.step_count.max()) == 0
        assert float(host.batch.time.max()) == pytest.approx(0.005)
        assert torch.isfinite(host.batch.obs).all()
        dev.close()
        host.close()
    finally:
        del rf.REWARD_FUNCTIONS["stand_host"]


def test_vecenv_seeded_worker_streams_match_golden(model):
    """SB3 exactness (train_sb3.py:203, custom_env.py:99-110): built from the reference's
    ``[make_env(env_config, i) for i in range(4)]`` form, after ``seed(100)`` env i's first reset
    and its next two auto-resets use the noise of worker i's np.random stream (seed 100 + i) --
    the golden fixture -- and land on the oracle env's post-reset state (fp64, <= 1e-12)."""
    import os

    from conftest import GOLDEN
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    from oracle.env import OracleHumanoidEnv
    g = np.load(os.path.join(GOLDEN, "reset_noise_golden.npz"))

    def make_env(env_config, rank):          # the reference's factory shape (train_sb3.py:108-115)
        def _init():                         # closes over env_config; must not be called
            raise AssertionError(f"factory called ({env_config})")
        return _init
    cfg = dict(CFG)
    fns = [make_env(cfg, i) for i in range(4)]
    venv = HumanoidVecEnv(fns, precision="fp64")
    assert venv.num_envs == 4
    assert venv.seed(100) == [100, 101, 102, 103]
    obs = venv.reset()
    for k in range(3):
        for i in range(4):
            ref = OracleHumanoidEnv(cfg)
            ob, _ = ref.reset(pos_noise=g[f"stream_pos_{100 + i}_{k}"], vel_noise=g[f"stream_vel_{100 + i}_{k}"])
            assert np.abs(obs[i] - ob).max() <= 1e-12 * (1 + np.abs(ob).max()), (k, i)
        if k == 2:
            break
        # run every env to the end of its episode: the auto-reset draws the stream's next block
        st = venv.batch.get_state()
        venv.batch.set_state(time=st["time"] + 0.015 * 666)
        venv.batch.step_count.fill_(666)
        venv.step_async(np.zeros((4, 21), np.float32))
        obs, _, dones, infos = venv.step_wait()
        assert dones.all() and all(inf["step_count"] == 667 for inf in infos)
    venv.close()


def _reference_step_wait(env, actions):
    """The round-4 step_wait (one blocking copy per field, eager info dicts), kept as the reference the
    packed / lazy version must equal: obs, rewards, dones and every info dict."""
    import torch
    obs, rew, term, trunc = env.step_tensors(torch.as_tensor(actions, device=env.batch.device))
    obs_np = obs.double().cpu().numpy()
    rew_np = rew.double().cpu().numpy()
    term_np = term.cpu().numpy().astype(bool)
    trunc_np = trunc.cpu().numpy().astype(bool)
    dones = term_np | trunc_np
    tot = env.batch.total_reward.double().cpu().numpy()
    step_count = env.batch.step_count.cpu().numpy()
    term_obs = env.batch.terminal_obs.double().cpu().numpy()
    step_count = np.where(dones, env.batch.terminal_step_count.cpu().numpy(), step_count)
    tot = np.where(dones, env.batch.terminal_total_reward.double().cpu().numpy(), tot)
    infos = []
    for i in range(env.num_envs):
        info = {"reward_components": {}, "height": None, "step_count": int(step_count[i]),   # custom_env.py:216-224
                "truncated": bool(trunc_np[i]), "truncation_info": {"reason": "timeout"} if trunc_np[i] else {},
                "terminated": bool(term_np[i]), "total_reward": float(tot[i])}
        if dones[i]:
            info["terminal_observation"] = term_obs[i]
            info["TimeLimit.truncated"] = bool(trunc_np[i] and not term_np[i])
            info["height"] = float(term_obs[i][0])
        else:
            info["height"] = float(obs_np[i][0])
        infos.append(info)
    return obs_np, rew_np, dones, infos


@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_vecenv_step_wait_equals_the_reference_path_on_episode_boundaries(model, prec):
    """step_wait's packed single copy and lazy StepInfos equal the eager per-field path on steps where
    envs terminate (time >= duration), are truncated (750 steps: TimeLimit.truncated) or run on:
    obs, rewards, dones, and every info dict key by key, with the same Python types."""
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    n = 64
    envs = [HumanoidVecEnv(CFG, n_envs=n, model=model, seed=5, precision=prec) for _ in range(2)]
    for e in envs:
        e.reset()
        st = e.batch.get_state()
        t = st["time"].copy()
        t[: n // 2] += 0.015 * (664 - np.arange(n // 2) % 3)      # these reach duration within 3 steps
        e.batch.set_state(time=t)
        e.batch.step_count[n // 2: 3 * n // 4].fill_(748)           # these hit max_steps (750)
    rng = np.random.default_rng(1)
    ends = set()
    for k in range(4):
        a = rng.uniform(-1, 1, (n, 21)).astype(np.float32)
        envs[0].step_async(a)
        o1, r1, d1, i1 = envs[0].step_wait()
        o2, r2, d2, i2 = _reference_step_wait(envs[1], a)
        np.testing.assert_array_equal(o1, o2)
        np.testing.assert_array_equal(r1, r2)
        np.testing.assert_array_equal(d1, d2)
        assert len(i1) == len(i2) == n and type(d1[0]) is type(d2[0])
        for i in range(n):
            x, y = i1[i], i2[i]
            assert x.keys() == y.keys(), (k, i)
            for key in y:
                if key == "terminal_observation":
                    np.testing.assert_array_equal(x[key], y[key])
                else:
                    assert x[key] == y[key] and type(x[key]) is type(y[key]), (k, i, key, x[key], y[key])
            if d2[i]:
                ends.add("trunc" if y["TimeLimit.truncated"] else "term")
        assert [a["step_count"] for a in i1[-3:]] == [b["step_count"] for b in i2[-3:]]   # slices
    assert ends == {"trunc", "term"}
    for e in envs:
        e.close()
