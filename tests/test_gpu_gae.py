"""hs_gae (HIP reverse-scan GAE, gae.hip) through the C ABI vs the SB3 2.3.2 restatement.

SB3 is not installed here, so the anchor is the scalar-loop restatement of
RolloutBuffer.compute_returns_and_advantage in tests/test_ppo.py (parity unpinned against SB3
itself).  The kernel computes in fp32; tolerance: 2e-5 relative to the advantage scale.
"""
import numpy as np
import pytest

from test_ppo import _sb3_gae

pytestmark = pytest.mark.gpu


def _inputs(T, N, seed, p_start=0.05):
    rng = np.random.default_rng(seed)
    r = rng.normal(size=(T, N)).astype(np.float32)
    v = rng.normal(size=(T, N)).astype(np.float32)
    st = (rng.uniform(size=(T, N)) < p_start).astype(np.float32)
    lv = rng.normal(size=N).astype(np.float32)
    ld = (rng.uniform(size=N) < 0.3).astype(np.float32)
    return r, v, st, lv, ld


def _device(*xs):
    import torch
    return [torch.tensor(x, device="cuda") for x in xs]


@pytest.mark.parametrize("T,N", [(37, 300), (8, 64), (1, 5), (9, 257), (64, 1), (257, 300), (1000, 70), (256, 1),
                                 (2048, 130)])
def test_gae_kernel_matches_sb3_restatement(T, N):
    """T >= 256 takes the three-launch path (gae.hip GAE_SPLIT_T): (257, 300) ends on a one-step chunk."""
    from mujocoposelearning_amd.ppo import gae_device
    r, v, st, lv, ld = _inputs(T, N, seed=T * 1000 + N)
    ea, er = _sb3_gae(r.astype(np.float64), v.astype(np.float64), st.astype(np.float64),
                      lv.astype(np.float64), ld.astype(np.float64), 0.99, 0.95)
    adv, ret = gae_device(*_device(r, v, st, lv, ld), 0.99, 0.95)
    adv, ret = adv.cpu().numpy(), ret.cpu().numpy()
    scale = 1 + np.abs(ea).max()
    assert np.abs(adv - ea).max() <= 2e-5 * scale
    assert np.abs(ret - er).max() <= 2e-5 * scale


def test_gae_kernel_full_rollout_vs_torch_loop():
    """ppo_kwargs n_steps=2048 x 4096 envs (configs[1]): HIP scan == the fp32 torch loop."""
    import torch
    from mujocoposelearning_amd.ppo import gae, gae_device
    T, N = 2048, 4096
    r, v, st, lv, ld = _inputs(T, N, seed=7, p_start=1 / 667)
    ref_adv, ref_ret = gae(*[torch.tensor(x) for x in (r, v, st, lv, ld)], 0.99, 0.95)   # CPU torch loop
    adv, ret = gae_device(*_device(r, v, st, lv, ld), 0.99, 0.95)
    torch.cuda.synchronize()
    scale = 1 + ref_adv.abs().max().item()
    assert (adv.cpu() - ref_adv).abs().max().item() <= 2e-5 * scale
    assert (ret.cpu() - ref_ret).abs().max().item() <= 2e-5 * scale


def test_gae_kernel_episode_boundaries_cut_the_scan():
    """With every episode_start set, advantages reduce to one-step TD errors."""
    from mujocoposelearning_amd.ppo import gae_device
    T, N = 16, 70
    r, v, _, lv, _ = _inputs(T, N, seed=3)
    st = np.ones((T, N), np.float32)
    ld = np.ones(N, np.float32)
    adv, _ = gae_device(*_device(r, v, st, lv, ld), 0.99, 0.95)
    np.testing.assert_allclose(adv.cpu().numpy(), r - v, rtol=1e-6, atol=1e-6)


def test_gae_empty_sizes_are_noops():
    import torch
    from mujocoposelearning_amd import _lib
    lib = _lib.lib()
    z = torch.zeros(1, device="cuda")
    for T, N in ((0, 5), (5, 0)):
        assert lib.hs_gae(*[z.data_ptr()] * 7, T, N, 0.99, 0.95, None) == 0
    assert lib.hs_gae(*[z.data_ptr()] * 7, -1, 5, 0.99, 0.95, None) != 0
