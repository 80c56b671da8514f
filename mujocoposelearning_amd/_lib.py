"""ctypes binding of the hsim C ABI (include/hsim.h).

The native library is REQUIRED: importing this module raises if ``libhsim.so`` is missing
(there is no CPU fallback in the product path -- the CPU restatement lives in ``oracle/``
and is test infrastructure only).
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HSIM_LIB", os.path.join(HERE, "libhsim.so"))   # HSIM_LIB: diagnostic builds

HS_FP32, HS_FP64 = 0, 1
HS_FULL_STATE = 0x100      # OR-ed into hs_batch_create's precision: cfrc_ext / subtree_linvel + 448-dim obs
HS_REWARD_NONE, HS_REWARD_STAND, HS_REWARD_KNEELING, HS_REWARD_WALK = -1, 0, 1, 2
HS_NWARN = 5
HS_AUXDIM = 40
HS_OUT_AUX, HS_OUT_CTRL = 1, 2   # hs_env_config.outputs bits
HS_SCHED_AUTO, HS_SCHED_DIRECT, HS_SCHED_SINGLE, HS_SCHED_FIXED_ORDER = 0, 1, 2, 3   # hs_env_config.schedule
DBGDIM = 32768


class hs_env_config(C.Structure):
    _fields_ = [("frame_skip", C.c_int), ("max_steps", C.c_int), ("reward_id", C.c_int), ("autoreset", C.c_int),
                ("max_newton", C.c_int), ("outputs", C.c_int), ("duration", C.c_double),
                ("init_height", C.c_double), ("noise_scale", C.c_double), ("kneel_params", C.c_double * 9),
                ("schedule", C.c_int)]


class hs_buffers(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("qpos", "qvel", "qacc_warmstart", "ctrl", "time", "step_count", "episode",
                                          "total_reward", "warning", "obs", "terminal_obs", "reward", "terminated",
                                          "truncated", "aux", "cfrc_ext", "subtree_linvel", "terminal_step_count",
                                          "terminal_total_reward")]


class hs_tape_out(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("obs", "reward", "terminated", "truncated")]


class hs_policy(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("w1", "b1", "w2", "b2", "w3", "b3", "log_std")] + \
               [("ld1", C.c_int), ("obs_dim", C.c_int), ("act_dim", C.c_int)]


class hs_rollout_bufs(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("obs", "obs_last", "actions", "log_probs", "episode_starts", "rewards",
                                          "dones", "episode_returns", "boot", "terminal_obs", "ep_acc",
                                          "episode_start", "actions_clipped", "counter_base")] + \
               [("seed", C.c_uint64), ("deterministic", C.c_int)]


class hs_batch_info(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("n_envs", "precision", "nq", "nv", "nu", "nbody", "obs_dim", "elem_size",
                                       "resident_con", "resident_efc", "wide_con", "wide_efc", "resident_waves",
                                       "bound_con_all", "bound_efc_all", "bound_con_floor", "bound_efc_floor")]


_LIB = None


def lib():
    """Load libhsim.so (build it with ``python -c 'import __graft_entry__ as g; g.build()'``)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"hsim native library not found at {LIB_PATH}; build it first "
                          f"(make -C mujocoposelearning_amd/csrc)")
    # Bind to the HIP runtime torch already loaded (same SONAME libamdhip64.so.7): one HIP
    # runtime per process, so torch-allocated buffers and streams are valid in the library.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, i, d, u64 = C.c_void_p, C.c_int, C.c_double, C.c_uint64
    sig = {
        "hs_model_load": (vp, [C.c_char_p, C.c_char_p, i]),
        "hs_model_free": (None, [vp]),
        "hs_model_field": (i, [vp, C.c_char_p, vp, i]),
        "hs_batch_create": (vp, [vp, i, i, u64, i, vp]),
        "hs_batch_destroy": (None, [vp]),
        "hs_batch_get_info": (i, [vp, vp]),
        "hs_get_buffers": (i, [vp, vp]),
        "hs_set_config": (i, [vp, vp]),
        "hs_get_config": (i, [vp, vp]),
        "hs_set_seed": (i, [vp, u64]),
        "hs_reset": (i, [vp, vp, vp, vp, vp]),
        "hs_step": (i, [vp, vp, vp]),
        "hs_step_tape": (i, [vp, vp, i, vp, vp]),
        "hs_tape_aborts": (i, [vp, vp]),
        "hs_last_tape_ms": (i, [vp, vp]),
        "hs_stream_orders": (i, [vp, vp]),
        "hs_rollout": (i, [vp, vp, vp, i, i, i, vp]),
        "hs_rollout_max_steps": (i, [vp]),
        "hs_set_autoreset_noise": (i, [vp, vp, vp]),
        "hs_physics_step": (i, [vp, vp, i, vp]),
        "hs_state_io": (i, [vp, i, vp, vp, vp, vp, vp]),
        "hs_kinematics": (i, [vp, i, vp, vp, vp, vp, vp, vp]),
        "hs_set_debug": (i, [vp, i]),
        "hs_debug_lose_handoff": (i, [vp, i]),
        "hs_get_debug": (i, [vp, vp, i]),
        "hs_synchronize": (i, [vp]),
        "hs_batch_counters": (i, [vp, vp]),
        "hs_gae": (i, [vp, vp, vp, vp, vp, vp, vp, i, i, C.c_float, C.c_float, vp]),
        "hs_reward_eval": (i, [vp, i, i, vp, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "hs_pack_outputs": (i, [vp, vp, i, i, vp]),
        "hs_reward": (i, [vp, i, vp, vp, vp]),
        "hs_ppo_act": (i, [vp, i, vp, i, vp, vp, u64, u64, vp, i, vp, vp, vp, vp, vp, i, i, vp]),
        "hs_ppo_post": (i, [vp, vp, vp, vp, vp, vp, vp, i, C.c_float, vp, vp, u64, vp, vp, vp, vp, vp, i, vp]),
        "hs_gauss_logp": (i, [vp, i, vp, vp, vp, i, i, vp]),
        "hs_gauss_logp_grad": (i, [vp, i, vp, vp, vp, vp, vp, i, i, vp]),
        "hs_ppo_loss_workspace": (u64, [i]),
        "hs_ppo_loss": (i, [vp, vp, vp, vp, vp, vp, i, C.c_float, i, vp, vp, vp, vp]),
        "hs_ppo_loss_grad": (i, [vp, vp, i, C.c_float, vp, vp, vp, vp, vp, vp]),
        "hs_adam_workspace": (u64, [u64]),
        "hs_adam_clip": (i, [i, vp, vp, vp, vp, vp, vp, vp, C.c_float, C.c_double, C.c_double, C.c_double, C.c_double,
                             vp]),
        "hs_mlp2_forward": (i, [vp, i, i, i, vp, i, vp, vp, i, vp, vp, i, vp, i, vp, i, vp]),
        "hs_colsum_partial_rows": (u64, [u64, u64]),
        "hs_relu_grad_colsum": (i, [vp, vp, u64, u64, vp, vp, vp]),
        "hs_dgrad_mask_partial_rows": (u64, [i, i]),
        "hs_dgrad_mask_workspace": (u64, [i]),
        "hs_dgrad_mask": (i, [vp, i, i, vp, i, vp, i, i, i, vp, vp, vp, vp]),
        "hs_colsum_pair": (i, [vp, u64, u64, vp, vp, u64, u64, vp, vp]),
        "hs_colsum_workspace": (u64, [u64, u64]),
        "hs_colsum": (i, [vp, u64, u64, vp, vp, vp, vp]),
        "hs_last_error": (C.c_char_p, []),
        "hs_version": (C.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = L
    return L


EXPORTED = ("hs_model_load", "hs_model_free", "hs_model_field", "hs_batch_create", "hs_batch_destroy",
            "hs_batch_get_info", "hs_get_buffers", "hs_set_config", "hs_set_seed", "hs_get_config", "hs_reset", "hs_step", "hs_step_tape", "hs_tape_aborts", "hs_last_tape_ms", "hs_stream_orders", "hs_rollout", "hs_rollout_max_steps", "hs_set_autoreset_noise",
            "hs_physics_step", "hs_state_io", "hs_kinematics", "hs_set_debug", "hs_debug_lose_handoff", "hs_get_debug", "hs_synchronize", "hs_batch_counters", "hs_gae",
            "hs_reward_eval", "hs_reward", "hs_pack_outputs",
            "hs_ppo_act", "hs_ppo_post", "hs_gauss_logp", "hs_gauss_logp_grad",
            "hs_ppo_loss_workspace", "hs_ppo_loss", "hs_ppo_loss_grad", "hs_adam_workspace", "hs_adam_clip",
            "hs_mlp2_forward", "hs_colsum_partial_rows", "hs_relu_grad_colsum", "hs_dgrad_mask_partial_rows",
            "hs_dgrad_mask_workspace", "hs_dgrad_mask", "hs_colsum_pair",
            "hs_colsum_workspace", "hs_colsum", "hs_last_error", "hs_version")


class HsimError(RuntimeError):
    pass


def check(rc):
    if rc is None or (isinstance(rc, int) and rc < 0):
        raise HsimError(lib().hs_last_error().decode())
    return rc
