"""mujocoposelearning_amd -- MI355X-native batched humanoid simulation + PPO rollout engine.

Drop-in for the hot path of redradman/MujocoPoseLearning: the per-process
``mujoco.mj_step`` / SB3 ``SubprocVecEnv`` path of custom_env.py, re-built as HIP kernels
for gfx950 behind the same ``HumanoidEnv`` / VecEnv / ``REWARD_FUNCTIONS`` surface.
Heavy modules (torch, the native library) load lazily on first use.
"""
import os as _os

__version__ = "0.2.0"
# the reference's model (XML/humanoid.xml, custom_env.py:53), shipped as package data
HUMANOID_XML = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "assets", "humanoid.xml")

from .reward_functions import REWARD_FUNCTIONS, robust_kneeling_reward, stand_reward, walk_reward  # noqa: F401
from .utils import quaternion_to_euler  # noqa: F401


def __getattr__(name):
    if name == "HumanoidEnv":
        from .env import HumanoidEnv
        return HumanoidEnv
    if name == "HumanoidVecEnv":
        from .vec_env import HumanoidVecEnv
        return HumanoidVecEnv
    if name in ("HsModel", "load_model"):
        from . import model
        return getattr(model, name)
    if name in ("PPO", "ActorCritic"):
        from . import ppo
        return getattr(ppo, name)
    if name == "train_humanoid":
        from .train import train_humanoid
        return train_humanoid
    if name == "HsBatch":
        from .batch import HsBatch
        return HsBatch
    raise AttributeError(name)
