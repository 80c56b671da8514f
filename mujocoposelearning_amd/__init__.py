"""mujocoposelearning_amd -- MI355X-native batched humanoid simulation + PPO rollout engine.

Drop-in for the hot path of redradman/MujocoPoseLearning: the per-process
``mujoco.mj_step`` / SB3 ``SubprocVecEnv`` path of custom_env.py, re-built as HIP kernels
for gfx950 behind the same ``HumanoidEnv`` / VecEnv / ``REWARD_FUNCTIONS`` surface.
"""
__version__ = "0.1.0"
