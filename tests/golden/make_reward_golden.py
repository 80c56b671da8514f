"""Generate reward / euler golden vectors from the REFERENCE's own Python (run in the build
container only, where /root/reference exists; the GPU box never runs this).

The reference functions (reward_functions.py:66-269, utils.py:3-21) need only numpy, so
they are imported from /root/reference and evaluated on a duck-typed ``env_data``
(SimpleNamespace with the MjData fields they read).  Inputs and outputs are written to
``tests/golden/reward_golden.npz``; no reference source is copied.

Also writes ``reset_noise_golden.npz``: the legacy-MT19937 reset noise stream of
custom_env.py:99-117 for seeds 0..4 (pos noise drawn before vel noise), and three consecutive
resets of SubprocVecEnv workers 0..3 after VecEnv.seed(100) (seeds 100..103).
"""
import os
import sys
from types import SimpleNamespace

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.path.insert(0, REF)
    import reward_functions as rf  # noqa: E402  (reference module, evaluated not copied)
    import utils as ru  # noqa: E402

    rng = np.random.default_rng(1234)
    keys = {
        "squat": [0, 0, 0.596, 0.988015, 0, 0.154359, 0, 0, 0.4, 0, -0.25, -0.5, -2.5, -2.65, -0.8, 0.56,
                  -0.25, -0.5, -2.5, -2.65, -0.8, 0.56, 0, 0, 0, 0, 0, 0],
        "stand_on_left_leg": [0, 0, 1.21948, 0.971588, -0.179973, 0.135318, -0.0729076, -0.0516, -0.202, 0.23,
                              -0.24, -0.007, -0.34, -1.76, -0.466, -0.0415, -0.08, -0.01, -0.37, -0.685, -0.35,
                              -0.09, 0.109, -0.067, -0.7, -0.05, 0.12, 0.16],
    }
    cases = []
    # keyframe cases (SURVEY.md 4.1 observed values)
    for name, q in keys.items():
        cases.append(dict(qpos=np.array(q), qvel=np.zeros(27), ctrl=np.zeros(21), time=0.005,
                          cfrc_ext=np.zeros((17, 6)), subtree_com=np.zeros((17, 3)), subtree_linvel=np.zeros((17, 3)),
                          qfrc_actuator=np.zeros(27)))
    # random states: heights spanning both branches, random unit quats, some with nonzero cfrc_ext
    for i in range(200):
        q = np.zeros(28)
        q[:3] = rng.normal(0, 0.3, 3)
        q[2] = rng.uniform(0.0, 1.6)
        quat = rng.normal(size=4)
        if i % 3 == 0:                       # near-upright
            quat = np.array([1.0, *rng.normal(0, 0.15, 3)])
        q[3:7] = quat / np.linalg.norm(quat)
        q[7:] = rng.uniform(-1.5, 1.5, 21)
        qvel = rng.normal(0, 1.0, 27)
        ctrl = rng.uniform(-1.2, 1.2, 21)
        gear = np.array([40, 40, 40, 40, 40, 120, 80, 20, 20, 40, 40, 120, 80, 20, 20, 20, 20, 40, 20, 20, 40.0])
        qfa = np.zeros(27)
        qfa[6:] = gear * np.clip(ctrl, -1, 1)
        cf = np.zeros((17, 6)) if i % 2 == 0 else rng.normal(0, 50, (17, 6))
        sc = rng.normal(0, 0.2, (17, 3))
        sl = np.zeros((17, 3)) if i % 4 else rng.normal(0, 1, (17, 3))
        cases.append(dict(qpos=q, qvel=qvel, ctrl=ctrl, time=float(rng.uniform(0, 10)), cfrc_ext=cf,
                          subtree_com=sc, subtree_linvel=sl, qfrc_actuator=qfa))
    # NaN-pitch edge case: |2(wy - zx)| > 1 after rounding (non-unit quaternion input)
    q = np.zeros(28); q[2] = 1.2; q[3:7] = [0.8, 0.0, 0.8, 0.0]
    cases.append(dict(qpos=q, qvel=np.zeros(27), ctrl=np.zeros(21), time=1.0, cfrc_ext=np.zeros((17, 6)),
                      subtree_com=np.zeros((17, 3)), subtree_linvel=np.zeros((17, 3)), qfrc_actuator=np.zeros(27)))

    out = {k: np.stack([c[k] for c in cases]) for k in cases[0]}
    names = ["default", "stand", "kneeling", "walk"]
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for n in names:
            out["reward_" + n] = np.array([rf.REWARD_FUNCTIONS[n](SimpleNamespace(**c), None) for c in cases], float)
        out["euler"] = np.array([ru.quaternion_to_euler(c["qpos"][3:7]) for c in cases], float)
    np.savez_compressed(os.path.join(OUT, "reward_golden.npz"), **out)

    noise = {}
    for s in range(5):
        np.random.seed(s)
        noise[f"pos_{s}"] = np.random.uniform(low=-0.01, high=0.01, size=28)
        noise[f"vel_{s}"] = np.random.uniform(low=-0.01, high=0.01, size=27)
    # SubprocVecEnv worker streams after VecEnv.seed(100): worker i reset(seed=100 + i), then two
    # auto-resets (reset(seed=None)) continuing the worker's global stream (custom_env.py:99-110)
    for i in range(4):
        np.random.seed(100 + i)
        for k in range(3):
            noise[f"stream_pos_{100 + i}_{k}"] = np.random.uniform(low=-0.01, high=0.01, size=28)
            noise[f"stream_vel_{100 + i}_{k}"] = np.random.uniform(low=-0.01, high=0.01, size=27)
    np.savez(os.path.join(OUT, "reset_noise_golden.npz"), **noise)
    print("wrote", len(cases), "reward cases")


if __name__ == "__main__":
    main()
