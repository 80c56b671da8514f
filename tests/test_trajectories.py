"""Trajectory keyframe XML (generate_trajectories.py:6-72) -- pinned by the reference's own output
file trajectories/humanoid_trajectory.xml (copied as tests/golden/humanoid_trajectory.xml: 4
model keyframes + 'initial_pose' + 150 rollout keys every 5 env steps until the 750-step
truncation, time = step * 0.005)."""
import os
import xml.etree.ElementTree as ET

import numpy as np

from conftest import GOLDEN, XML

TRAJ = os.path.join(GOLDEN, "humanoid_trajectory.xml")


def _keys(path):
    return ET.parse(path).getroot().find("keyframe").findall("key")


def test_reference_trajectory_file_structure_and_plausibility():
    keys = _keys(TRAJ)
    assert [k.get("name") for k in keys[:5]] == ["squat", "stand_on_left_leg", "prone", "supine", "initial_pose"]
    roll = keys[4:]
    assert len(roll) == 151
    times = [float(k.get("time")) for k in roll]
    assert times[0] == 0.0 and times[1] == 0.0
    assert np.allclose(np.diff(times[1:]), 0.025) and times[-1] == 3.725     # 150 keys, steps 0..745
    for k in roll:
        q = np.array(k.get("qpos").split(), float)
        v = np.array(k.get("qvel").split(), float)
        assert q.shape == (28,) and v.shape == (27,)
        assert abs(np.linalg.norm(q[3:7]) - 1) < 1e-5 and -0.5 < q[2] < 2.0
    q0 = np.array(roll[0].get("qpos").split(), float)
    assert abs(q0[2] - 1.282) < 0.002 and np.allclose(q0[3:7], [1, 0, 0, 0], atol=1e-4)   # reset pose


def test_trajectory_xml_compiles_to_the_same_model():
    from mujocoposelearning_amd.model import HsModel
    a, b = HsModel(XML), HsModel(TRAJ)
    for f in ("body_mass", "body_pos", "jnt_range", "jnt_axis", "dof_armature", "geom_size", "actuator_gear",
              "body_invweight0", "dof_invweight0"):
        assert np.array_equal(a.field(f), b.field(f)), f
    assert b.opt.timestep == 0.005
    for k in ("squat", "prone", "supine", "stand_on_left_leg"):
        assert np.array_equal(a.keyframe(k), b.keyframe(k))
    q0 = np.array(_keys(TRAJ)[4].get("qpos").split(), float)
    assert np.allclose(b.keyframe("initial_pose"), q0)


class _FakeEnv:
    """HumanoidEnv-shaped stand-in: truncates at 750 env steps like custom_env.py:201."""

    def __init__(self):
        self.t = 0
        self.data = type("D", (), {})()

    def _sync(self):
        self.data.qpos = np.r_[0, 0, 1.282 + 1e-4 * self.t, 1, 0, 0, 0, np.full(21, 0.001 * self.t)]
        self.data.qvel = np.full(27, -0.002 * self.t)

    def reset(self):
        self.t = 0
        self._sync()
        return np.zeros(352), {}

    def step(self, a):
        assert a.shape == (21,)
        self.t += 1
        self._sync()
        return np.zeros(352), 0.0, False, self.t >= 750, {}


def test_writer_reproduces_reference_layout(tmp_path):
    from mujocoposelearning_amd.trajectories import write_trajectory_xml
    out = write_trajectory_xml(_FakeEnv(), lambda o: np.zeros(21, np.float32), XML, tmp_path / "t" / "traj.xml",
                               num_steps=1000, step_interval=5, timestep=0.005)
    ours, ref = _keys(out), _keys(TRAJ)
    assert [k.get("name") for k in ours] == [k.get("name") for k in ref]
    assert [k.get("time") for k in ours] == [k.get("time") for k in ref]
    k1 = ours[5]
    assert k1.get("qpos").split()[2] == "1.282000" and len(k1.get("qvel").split()) == 27
    assert open(out, "rb").read(38) == b"<?xml version='1.0' encoding='utf-8'?>"
