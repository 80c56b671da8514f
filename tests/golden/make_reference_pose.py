"""Extract the reference's one recorded MuJoCo state into a fixture (data only).

Source: /root/reference/trajectories/humanoid_trajectory.xml, <key name="initial_pose">, written by
generate_trajectories.py:30-41 right after HumanoidEnv.reset() (custom_env.py:97-121), i.e. the state
after mj_resetData, qpos = init + U(+-0.01) noise (z x0.1, no quaternion noise), qvel = U(+-0.01) noise
and ONE mujoco.mj_step with ctrl = 0, printed with 6 decimals by MuJoCo 3.2.5 itself.
Run: python tests/golden/make_reference_pose.py  ->  tests/golden/reference_initial_pose.json
"""
import json
import os
import xml.etree.ElementTree as ET

SRC = "/root/reference/trajectories/humanoid_trajectory.xml"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_initial_pose.json")

if __name__ == "__main__":
    key = next(k for k in ET.parse(SRC).getroot().iter("key") if k.get("name") == "initial_pose")
    out = {"source": "trajectories/humanoid_trajectory.xml <key name=initial_pose> (generate_trajectories.py:30-41)",
           "time": key.get("time"),
           "qpos": [float(x) for x in key.get("qpos").split()],
           "qvel": [float(x) for x in key.get("qvel").split()]}
    json.dump(out, open(OUT, "w"), indent=1)
    print(f"wrote {OUT}: nq={len(out['qpos'])} nv={len(out['qvel'])}")
