"""Render path (custom_env.py:273-321, train_sb3.py:41-61): camera parsing, ray-primitive
intersections and a full frame, on CPU.  The poses come from the fp64 oracle here (the product
gets them from the GPU kinematics; tests/test_gpu_render.py checks those against the oracle).
Frames have no reference pixels to match (MuJoCo's OpenGL renderer is not in the image), so the
checks are geometric: what must be sky, floor or body from the camera's projection."""
import math
import os
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import XML


def _pose(o):
    gm = o.get("geom_xmat").reshape(-1, 3, 3)
    return {"xpos": o.get("xpos"), "xmat": o.get("xmat"), "geom_xpos": o.get("geom_xpos"),
            "geom_zaxis": gm[:, :, 2].copy(), "com": o.get("subtree_com")[0].copy()}


class _OracleBatch:
    """Stands in for HsBatch.kinematics with the oracle's mj_kinematics/mj_comPos."""

    def __init__(self):
        from oracle.oracle import Oracle
        self.o = Oracle(XML)

    def kinematics(self, env=0, qpos=None):
        keep = self.o.qpos.copy()
        if qpos is not None:
            self.o.qpos[:] = qpos
        self.o.forward()
        out = _pose(self.o)
        self.o.qpos[:] = keep
        self.o.forward()
        return out


def _data(batch):
    return SimpleNamespace(_env=SimpleNamespace(_batch=batch, _idx=0))


@pytest.fixture(scope="module")
def model():
    from mujocoposelearning_amd.model import HsModel
    return HsModel(XML)


def test_cameras_parsed_in_mujoco_order():
    from mujocoposelearning_amd.render import parse_cameras
    cams = parse_cameras(XML)
    assert [c.name for c in cams] == ["back", "side", "egocentric"]
    side = cams[1]
    assert side.id == 1 and side.body == 1 and side.mode == "trackcom" and side.fovy == 45.0
    # xyaxes "1 0 0 0 1 2": looks along -z = (0, 2, -1)/sqrt(5)
    np.testing.assert_allclose(-side.rot[:, 2], np.array([0, 2, -1]) / math.sqrt(5), atol=1e-12)
    assert cams[2].body == 2 and cams[2].mode == "fixed" and cams[2].fovy == 80.0


def test_model_camera_lookup(model):
    assert model.camera("side").id == 1
    with pytest.raises(KeyError):
        model.camera("nope")


def test_ray_primitives():
    from mujocoposelearning_amd.render import _capsule_hit, _sphere_hit
    o = np.array([0.0, -5.0, 0.0])
    d = np.array([[0, 1, 0], [0, 1, 0], [0, 1, 0], [1, 0, 0]], float)
    d[1] = [0, 5, 0.95]        # aims at the upper cap region
    d[1] /= np.linalg.norm(d[1])
    # capsule along z from -1 to 1, radius 0.5 at the origin
    t = _capsule_hit(o, d, np.array([0, 0, -1.0]), np.array([0, 0, 1.0]), 0.5)
    assert t[0] == pytest.approx(4.5)
    assert np.isfinite(t[1]) and t[1] > 4.5
    assert np.isinf(t[3])
    p = o + t[1] * d[1]
    q = np.array([0, 0, np.clip(p[2], -1, 1)])
    assert np.linalg.norm(p - q) == pytest.approx(0.5, abs=1e-9)
    ts = _sphere_hit(o, d[[0, 3]], np.zeros(3), 1.0)
    assert ts[0] == pytest.approx(4.0) and np.isinf(ts[1])


def test_side_camera_frame(model):
    from mujocoposelearning_amd.render import BODY_RGB, Renderer
    b = _OracleBatch()
    q = model.qpos0.copy()
    b.o.qpos[:] = q
    r = Renderer(model, height=120, width=160)
    r.update_scene(_data(b), camera=model.camera("side").id)
    pose, (cpos, R, fovy) = r._scene
    # trackcom at qpos0: camera = torso frame (identity) + (0, -3, 1)
    np.testing.assert_allclose(cpos, pose["xpos"][1] + [0, -3, 1], atol=1e-9)
    img = r.render()
    assert img.shape == (120, 160, 3) and img.dtype == np.uint8
    # top row looks up at the sky (blue-ish gradient), bottom row down at the floor
    assert img[0, :, 2].mean() > img[0, :, 0].mean()
    assert img[-1].std() > 0 or img[-1].mean() > 0
    # the torso's projection is body-coloured (red > blue), the corners are not
    f = 0.5 * 120 / math.tan(math.radians(fovy) / 2)
    pc = R.T @ (pose["geom_xpos"][0] - cpos)
    u, v = int(80 + f * pc[0] / -pc[2]), int(60 - f * pc[1] / -pc[2])
    px = img[v, u].astype(float)
    assert px[0] > px[2] + 20, px
    assert abs(px[0] / px[1] - BODY_RGB[0] / BODY_RGB[1]) < 0.1
    assert img[0, 0, 0] < img[0, 0, 2]


def test_write_video_gif(tmp_path):
    from PIL import Image

    from mujocoposelearning_amd.render import write_video
    frames = [np.full((8, 10, 3), k * 20, np.uint8) for k in range(5)]
    p = write_video(str(tmp_path / "v.gif"), frames, fps=60)
    im = Image.open(p)
    assert im.n_frames == 5 and im.size == (10, 8)
    assert os.path.getsize(p) > 0
