"""Renderer -- the engine's stand-in for ``mujoco.Renderer`` on the reference's video path.

The reference renders from the ``side`` camera into 480x640 frames (custom_env.py:273-289) and
writes them with ``mediapy.write_video`` (custom_env.py:291-321), driven by the video callback
(train_sb3.py:41-61).  MuJoCo's OpenGL renderer, mediapy and ffmpeg are not in this image, so
this module draws the same scene on the host by ray casting:

* the poses come from the GPU kinematics of the env being drawn (``hs_kinematics`` in the C ABI,
  one single-wave launch per frame; nothing here steps physics);
* geoms: the plane floor (checker ``grid`` material, 0.5 m squares), capsules and spheres in the
  ``body`` material colour, lit by a headlight plus the ``top`` light above the COM;
* cameras are read from the MJCF (``pos``, ``xyaxes``/``quat``, ``fovy``, ``mode``), with
  MuJoCo's ``fixed`` and ``trackcom`` semantics (trackcom: the qpos0 offset from the root
  subtree COM and the qpos0 world orientation, mj_camlight);
* the sky is the model's gradient skybox colours.

It is off the step path and is not pixel-identical to MuJoCo's renderer (lighting model,
no shadows/reflections/haze): parity for frames is unpinned by construction.
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from types import SimpleNamespace

import numpy as np

PLANE, SPHERE, CAPSULE = 0, 2, 3          # mjtGeom codes used by the compiler
BODY_RGB = np.array([0.8, 0.6, 0.4])      # humanoid.xml:30 material "body"
FLOOR_RGB = (np.array([0.1, 0.2, 0.3]), np.array([0.2, 0.3, 0.4]))   # humanoid.xml:31 checker
SKY_TOP, SKY_BOTTOM = np.array([0.3, 0.5, 0.7]), np.zeros(3)         # humanoid.xml:28 gradient


def _vec(text, n, default):
    if text is None:
        return np.array(default, float)
    v = np.array([float(x) for x in text.split()], float)
    if v.size != n:
        raise ValueError(f"expected {n} numbers, got {text!r}")
    return v


def _quat2mat(q):
    w, x, y, z = np.asarray(q, float) / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _cam_rot(el):
    """Camera frame (columns x, y, z; the camera looks along -z) from xyaxes or quat."""
    if el.get("xyaxes") is not None:
        v = _vec(el.get("xyaxes"), 6, None)
        x = v[:3] / np.linalg.norm(v[:3])
        y = v[3:] - x * (x @ v[3:])
        y /= np.linalg.norm(y)
        return np.stack([x, y, np.cross(x, y)], axis=1)
    return _quat2mat(_vec(el.get("quat"), 4, (1, 0, 0, 0)))


def parse_cameras(xml_path):
    """MJCF <camera> elements in document order (MuJoCo camera ids): name, body id (MuJoCo body
    order = <body> document order, world = 0), local pos / rotation, fovy, mode."""
    root = ET.parse(xml_path).getroot()
    cams, counter = [], [0]

    def walk(el, body_id):
        for ch in el:
            if ch.tag == "body":
                counter[0] += 1
                walk(ch, counter[0])
            elif ch.tag == "camera":
                cams.append(SimpleNamespace(id=len(cams), name=ch.get("name"), body=body_id,
                                            pos=_vec(ch.get("pos"), 3, (0, 0, 0)), rot=_cam_rot(ch),
                                            fovy=float(ch.get("fovy", 45.0)), mode=ch.get("mode", "fixed")))
    wb = root.find("worldbody")
    if wb is not None:
        walk(wb, 0)
    return cams


def _capsule_hit(o, d, a, b, r):
    """Nearest t >= 0 of rays o + t d against the capsule (segment a-b, radius r); inf = miss."""
    ba = b - a
    oa = o - a
    baba = ba @ ba
    bard = d @ ba
    baoa = oa @ ba
    rdoa = np.einsum("ij,ij->i", d, oa) if oa.ndim == 2 else d @ oa
    oaoa = np.einsum("ij,ij->i", oa, oa) if oa.ndim == 2 else oa @ oa
    k2 = baba - bard * bard
    k1 = baba * rdoa - baoa * bard
    k0 = baba * oaoa - baoa * baoa - r * r * baba
    h = k1 * k1 - k2 * k0
    t = np.full(d.shape[0], np.inf)
    ok = h >= 0
    with np.errstate(invalid="ignore", divide="ignore"):
        tc = (-k1 - np.sqrt(np.where(ok, h, 0))) / k2
        y = baoa + tc * bard
        body = ok & (y > 0) & (y < baba) & (tc > 0)
        t = np.where(body, tc, t)
        # end caps: the sphere at whichever end the cylinder test fell past
        oc = np.where((y <= 0)[:, None], oa, o - b)
        bb = np.einsum("ij,ij->i", d, oc)
        cc = np.einsum("ij,ij->i", oc, oc) - r * r
        hh = bb * bb - cc
        tcap = -bb - np.sqrt(np.where(hh > 0, hh, 0))
        cap = ok & ~body & (hh > 0) & (tcap > 0)
    return np.where(cap, tcap, t)


def _sphere_hit(o, d, c, r):
    oc = o - c
    b = d @ oc
    cc = oc @ oc - r * r
    h = b * b - cc
    with np.errstate(invalid="ignore"):
        t = -b - np.sqrt(np.where(h > 0, h, 0))
    return np.where((h > 0) & (t > 0), t, np.inf)


class Renderer:
    """mujoco.Renderer(model, height, width) surface: update_scene(data, camera), render(), close()."""

    def __init__(self, model, height=240, width=320):
        self.model = model
        self.height, self.width = int(height), int(width)
        self.cameras = parse_cameras(model.path)
        self._gtype = np.asarray(model.geom_type, int)
        self._gsize = np.asarray(model.geom_size, float)
        self._scene = None
        self._cam0 = {}

    # -- camera -----------------------------------------------------------------------------
    def _resolve(self, camera):
        if camera is None or camera == -1:
            return None
        if isinstance(camera, str):
            for c in self.cameras:
                if c.name == camera:
                    return c
            raise ValueError(f"camera {camera!r} not found in {self.model.path}")
        return self.cameras[int(camera)]

    def _camera_pose(self, cam, batch, env, pose):
        if cam is None:   # free camera: <visual><global> azimuth 120, elevation -20 around the COM
            az, el = math.radians(120.0), math.radians(-20.0)
            fwd = np.array([math.cos(el) * math.cos(az), math.cos(el) * math.sin(az), math.sin(el)])
            z = -fwd
            x = np.cross(np.array([0.0, 0.0, 1.0]), z)
            x /= np.linalg.norm(x)
            return pose["com"] - 3.0 * fwd, np.stack([x, np.cross(z, x), z], axis=1), 45.0
        bx, bR = pose["xpos"][cam.body], pose["xmat"][cam.body].reshape(3, 3)
        if cam.mode == "trackcom":
            if cam.id not in self._cam0:   # cam_pos0 / cam_mat0: offsets at qpos0 (mj_setConst)
                p0 = batch.kinematics(env, qpos=self.model.qpos0)
                R0 = p0["xmat"][cam.body].reshape(3, 3)
                self._cam0[cam.id] = (p0["xpos"][cam.body] + R0 @ cam.pos - p0["com"], R0 @ cam.rot)
            off, R = self._cam0[cam.id]
            return pose["com"] + off, R, cam.fovy
        return bx + bR @ cam.pos, bR @ cam.rot, cam.fovy

    def update_scene(self, data, camera=None):
        """``data``: an env's data view (HsData).  ``camera``: id, name or None (free camera)."""
        env = data._env
        batch, idx = env._batch, env._idx
        pose = batch.kinematics(idx)
        self._scene = (pose, self._camera_pose(self._resolve(camera), batch, idx, pose))

    # -- drawing ----------------------------------------------------------------------------
    def render(self):
        if self._scene is None:
            raise RuntimeError("update_scene() first")
        pose, (cpos, R, fovy) = self._scene
        H, W = self.height, self.width
        f = 0.5 * H / math.tan(math.radians(fovy) / 2)
        key = (R.tobytes(), fovy)
        if getattr(self, "_rays_key", None) != key:   # trackcom / free cameras keep their orientation
            u = (np.arange(W) + 0.5 - 0.5 * W) / f
            v = (0.5 * H - np.arange(H) - 0.5) / f
            uu, vv = np.meshgrid(u, v)
            d = uu[..., None] * R[:, 0] + vv[..., None] * R[:, 1] - R[:, 2]
            self._rays = (d / np.linalg.norm(d, axis=-1, keepdims=True)).reshape(-1, 3)
            self._sky = SKY_BOTTOM + (0.5 * (self._rays[:, 2:3] + 1)) * (SKY_TOP - SKY_BOTTOM)
            self._rays_key = key
        d = self._rays
        n_pix = d.shape[0]
        tbest = np.full(n_pix, np.inf)
        gid = np.full(n_pix, -1)
        gpos, gax = pose["geom_xpos"], pose["geom_zaxis"]
        for g, typ in enumerate(self._gtype):
            if typ == PLANE:
                nrm = gax[g]
                den = d @ nrm
                with np.errstate(divide="ignore", invalid="ignore"):
                    t = ((gpos[g] - cpos) @ nrm) / den
                t = np.where((den < 0) & (t > 0), t, np.inf)
                sel = slice(None)
            else:
                r = self._gsize[g, 0]
                hl = self._gsize[g, 1] if typ == CAPSULE else 0.0
                sel = self._footprint(gpos[g], r + hl, cpos, R, f)
                if sel is None:
                    continue
                if typ == CAPSULE:
                    t = _capsule_hit(cpos, d[sel], gpos[g] - hl * gax[g], gpos[g] + hl * gax[g], r)
                elif typ == SPHERE:
                    t = _sphere_hit(cpos, d[sel], gpos[g], r)
                else:
                    continue
            closer = t < tbest[sel]
            tb = tbest[sel]
            gb = gid[sel]
            tb[closer] = t[closer]
            gb[closer] = g
            tbest[sel] = tb
            gid[sel] = gb
        img = self._shade(d, tbest, gid, cpos, pose)
        return (np.clip(img, 0, 1) * 255 + 0.5).astype(np.uint8).reshape(H, W, 3)

    def _footprint(self, c, rad, cpos, R, f):
        """Flat pixel indices that a bounding sphere can cover (None: off screen)."""
        H, W = self.height, self.width
        pc = R.T @ (c - cpos)
        depth = -pc[2]
        if depth <= rad + 1e-3:   # camera inside / behind: test everything
            return np.arange(H * W) if depth > -rad else None
        cu = 0.5 * W + f * pc[0] / depth
        cv = 0.5 * H - f * pc[1] / depth
        sr = f * rad / math.sqrt(depth * depth - rad * rad) + 2
        u0, u1 = max(int(cu - sr), 0), min(int(cu + sr) + 1, W)
        v0, v1 = max(int(cv - sr), 0), min(int(cv + sr) + 1, H)
        if u0 >= u1 or v0 >= v1:
            return None
        vs, us = np.mgrid[v0:v1, u0:u1]
        return (vs * W + us).ravel()

    def _shade(self, d, t, gid, cpos, pose):
        img = self._sky.copy()
        hit = np.isfinite(t)
        if not hit.any():
            return img
        p = cpos + t[hit, None] * d[hit]
        g = gid[hit]
        gpos, gax = pose["geom_xpos"], pose["geom_zaxis"]
        nrm = np.empty_like(p)
        col = np.empty_like(p)
        typ = self._gtype[g]
        fl = typ == PLANE
        if fl.any():
            nrm[fl] = gax[g[fl]]
            chk = (np.floor(p[fl, 0] / 0.5) + np.floor(p[fl, 1] / 0.5)).astype(int) & 1
            col[fl] = np.where(chk[:, None] == 0, FLOOR_RGB[0], FLOOR_RGB[1])
        bd = ~fl
        if bd.any():
            gb = g[bd]
            hl = np.where(self._gtype[gb] == CAPSULE, self._gsize[gb, 1], 0.0)
            a = gpos[gb] - hl[:, None] * gax[gb]
            s = np.clip(np.einsum("ij,ij->i", p[bd] - a, gax[gb]), 0, 2 * hl)
            q = a + s[:, None] * gax[gb]
            nn = p[bd] - q
            nrm[bd] = nn / np.maximum(np.linalg.norm(nn, axis=1, keepdims=True), 1e-12)
            col[bd] = BODY_RGB
        head = np.clip(-np.einsum("ij,ij->i", nrm, d[hit]), 0, 1)
        light = pose["com"] + np.array([0.0, 0.0, 2.0])      # humanoid.xml:107 "top", trackcom
        ld = light - p
        ld /= np.linalg.norm(ld, axis=1, keepdims=True)
        top = np.clip(np.einsum("ij,ij->i", nrm, ld), 0, 1)
        img[hit] = col * (0.35 + 0.45 * head + 0.35 * top)[:, None]
        return img

    def close(self):
        self._scene = None


def write_video(path, frames, fps):
    """mediapy.write_video stand-in: an animated GIF (no mp4/h264 encoder in this image)."""
    from PIL import Image
    imgs = [Image.fromarray(np.asarray(f, np.uint8)) for f in frames]
    imgs[0].save(path, save_all=True, append_images=imgs[1:], duration=max(int(round(1000.0 / fps)), 10), loop=0)
    return path
