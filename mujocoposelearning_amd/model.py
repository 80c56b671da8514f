"""Compiled model handle -- the engine's counterpart of ``mujoco.MjModel``.

``load_model(path)`` replaces ``mujoco.MjModel.from_xml_path`` (reference custom_env.py:53)
and exposes MjModel-style attributes (``nq``, ``nv``, ``nu``, ``body_mass`` ...) read through
the C ABI's ``hs_model_field``.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import HsimError, lib

_INT_FIELDS = {"nq", "nv", "nu", "nbody", "njnt", "ngeom", "ntendon"}
_SHAPES = {"body_pos": 3, "body_quat": 4, "body_ipos": 3, "body_iquat": 4, "body_inertia": 3,
           "body_inertia_full": (3, 3), "body_invweight0": 2, "jnt_pos": 3, "jnt_axis": 3, "jnt_range": 2,
           "jnt_solref": 2, "jnt_solimp": 5, "geom_size": 3, "geom_pos": 3, "geom_quat": 4,
           "geom_friction": 3, "geom_solref": 2, "geom_solimp": 5, "tendon_range": 2, "actuator_ctrlrange": 2,
           "collision_pairs": 2}


# the reference's model (XML/humanoid.xml, loaded at custom_env.py:53 / train_sb3.py:183-186),
# shipped as package data
HUMANOID_XML = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "humanoid.xml")


class HsModel:
    """Immutable compiled model (shareable across batches)."""

    def __init__(self, path):
        L = lib()
        err = C.create_string_buffer(512)
        h = L.hs_model_load(str(path).encode(), err, 512)
        if not h:
            raise HsimError(f"hs_model_load({path}): {err.value.decode()}")
        self._h = h
        self.path = str(path)
        for k in _INT_FIELDS:
            setattr(self, k, int(self.field(k)[0]))

    @property
    def handle(self):
        return self._h

    def field(self, name):
        L = lib()
        n = L.hs_model_field(self._h, name.encode(), None, 0)
        if n < 0:
            raise HsimError(L.hs_last_error().decode())
        out = np.zeros(max(n, 1), np.float64)
        L.hs_model_field(self._h, name.encode(), out.ctypes.data, n)
        out = out[:n]
        shp = _SHAPES.get(name)
        if shp is not None:
            out = out.reshape((-1,) + (shp if isinstance(shp, tuple) else (shp,)))
        return out

    @property
    def opt(self):
        """MjModel.opt subset (generate_trajectories.py:46 reads opt.timestep)."""
        from types import SimpleNamespace
        return SimpleNamespace(timestep=float(self.field("opt_timestep")[0]), gravity=self.field("opt_gravity"))

    def keyframe(self, name):
        return self.field("key_" + name)

    def camera(self, name):
        """MjModel.camera(name) subset (custom_env.py:286 reads ``.id``): MJCF cameras in id order."""
        from .render import parse_cameras
        for c in parse_cameras(self.path):
            if c.name == name:
                return c
        raise KeyError(f"Invalid name '{name}'. Valid names: {[c.name for c in parse_cameras(self.path)]}")

    @property
    def qpos0(self):
        return self.field("qpos0")

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        try:
            return self.field(name)
        except HsimError:
            raise AttributeError(name) from None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                lib().hs_model_free(h)
            except Exception:
                pass
            self._h = None


def load_model(path):
    return HsModel(path)
