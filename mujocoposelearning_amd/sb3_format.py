"""SB3 2.3.2 checkpoint zip format for the on-device PPO (reference: ``model.save`` at
train_sb3.py:234 and ``PPO.load`` at render_policy.py:8).

SB3's ``BaseAlgorithm.save`` writes a zip with:
  data                     JSON of the algorithm's attributes (objects SB3 cannot JSON-encode are
                           cloudpickled under ":serialized:" keys)
  policy.pth               torch.save(policy.state_dict())
  policy.optimizer.pth     torch.save(optimizer.state_dict())
  pytorch_variables.pth    torch.save({})  (PPO has none)
  _stable_baselines3_version, system_info.txt

This module writes that layout with the ``MlpPolicy`` parameter names of an ``ActorCriticPolicy``
(``mlp_extractor.policy_net.{0,2}``, ``mlp_extractor.value_net.{0,2}``, ``action_net``,
``value_net``, ``log_std``) and an ``Adam`` state whose parameter order matches SB3's
(``log_std`` first, then the sub-modules in registration order).  So:

* SB3 side: ``PPO("MlpPolicy", env, policy_kwargs=...).set_parameters("model.zip")`` loads the
  weights and optimizer state (set_parameters reads only policy.pth / policy.optimizer.pth; the
  "data" entry carries the plain hyper-parameters but no cloudpickled spaces -- nothing is
  pickled here, so ``PPO.load`` of the full object needs SB3's own save).
* hsim side: ``load_sb3_zip`` reads policy.pth (and the optimizer) of an SB3-saved zip with
  ``torch.load(weights_only=True)`` -- nothing in the file is executed.

SB3 is not installed in this image: the layout is restated from SB3 2.3.2's save_util.py and
policies.py (parity unpinned against a real SB3 zip; tests pin the names, shapes and order).
"""
from __future__ import annotations

import io
import json
import platform
import zipfile

import torch

SB3_VERSION = "2.3.2"
_PREFIX = (("pi_net.", "mlp_extractor.policy_net."), ("vf_net.", "mlp_extractor.value_net."))


def to_sb3_names(state_dict):
    out = {}
    for k, v in state_dict.items():
        for ours, theirs in _PREFIX:
            if k.startswith(ours):
                k = theirs + k[len(ours):]
                break
        out[k] = v
    return out


def from_sb3_names(state_dict):
    out = {}
    for k, v in state_dict.items():
        for ours, theirs in _PREFIX:
            if k.startswith(theirs):
                k = ours + k[len(theirs):]
                break
        out[k] = v
    return out


def _torch_bytes(obj):
    buf = io.BytesIO()
    torch.save(obj, buf)
    return buf.getvalue()


def save_sb3_zip(path, policy, optimizer=None, data=None):
    """Write ``path`` (".zip" appended if missing, as SB3 does) in SB3's checkpoint layout."""
    path = str(path)
    if not path.endswith(".zip"):
        path += ".zip"
    sd = {k: v.detach().cpu() for k, v in to_sb3_names(policy.state_dict()).items()}
    with zipfile.ZipFile(path, "w") as z:
        z.writestr("data", json.dumps(data or {}, indent=4, default=str))
        z.writestr("policy.pth", _torch_bytes(sd))
        if optimizer is not None:
            z.writestr("policy.optimizer.pth", _torch_bytes(optimizer.state_dict()))
        z.writestr("pytorch_variables.pth", _torch_bytes({}))
        z.writestr("_stable_baselines3_version", SB3_VERSION)
        z.writestr("system_info.txt", f"- OS: {platform.platform()}\n- Python: {platform.python_version()}\n"
                                      f"- PyTorch: {torch.__version__}\n- Stable-Baselines3: {SB3_VERSION}"
                                      f" (format written by mujocoposelearning_amd)\n")
    return path


def load_sb3_zip(path, policy, optimizer=None, map_location="cpu"):
    """Load policy (and optimizer) state from an SB3-layout zip; returns the parsed "data" dict
    (its ":serialized:" entries, if any, are left undecoded -- they are never unpickled)."""
    path = str(path)
    if not path.endswith(".zip") and not zipfile.is_zipfile(path):
        path += ".zip"
    with zipfile.ZipFile(path) as z:
        names = set(z.namelist())
        if "policy.pth" not in names:
            raise ValueError(f"{path}: no policy.pth entry (not an SB3 checkpoint)")
        sd = torch.load(io.BytesIO(z.read("policy.pth")), map_location=map_location, weights_only=True)
        policy.load_state_dict(from_sb3_names(sd))
        if optimizer is not None and "policy.optimizer.pth" in names:
            opt = torch.load(io.BytesIO(z.read("policy.optimizer.pth")), map_location=map_location, weights_only=True)
            optimizer.load_state_dict(opt)
        data = json.loads(z.read("data")) if "data" in names else {}
    return data
