"""ORACLE (test infrastructure only): the fp64 restatement with chosen stages computed in fp32.

``hsim_oracle.c`` is compiled a third time as C++ with ``oracle/precemu.h`` force-included: every
arithmetic result of a stage whose bit is set in ``mask`` is rounded to float (the correctly rounded
fp32 result), the other stages stay fp64.  With every bit set and the model and state rounded to
float this is an fp32 engine in the oracle's own operation order; clearing one stage's bit shows how
much of the fp32 engine's trajectory divergence that stage's rounding causes.  Stage
bits are the ORC_STAGE ids of hsim_oracle.c (``STAGES``).  Never used by the product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from .oracle import Oracle, OrcData, OrcModel

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libhsim_oracle_precemu.so")
STAGES = ["kinematics", "com_pos", "tendon", "crb", "collision", "make_constraint", "com_vel", "passive",
          "reference_constraint", "rne", "actuation", "smooth", "solver", "euler", "other",
          "solver_hessian", "solver_cholesky", "solver_linesearch"]
ALL = (1 << len(STAGES)) - 1
_LIB = None


def build(force=False):
    src = os.path.join(HERE, "hsim_oracle.c")
    hdr = os.path.join(HERE, "precemu.h")
    newest = max(os.path.getmtime(src), os.path.getmtime(hdr))
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < newest:
        os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
        tmp = f"{LIB_PATH}.{os.getpid()}.tmp"
        subprocess.check_call(["g++", "-x", "c++", "-std=c++17", "-O2", "-fPIC", "-shared", "-include", hdr, src,
                               "-o", tmp])
        os.replace(tmp, LIB_PATH)
    return LIB_PATH


def lib():
    global _LIB
    if _LIB is None:
        L = C.CDLL(build())
        for fn in ("orc_reset_data", "orc_forward", "orc_step"):
            getattr(L, fn).argtypes = [C.c_void_p, C.c_void_p]
            getattr(L, fn).restype = None
        L.orc_step_n_full.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        L.orc_step_n_full.restype = None
        assert L.orc_sizeof_model() == C.sizeof(OrcModel) and L.orc_sizeof_data() == C.sizeof(OrcData)
        _LIB = L
    return _LIB


def set_mask(mask):
    C.c_uint.in_dll(lib(), "orc_prec_mask").value = int(mask) & 0xFFFFFFFF


def mask_of(fp32_stages):
    m = 0
    for s in fp32_stages:
        m |= 1 << STAGES.index(s)
    return m


def round_model(M):
    """The model data an fp32 engine holds (DevModel<float>): every float field rounded."""
    out = {}
    for k, v in M.items():
        a = np.asarray(v) if not isinstance(v, dict) else v
        out[k] = a.astype(np.float32).astype(np.float64) if isinstance(a, np.ndarray) and a.dtype == np.float64 else v
        if isinstance(v, float):
            out[k] = float(np.float32(v))
    return out


class PrecOracle(Oracle):
    """An Oracle stepped by the precision-emulating build (call set_mask before stepping)."""

    def __init__(self, model_path=None, M=None):
        super().__init__(model_path, M)
        self.lib = lib()
        self.reset_data()
