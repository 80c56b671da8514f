"""Diagnostic: per-state PGS kernel vs oracle PGS (qacc error, rows, sweeps) for fp32 and fp64."""
import os
import sys
import tempfile
import pathlib

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
from test_gpu_pgs import _pgs_xml, _contact_states, _gpu_one_substep, _oracle_one_substep  # noqa: E402
from mujocoposelearning_amd.model import HsModel  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

tmp = pathlib.Path(tempfile.mkdtemp())
for prec, it, tol in (("fp32", 100, 1e-8), ("fp64", 100, 1e-8)):
    xml = _pgs_xml(tmp, it, tol)
    m, o = HsModel(xml), Oracle(xml)
    states = _contact_states(o.M, 24, seed=11)
    st, aux = _gpu_one_substep(m, states, prec)
    for i, (q, v, c) in enumerate(states):
        rq, rv, ra, nefc, nit = _oracle_one_substep(o, q, v, c)
        err = np.abs(aux[i, :27] - ra).max() / (1 + np.abs(ra).max())
        print(f"{prec} it={it} state {i:2d}: rows {nefc:3d}/{int(aux[i, 36]):3d} sweeps oracle {nit:4d} kernel "
              f"{int(aux[i, 37]):4d}  rel qacc err {err:.2e}", flush=True)
