import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# the parity-report helpers the long-horizon parity tests share (tools/probes/parity_report.py)
PROBES = os.path.join(ROOT, "tools", "probes")
if PROBES not in sys.path:
    sys.path.append(PROBES)

XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer-running test")


@pytest.fixture(scope="session")
def xml_path():
    return XML


@pytest.fixture(scope="session")
def oracle_model():
    from oracle.model import compile_mjcf
    return compile_mjcf(XML)
