"""Host sanitizer runs, CPU only -- GPU sanitizer builds are not
available on the MI355X pool.

* The product's MJCF compiler (mjcf.cpp, the replacement of mujoco.MjModel.from_xml_path at
  reference custom_env.py:53) built with -fsanitize=address,undefined behind tools/mjcf_check.cpp
  (compile, read every field, build both device layouts) over the shipped model, <option>
  overrides and malformed inputs: valid models load, malformed ones are rejected with a message,
  and no sanitizer report is raised for any of them.
* The oracle's C restatement (oracle/hsim_oracle.c) built the same way and loaded into a Python
  process with the ASan runtime preloaded, running the oracle physics / env test files plus
  contact-rich lying states.
"""
import os
import re
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT, XML

ASAN = os.path.join(ROOT, "build", "asan")
pytestmark = pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None,
                                reason="needs gcc/g++ with libasan")


@pytest.fixture(scope="module")
def built():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "mujocoposelearning_amd", "csrc"), "asan"])
    return ASAN


def _variants(tmp_path):
    src = open(XML).read()
    cases = {}

    def sub(name, old, new, expect):
        assert old in src, old
        p = tmp_path / f"{name}.xml"
        p.write_text(src.replace(old, new, 1))
        cases[name] = (str(p), expect)

    sub("ok_timestep", '<option timestep="0.005"/>', '<option timestep="0.002"/>', "OK")
    sub("ok_overrides", '<option timestep="0.005"/>',
        '<option timestep="0.004" gravity="0 0 -9" iterations="50" tolerance="1e-10"/>', "OK")
    sub("ok_pgs", '<option timestep="0.005"/>', '<option timestep="0.005" solver="PGS"/>', "OK")
    sub("empty_timestep", '<option timestep="0.005"/>', '<option timestep=""/>', "timestep")
    sub("bad_timestep", '<option timestep="0.005"/>', '<option timestep="-1"/>', "timestep")
    sub("short_gravity", '<option timestep="0.005"/>', '<option gravity="0 0"/>', "gravity")
    sub("text_iterations", '<option timestep="0.005"/>', '<option iterations="abc"/>', "iterations")
    sub("empty_impratio", '<option timestep="0.005"/>', '<option impratio=""/>', "impratio")
    sub("bad_solver", '<option timestep="0.005"/>', '<option solver="CG"/>', "solver")
    sub("short_fromto", 'fromto="0 0 0 0 0 -.3"  size=".049"', 'fromto="0 0 0 0 0"  size=".049"', "fromto")
    sub("short_zaxis", 'zaxis="1 1 1"', 'zaxis="1 1"', "zaxis")
    sub("empty_coef", 'coef=".5"', 'coef=""', "coef")
    sub("exclude_no_body", '<exclude body1="waist_lower" body2="thigh_right"/>', '<exclude body2="thigh_right"/>',
        "exclude")
    sub("key_short", '<key name="squat"', '<key name="bad" qpos="0 0 1"/>\n    <key name="squat"', "key qpos")
    sub("truncated", src[len(src) // 2:], "", "parse")
    (tmp_path / "empty.xml").write_text("")
    cases["empty"] = (str(tmp_path / "empty.xml"), "ERR")
    (tmp_path / "garbage.xml").write_bytes(bytes(range(256)) * 4)
    cases["garbage"] = (str(tmp_path / "garbage.xml"), "ERR")
    return cases


def test_mjcf_compiler_under_asan_ubsan(built, tmp_path):
    cases = _variants(tmp_path)
    paths = [XML] + [p for p, _ in cases.values()]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(built, "mjcf_check"), *paths], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    lines = r.stdout.splitlines()
    assert len(lines) == len(paths)
    assert lines[0] == "OK 28 27 21 159"
    for (name, (_, expect)), line in zip(cases.items(), lines[1:]):
        if expect == "OK":
            assert line.startswith("OK 28 27 21"), (name, line)
        else:
            assert line.startswith("ERR"), (name, line)
            if expect != "ERR":
                assert re.search(expect, line, re.I), (name, line)


_ORACLE_SCRIPT = r"""
import sys
import numpy as np
sys.path.insert(0, {root!r})
import oracle.oracle as oo
from oracle.oracle import Oracle
o = Oracle({xml!r})
assert oo.lib()._name == {lib!r}, oo.lib()._name
sys.path.insert(0, {tests!r})
from test_gpu_contacts import lying_states
qs = lying_states(o, 6, seed=1)
rng = np.random.default_rng(0)
for q in qs:                       # contact-rich states (> 32 contacts) through 200 substeps
    o.reset_data()
    o.qpos[:] = q
    o.step(rng.uniform(-1, 1, 21), 200)
    assert np.isfinite(o.qpos).all()
print("oracle-asan-ok")
"""


def test_oracle_restatement_under_asan_ubsan(built):
    lib = os.path.join(built, "libhsim_oracle.so")
    env = dict(os.environ, HSIM_ORACLE_LIB=lib, LD_PRELOAD=subprocess.check_output(
        ["gcc", "-print-file-name=libasan.so"], text=True).strip(),
        ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    tests = os.path.join(ROOT, "tests")
    r = subprocess.run([sys.executable, "-c", _ORACLE_SCRIPT.format(root=ROOT, xml=XML, lib=lib, tests=tests)],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0 and "oracle-asan-ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
                        os.path.join(tests, "test_oracle_physics.py"), os.path.join(tests, "test_env_semantics.py")],
                       capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
