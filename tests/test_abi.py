"""The C-ABI library loads and exports every entry point include/hsim.h declares (CPU only:
no compute calls), and misuse fails loudly with a message."""
import ctypes as C
import os
import re

import pytest

from conftest import ROOT, XML

HEADER = os.path.join(ROOT, "include", "hsim.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hs_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from mujocoposelearning_amd import _lib
    L = _lib.lib()
    names = declared_functions()
    assert len(names) >= 18
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_lib.EXPORTED)


def test_version_and_errors():
    from mujocoposelearning_amd import _lib
    L = _lib.lib()
    assert b"gfx950" in L.hs_version()
    err = C.create_string_buffer(256)
    assert not L.hs_model_load(b"/nonexistent.xml", err, 256)
    assert b"cannot open" in err.value
    assert L.hs_set_config(None, None) < 0 and b"null" in L.hs_last_error()
    assert L.hs_step(None, None, None) < 0


def test_model_fields_through_abi():
    from mujocoposelearning_amd.model import HsModel
    m = HsModel(XML)
    assert (m.nq, m.nv, m.nu, m.nbody) == (28, 27, 21, 17)
    assert m.field("body_mass").sum() == pytest.approx(40.84402122162132)
    with pytest.raises(Exception, match="unknown model field"):
        m.field("no_such_field")


def test_batch_create_without_gpu_fails_loudly():
    """No silent CPU fallback: creating a batch without a GPU raises."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from mujocoposelearning_amd.batch import HsBatch
    from mujocoposelearning_amd.model import HsModel
    with pytest.raises(RuntimeError, match="GPU"):
        HsBatch(HsModel(XML), 4)


def test_config_struct_layout():
    """The ctypes mirrors follow include/hsim.h field by field (names, order, pointer size)."""
    import os
    import re
    from mujocoposelearning_amd import _lib
    assert C.sizeof(_lib.hs_env_config) == 6 * 4 + 3 * 8 + 9 * 8 + 8      # + schedule (padded)
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "hsim.h")).read()
    body = re.search(r"typedef struct \{(.*?)\} hs_buffers;", hdr, re.S).group(1)
    names = re.findall(r"\*\s*(\w+);", body)
    assert [n for n, _ in _lib.hs_buffers._fields_] == names
    assert C.sizeof(_lib.hs_buffers) == len(names) * 8
    assert _lib.HS_FULL_STATE == int(re.search(r"HS_FULL_STATE = (0x[0-9a-fA-F]+)", hdr).group(1), 16)


def test_trainer_entry_points_validate_arguments():
    """The PPO kernels' entry points reject bad sizes / null buffers with a message before touching
    the device (runs on the CPU: nothing is launched), and report their workspace sizes."""
    from mujocoposelearning_amd import _lib
    L = _lib.lib()

    def err(rc):
        assert rc < 0
        return L.hs_last_error().decode()

    assert "A <= 32" in err(L.hs_ppo_act(None, 40, None, 1, None, None, 0, 0, None, 0, None, None, None, None, None,
                                         8, 33, None))
    assert "null" in err(L.hs_ppo_post(None, None, None, None, None, None, None, 0, 0.9, None, None, 0, None, None,
                                       None, None, None, 4, None))
    assert "null" in err(L.hs_ppo_loss(None, None, None, None, None, None, 8, 0.2, 1, None, None, None, None))
    assert "null" in err(L.hs_ppo_loss_grad(None, None, 8, 0.2, None, None, None, None, None, None))
    assert "nt" in err(L.hs_adam_clip(17, None, None, None, None, None, None, None, 0.5, 3e-4, 0.9, 0.999, 1e-5,
                                      None))
    assert "null" in err(L.hs_colsum(None, 4, 4, None, None, None, None))
    assert "null" in err(L.hs_relu_grad_colsum(None, None, 4, 4, None, None, None))
    assert "null" in err(L.hs_colsum_pair(None, 4, 4, None, None, 4, 4, None, None))
    assert "negative" in err(L.hs_gae(None, None, None, None, None, None, None, -1, 4, 0.99, 0.95, None))
    # outputs overlapping inputs are rejected (the long-rollout path keeps its carries in the outputs);
    # fake, never-dereferenced addresses: [T][N] = 4 x 8 floats = 128 B each
    gae = lambda r, v, s, lv, ld, a, ret: L.hs_gae(r, v, s, lv, ld, a, ret, 4, 8, 0.99, 0.95, None)  # noqa: E731
    base = 1 << 20
    r, v, s, lv, ld = base, base + 128, base + 256, base + 384, base + 416
    assert "overlaps an input" in err(gae(r, v, s, lv, ld, v + 64, base + 4096))
    assert "advantages and returns overlap" in err(gae(r, v, s, lv, ld, base + 4096, base + 4096 + 64))
    assert "last_values" in err(gae(r, v, s, lv, ld, base + 4096, lv + 16))
    # the fused policy forward: nn.Linear layouts (ld1 >= D, ld2 / ld3 >= 256), A <= 32, D <= 512
    mlp = lambda D, N, ld1, ld2, ld3, A: L.hs_mlp2_forward(None, D, D, N, None, ld1, None, None, ld2, None,  # noqa: E731
                                                           None, ld3, None, A, None, A, None)
    assert "ld1 >= D" in err(mlp(352, 8, 256, 256, 256, 21))
    assert "A <= 32" in err(mlp(352, 8, 352, 256, 256, 33))
    assert "D <= 512" in err(mlp(600, 8, 600, 256, 256, 21))
    assert "null" in err(mlp(352, 8, 352, 256, 256, 21))
    assert mlp(352, 0, 352, 256, 256, 21) == 0
    dg = lambda G, ldg, K, W, ldw, X, ldx, B, N: L.hs_dgrad_mask(G, ldg, K, W, ldw, X, ldx, B, N, X, W,  # noqa: E731
                                                                 None, None)
    assert "N == 256" in err(dg(None, 21, 21, None, 256, None, 256, 8, 128))
    assert "K % 16" in err(dg(None, 40, 40, None, 256, None, 256, 8, 256))
    assert "ldx >= N" in err(dg(None, 21, 21, None, 256, None, 100, 8, 256))
    assert "null" in err(dg(None, 21, 21, None, 256, None, 256, 8, 256))
    assert dg(None, 256, 256, None, 256, None, 256, 0, 256) == 0
    assert "16-byte aligned" in err(L.hs_dgrad_mask(4, 256, 256, 16, 256, 16, 256, 8, 256, 16, 16, 16, None))
    assert "workspace" in err(L.hs_dgrad_mask(16, 256, 256, 16, 256, 16, 256, 8, 256, 16, 16, None, None))
    assert L.hs_dgrad_mask_workspace(256) == 256 * 256 and L.hs_dgrad_mask_workspace(21) == 0
    assert L.hs_dgrad_mask_partial_rows(32768, 256) == 512 and L.hs_dgrad_mask_partial_rows(4096, 256) == 256
    assert L.hs_dgrad_mask_partial_rows(37, 21) == 2 and L.hs_dgrad_mask_partial_rows(0, 21) == 0
    # empty problems are no-ops, not errors
    assert L.hs_ppo_loss(None, None, None, None, None, None, 0, 0.2, 1, None, None, None, None) == 0
    assert L.hs_colsum(None, 0, 0, None, None, None, None) == 0
    # workspace sizes: loss 3B + 4 blocks + 2; colsum partial rows bounded; Adam one partial per 1024 elements
    assert L.hs_ppo_loss_workspace(32768) == 3 * 32768 + 4 * 128 + 2
    assert 1 <= L.hs_colsum_partial_rows(32768, 256) <= 32768 // 64
    assert L.hs_colsum_workspace(16, 90112) == 0          # single pass for short matrices
    assert L.hs_adam_workspace(317995) == (317995 + 1023) // 1024 + 64   # + one rounding partial per chunk of 16


def test_header_is_plain_c():
    """include/hsim.h is a C-ABI header: it compiles as C and as C++ with no torch/HIP types."""
    import shutil
    import subprocess
    hdr = os.path.join(ROOT, "include", "hsim.h")
    code = re.sub(r"/\*.*?\*/", "", open(hdr).read(), flags=re.S)       # declarations only
    assert "torch" not in code and "hip" not in code.replace("hsim", "")
    for cc, lang in (("gcc", "c"), ("g++", "c++")):
        if shutil.which(cc):
            subprocess.run([cc, "-fsyntax-only", "-Wall", "-Werror", "-x", lang, hdr], check=True)


def test_struct_layouts_match_the_c_compiler(tmp_path):
    """Size and every field offset of the ctypes mirrors equal what the C compiler lays out for
    include/hsim.h (hs_env_config, hs_buffers, hs_batch_info)."""
    import shutil
    import subprocess
    from mujocoposelearning_amd import _lib
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    structs = {"hs_env_config": _lib.hs_env_config, "hs_buffers": _lib.hs_buffers, "hs_batch_info": _lib.hs_batch_info}
    # the INTEGRATION.md stub's own mirror of hs_env_config must match too
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    stub = re.search(r"(class HsEnvConfig\(C.Structure\):.*?\]\n)", text, re.S).group(1)
    ns = {"C": C}
    exec(stub, ns)
    structs["hs_env_config_stub"] = ns["HsEnvConfig"]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "hsim.h"', "int main(void) {"]
    for name, cls in structs.items():
        cname = name.replace("_stub", "")
        lines.append(f'  printf("{name} size %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'  printf("{name} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("  return 0;\n}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l}
    for name, cls in structs.items():
        assert got[(name, "size")] == C.sizeof(cls), name
        for f, _ in cls._fields_:
            assert got[(name, f)] == getattr(cls, f).offset, (name, f)


def test_batch_buffer_views_are_not_shadowed_by_methods():
    """HsBatch serves its device buffers (b.obs, b.reward, ...) through __getattr__, which a class
    attribute of the same name would shadow silently (a method named ``reward`` once did)."""
    from mujocoposelearning_amd import _lib
    from mujocoposelearning_amd.batch import HsBatch
    names = [f[0] for f in _lib.hs_buffers._fields_]
    assert "reward" in names and "obs" in names
    assert [n for n in names if hasattr(HsBatch, n)] == []
