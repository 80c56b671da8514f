"""Static instruction census of a step-kernel instance from the gfx950 code object.

Disassembles the kernel (llvm-objdump on the .hip_fatbin offload bundle of build/obj/hs_kernels_<p>.o)
and counts its instructions by class: fp64 arithmetic, fp32 arithmetic, transcendental, register
moves between the VGPR and AGPR files (spill traffic), lane movement (readlane / writelane / DPP /
permlane / bpermute), selects, integer / address work, scalar work, memory (LDS / global / scalar
loads).  Static counts weigh every instruction once; tools/census_dynamic.md pairs them with
rocprofv3's SQ_INSTS_* counters of one launch (profiles/r6*/census_*).

Usage: python tools/census.py [f64|f32] [kernel-substring] [--json out.json]
"""
import collections
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(obj):
    """The gfx950 ELF of a hipcc -c object's offload bundle."""
    td = tempfile.mkdtemp()
    fat = os.path.join(td, "fat.bin")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", obj, os.path.join(td, "o")])
    data = open(fat, "rb").read()
    pos = 0
    while True:
        pos = data.find(b"__CLANG_OFFLOAD_BUNDLE__", pos)
        if pos < 0:
            raise RuntimeError("no gfx950 code object in " + obj)
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, idl = struct.unpack_from("<QQQ", data, p)
            p += 24
            ident = data[p:p + idl].decode()
            p += idl
            if "gfx950" in ident:
                co = os.path.join(td, "co.elf")
                open(co, "wb").write(data[pos + off: pos + off + size])
                return co
        pos += 24


def disassemble(co, kernel_sub):
    txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", "--mcpu=gfx950", co],
                         capture_output=True, text=True, check=True).stdout
    out, name, cur = {}, None, None
    for line in txt.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            name = m.group(1)
            cur = out.setdefault(name, []) if kernel_sub in name else None
            continue
        if cur is not None:
            m = re.match(r"^\s+([a-z_0-9]+)(\s.*)?$", line)
            if m and not line.strip().startswith(";"):
                cur.append((m.group(1), (m.group(2) or "").strip()))
    return out


CLASSES = [
    ("fp64 fma/mul/add", lambda o, a: re.match(r"v_(fma|mul|add|fmac|sub)_f64|v_(fma|mul|add)_f64", o)),
    ("fp64 transcendental / special", lambda o, a: re.match(r"v_(rsq|rcp|sqrt|div_scale|div_fmas|div_fixup|frexp|ldexp|trig|fract|floor|ceil|trunc|rndne|max|min|cmp|cmpx)_.*f64", o)),
    ("fp32 arithmetic", lambda o, a: re.match(r"v_(fma|mul|add|sub|fmac|mac|max|min|med3|rcp|rsq|sqrt|exp|log|cmp|cmpx|pk_fma|pk_mul|pk_add)_.*f32", o)),
    ("AGPR<->VGPR moves (spill traffic)", lambda o, a: o.startswith("v_accvgpr")),
    ("lane movement", lambda o, a: o.startswith(("v_readlane", "v_writelane", "v_readfirstlane", "v_permlane", "ds_bpermute",
                                                   "ds_permute", "ds_swizzle")) or "row_" in a or "quad_perm" in a or "dpp" in o),
    ("selects", lambda o, a: o.startswith("v_cndmask")),
    ("vector moves", lambda o, a: o.startswith(("v_mov_b32", "v_mov_b64", "v_pk_mov"))),
    ("vector int / address / bitwise", lambda o, a: o.startswith(("v_lshl", "v_lshr", "v_ashr", "v_and", "v_or", "v_xor",
                                                                 "v_add_u32", "v_sub_u32", "v_add_co", "v_addc", "v_sub_co",
                                                                 "v_subb", "v_mad_u", "v_mad_i", "v_mul_lo", "v_mul_hi",
                                                                 "v_mul_u32", "v_mul_i32", "v_bfe", "v_bfi", "v_alignbit",
                                                                 "v_cmp_", "v_cmpx_", "v_min_", "v_max_", "v_not", "v_bcnt",
                                                                 "v_ffbl", "v_ffbh", "v_lshl_add", "v_add_lshl", "v_add3",
                                                                 "v_or3", "v_and_or", "v_xad", "v_cvt_"))),
    ("scalar ALU", lambda o, a: o.startswith("s_") and not o.startswith(("s_load", "s_buffer", "s_store", "s_waitcnt",
                                                                          "s_cbranch", "s_branch", "s_nop", "s_sleep",
                                                                          "s_endpgm", "s_setprio", "s_barrier", "s_memtime",
                                                                          "s_memrealtime", "s_getpc", "s_setpc", "s_swappc"))),
    ("scalar loads", lambda o, a: o.startswith(("s_load", "s_buffer_load"))),
    ("waits / nops / branches", lambda o, a: o.startswith(("s_waitcnt", "s_nop", "s_cbranch", "s_branch", "s_setprio", "s_sleep",
                                                         "s_endpgm", "s_barrier"))),
    ("LDS", lambda o, a: o.startswith("ds_")),
    ("global / buffer memory", lambda o, a: o.startswith(("global_", "buffer_", "flat_", "scratch_"))),
]


def classify(ins):
    c = collections.Counter()
    ops = collections.Counter()
    for o, a in ins:
        ops[o] += 1
        for name, f in CLASSES:
            if f(o, a):
                c[name] += 1
                break
        else:
            c["other"] += 1
    return c, ops


def main(argv):
    prec = argv[1] if len(argv) > 1 and argv[1] in ("f64", "f32") else "f64"
    sub = argv[2] if len(argv) > 2 and not argv[2].startswith("--") else "step_kernel_queueIdLi27ELb0ELb0E"
    obj = os.path.join(ROOT, "build", "obj", f"hs_kernels_{prec}.o")
    ks = disassemble(code_object(obj), sub)
    report = {}
    for k, ins in ks.items():
        c, ops = classify(ins)
        tot = sum(c.values())
        print(f"{k}: {tot} instructions")
        for name, n in c.most_common():
            print(f"  {name:36s} {n:7d}  {100 * n / tot:5.1f}%")
        print("  top opcodes:", ", ".join(f"{o} {n}" for o, n in ops.most_common(25)))
        report[k] = {"total": tot, "classes": dict(c), "opcodes": dict(ops)}
    if "--json" in argv:
        json.dump(report, open(argv[argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv)
