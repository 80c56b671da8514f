"""Dynamic instruction census of the fp64 step kernel from profiles/census.sh (rocprofv3 SQ_INSTS_*
passes over bench.py's default window), per env step, beside the static census (tools/census.py).

Usage: python tools/census_report.py <tag> [n_envs] [timed]   (reads gpurun_out/census_<tag>/)
Prints a markdown table; SQ_INSTS_* count wave instructions (one per 64-lane wave instruction).
"""
import csv
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STATS_STEPS = 3


def is_step(name):
    return "step_kernel_queue<double, 27, false, false>" in name


def load(src, sub, timed):
    by = {}
    f = os.path.join(src, sub, f"{sub}_counter_collection.csv")
    for r in csv.DictReader(open(f)):
        if is_step(r["Kernel_Name"]):
            by.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(by)[-timed - STATS_STEPS:-STATS_STEPS]
    return {k: statistics.mean(by[i][k] for i in ids) for k in by[ids[0]]}, len(ids)


def census(tag, n_envs=4096, timed=50):
    src = os.path.join(ROOT, "gpurun_out", f"census_{tag}")
    c = {}
    n = None
    for sub in ("v1", "v2", "v3"):
        if os.path.exists(os.path.join(src, sub)):
            d, n = load(src, sub, timed)
            c.update(d)
    per = {k: v / n_envs for k, v in c.items()}
    valu = per["SQ_INSTS_VALU"]
    f64 = per["SQ_INSTS_VALU_FMA_F64"] + per["SQ_INSTS_VALU_MUL_F64"] + per["SQ_INSTS_VALU_ADD_F64"]
    typed = f64 + per["SQ_INSTS_VALU_TRANS_F64"] + per["SQ_INSTS_VALU_INT32"] + per["SQ_INSTS_VALU_INT64"] + \
        per["SQ_INSTS_VALU_CVT"] + sum(per.get(f"SQ_INSTS_VALU_{o}_F32", 0.0) for o in ("FMA", "MUL", "ADD", "TRANS"))
    rows = [("VALU (all)", valu), ("  fp64 FMA", per["SQ_INSTS_VALU_FMA_F64"]), ("  fp64 MUL", per["SQ_INSTS_VALU_MUL_F64"]),
            ("  fp64 ADD", per["SQ_INSTS_VALU_ADD_F64"]), ("  fp64 transcendental", per["SQ_INSTS_VALU_TRANS_F64"]),
            ("  int32", per["SQ_INSTS_VALU_INT32"]), ("  int64", per["SQ_INSTS_VALU_INT64"]), ("  conversions", per["SQ_INSTS_VALU_CVT"]),
            ("  fp32 FMA/MUL/ADD/TRANS", sum(per.get(f"SQ_INSTS_VALU_{o}_F32", 0.0) for o in ("FMA", "MUL", "ADD", "TRANS"))),
            ("  untyped (moves, DPP / permlane, AGPR reads / writes, readlane / writelane, selects, compares, bitwise)", valu - typed),
            ("SALU", per.get("SQ_INSTS_SALU", 0.0)), ("SMEM", per.get("SQ_INSTS_SMEM", 0.0)), ("LDS", per.get("SQ_INSTS_LDS", 0.0)),
            ("branches", per.get("SQ_INSTS_BRANCH", 0.0)), ("VMEM reads", per.get("SQ_INSTS_VMEM_RD", 0.0)),
            ("VMEM writes", per.get("SQ_INSTS_VMEM_WR", 0.0))]
    lines = [f"| class (per env step, wave instructions / 2 envs per wave counted per env) | per env step | of VALU |", "|---|---|---|"]
    for name, v in rows:
        lines.append(f"| {name} | {v:,.0f} | {100 * v / valu:.1f}% |" if name.startswith("  ") or name == "VALU (all)"
                     else f"| {name} | {v:,.0f} | |")
    if "SQ_INSTS_VALU_FLOPS_FP64" in per:
        lines.append(f"| fp64 FLOPs (SQ_INSTS_VALU_FLOPS_FP64) | {per['SQ_INSTS_VALU_FLOPS_FP64']:,.0f} | |")
    return c, per, "\n".join(lines), n


if __name__ == "__main__":
    tag = sys.argv[1] if len(sys.argv) > 1 else "r6b"
    n_envs = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    c, per, table, n = census(tag, n_envs)
    print(f"timed launches: {n}")
    print(table)
