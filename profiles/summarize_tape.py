"""Tape launch vs per-step launches from one profiles/collect_tape.sh run -> profiles/<tag>_tape_summary.md.

The bench run holds the headline's per-step launches and, after them, the tape leg: a fresh batch,
its untimed staggered episode (667 per-step launches), 5 warm-up steps and ONE tape launch of 50 env
steps (the longest step-kernel dispatch).  Compared: the tape dispatch against the median of the 50
per-step dispatches of the same batch right before its warm-up (same episode mix), per dispatch and
per env step.  SQ cycle counters are quad-cycles; GRBM_GUI_ACTIVE / 8 is the kernel's cycles per XCD.
python profiles/summarize_tape.py <tag> [k=50]"""
import csv
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "profiles"))
from summarize import is_step  # noqa: E402


def dispatches(path):
    rows = [r for r in csv.DictReader(open(path)) if is_step(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def counters(path):
    out = {}
    for r in csv.DictReader(open(path)):
        if is_step(r["Kernel_Name"]):
            out.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    return out


def pick(rows):
    """(tape dispatch, the 50 per-step dispatches before the warm-up) of a trace"""
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    it = max(range(len(rows)), key=lambda i: durs[i])
    return rows[it], rows[it - 55:it - 5]


def main(tag, k=50):
    k = int(k)
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    lines = [f"# Tape launch vs per-step launches, rocprofv3 `{tag}` (4096 envs, fp64, staggered episode mix)", "",
             f"Command: `bash profiles/collect_tape.sh {tag}`; `python profiles/summarize_tape.py {tag}`.", ""]
    tr = dispatches(os.path.join(src, "trace", "trace_kernel_trace.csv"))
    tape, per = pick(tr)
    dt = (int(tape["End_Timestamp"]) - int(tape["Start_Timestamp"])) / 1e6
    dp = statistics.median((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in per)
    lines += ["| | per-step launch (median of 50) | tape launch (50 env steps) |", "|---|---|---|",
              f"| kernel | `{per[0]['Kernel_Name'][:60]}` | same instance, p.nsteps = {k} |",
              f"| duration | {dp:.3f} ms | {dt:.3f} ms = **{dt / k:.3f} ms per env step** |",
              f"| env steps/s (4096 envs) | {4096 / dp * 1e3 / 1e6:.2f} M | {4096 * k / dt * 1e3 / 1e6:.2f} M |"]
    for name in ("fetch", "write"):
        p = os.path.join(src, name, f"{name}_counter_collection.csv")
        if os.path.exists(p):
            c = counters(p)
            rows = dispatches(os.path.join(src, name, f"{name}_kernel_trace.csv"))
            t, pr = pick(rows)
            cn = "FETCH_SIZE" if name == "fetch" else "WRITE_SIZE"
            vt = c.get(int(t["Dispatch_Id"]), {}).get(cn)
            vp = statistics.median(c.get(int(r["Dispatch_Id"]), {}).get(cn, 0.0) for r in pr)
            if vt is not None:
                lines.append(f"| {cn} (KiB, raw) | {vp:,.0f} per launch | {vt:,.0f} = {vt / k:,.0f} per env step |")
    p = os.path.join(src, "sq", "sq_counter_collection.csv")
    if os.path.exists(p):
        c = counters(p)
        rows = dispatches(os.path.join(src, "sq", "sq_kernel_trace.csv"))
        t, pr = pick(rows)
        ct = c[int(t["Dispatch_Id"])]
        cp = {n: statistics.median(c[int(r["Dispatch_Id"])][n] for r in pr) for n in ct}

        def row(label, f):
            lines.append(f"| {label} | {f(cp)} | {f(ct)} |")
        row("waves parked on s_waitcnt (SQ_WAIT_ANY / SQ_WAVE_CYCLES)", lambda x: f"{x['SQ_WAIT_ANY'] / x['SQ_WAVE_CYCLES']:.1%}")
        row("VALU busy (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES)", lambda x: f"{x['SQ_ACTIVE_INST_VALU'] / x['SQ_WAVE_CYCLES']:.1%}")
        row("issuing (SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES)", lambda x: f"{x['SQ_ACTIVE_INST_ANY'] / x['SQ_WAVE_CYCLES']:.1%}")
        row("waves (SQ_WAVES)", lambda x: f"{x['SQ_WAVES']:,.0f}")
        row("mean wave lifetime / kernel (SQ_WAVE_CYCLES*4/SQ_WAVES vs GRBM_GUI_ACTIVE/8)",
            lambda x: f"{x['SQ_WAVE_CYCLES'] * 4 / x['SQ_WAVES'] / (x['GRBM_GUI_ACTIVE'] / 8):.0%}")
        row("VALU instructions per env step (SQ_INSTS_VALU)",
            lambda x: f"{x['SQ_INSTS_VALU'] / (k if x is ct else 1) / 4096:,.0f} per env")
    text = "\n".join(lines) + "\n"
    open(os.path.join(ROOT, "profiles", f"{tag}_tape_summary.md"), "w").write(text)
    print(text)


if __name__ == "__main__":
    main(*sys.argv[1:])
