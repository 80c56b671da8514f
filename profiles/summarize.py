"""Summarize a profiles/collect.sh run into profiles/<tag>_summary.md + traffic_step_kernel.json.

HBM bytes per launch follow MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE and WRITE_SIZE come
from separate --pmc passes, are in KiB (x1024), and gfx950's FETCH_SIZE counts wide reads at 1/2,
so the corrected figure is 2*FETCH + WRITE (the raw figure is reported beside it).
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag="r01", n_envs=4096, precision="fp32", src=None):
    src = src or os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_stats.csv"))))
    ktrace = [r for r in csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_trace.csv")))
              if "step_kernel" in r["Kernel_Name"]]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in ktrace]
    steady = durs[7:] if len(durs) > 10 else durs     # skip reset + warmup launches
    def pmc(name):
        f = os.path.join(src, name.split("_")[0].lower(), f"{name.split('_')[0].lower()}_counter_collection.csv")
        rows = [r for r in csv.DictReader(open(f)) if "step_kernel" in r["Kernel_Name"]]
        vals = [float(r["Counter_Value"]) for r in rows]
        return vals, rows[0]
    fetch, row = pmc("FETCH_SIZE")
    write, _ = pmc("WRITE_SIZE")
    f_kib = statistics.mean(fetch[7:]) if len(fetch) > 10 else statistics.mean(fetch)
    w_kib = statistics.mean(write[7:]) if len(write) > 10 else statistics.mean(write)
    raw = (f_kib + w_kib) * 1024
    corrected = (2 * f_kib + w_kib) * 1024
    algo = 2162 * n_envs
    out = dict(tag=tag, n_envs=n_envs, precision=precision, kernel="step_kernel",
               avg_ms_steady=statistics.mean(steady), avg_ms_all=statistics.mean(durs), launches=len(durs),
               fetch_kib_per_launch=f_kib, write_kib_per_launch=w_kib, hbm_bytes_per_launch_raw=raw,
               hbm_bytes_per_launch=corrected, algo_bytes_per_launch=algo, traffic_over_algo=corrected / algo,
               vgpr=int(row["VGPR_Count"]), agpr=int(row["Accum_VGPR_Count"]), sgpr=int(row["SGPR_Count"]),
               lds_bytes=int(row["LDS_Block_Size"]), scratch_bytes_per_lane=int(row["Scratch_Size"]),
               grid=int(row["Grid_Size"]), workgroup=int(row["Workgroup_Size"]))
    json.dump(out, open(os.path.join(ROOT, "profiles", "traffic_step_kernel.json"), "w"), indent=1)
    lines = [f"# rocprofv3 summary `{tag}` -- step kernel, {n_envs} envs, {precision}", "",
             "Command: `bash profiles/collect.sh` (bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --groups 1 --free-groups 0 --no-configs)", "",
             "## Kernel stats (rocprofv3 --kernel-trace --stats)", "",
             "| kernel | calls | avg us | min us | max us | % |", "|---|---|---|---|---|---|"]
    for r in stats[:6]:
        name = r["Name"][:90].replace("|", "/")
        lines.append(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['MinNs']) / 1e3:.1f} | "
                     f"{float(r['MaxNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    lines += ["", f"Steady-state step_kernel launches (after reset + warmup): avg {out['avg_ms_steady']:.3f} ms "
                  f"over {len(steady)} launches (all {len(durs)} launches: {out['avg_ms_all']:.3f} ms).", "",
              "## HBM traffic per launch (separate --pmc passes)", "",
              f"- FETCH_SIZE {f_kib:,.0f} KiB, WRITE_SIZE {w_kib:,.0f} KiB",
              f"- raw (FETCH+WRITE)*1024 = {raw / 1e6:,.2f} MB; gfx950-corrected (2*FETCH+WRITE)*1024 = "
              f"{corrected / 1e6:,.2f} MB",
              f"- algorithmic {algo / 1e6:,.2f} MB (2162 B/env step x {n_envs}); traffic/algo = "
              f"{corrected / algo:.1f}x", "",
              "## Resources", "",
              f"VGPR {out['vgpr']} (+{out['agpr']} AGPR), SGPR {out['sgpr']}, LDS {out['lds_bytes']} B/workgroup, "
              f"scratch {out['scratch_bytes_per_lane']} B/lane, grid {out['grid']} threads x wg {out['workgroup']}."]
    sq = {}
    for sub in ("sq", "sq2"):
        f = os.path.join(src, sub, f"{sub}_counter_collection.csv")
        if not os.path.exists(f):
            continue
        by = {}
        for r in csv.DictReader(open(f)):
            if "step_kernel" in r["Kernel_Name"]:
                by.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
        ids = sorted(by, key=int)
        ids = ids[7:] if len(ids) > 10 else ids
        for k in by[ids[0]]:
            sq[k] = statistics.mean(by[i][k] for i in ids)
    if sq:
        out["sq"] = sq
        wc = sq.get("SQ_WAVE_CYCLES", 0)
        lines += ["", "## Issue / stall picture (SQ counters, per launch; SQ cycle counters are quad-cycles)", ""]
        for k in sorted(sq):
            lines.append(f"- {k}: {sq[k]:,.0f}")
        if wc:
            lines += ["",
                      f"- waves parked on s_waitcnt (SQ_WAIT_ANY / SQ_WAVE_CYCLES): {sq['SQ_WAIT_ANY'] / wc:.1%}",
                      f"- issuing (SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES): {sq['SQ_ACTIVE_INST_ANY'] / wc:.1%}",
                      f"- VALU instructions per wave per launch: {sq['SQ_INSTS_VALU'] / sq['SQ_WAVES']:,.0f}"]
            if "GRBM_GUI_ACTIVE" in sq:
                kc = sq["GRBM_GUI_ACTIVE"] / 8
                life = 4 * wc / sq["SQ_WAVES"]
                lines.append(f"- mean wave lifetime {life:,.0f} cycles vs kernel {kc:,.0f} cycles (GRBM_GUI_ACTIVE/8): "
                             f"{life / kc:.0%} -- the rest is the Newton-iteration tail (one wave per slot at 4096 envs)")
        json.dump(out, open(os.path.join(ROOT, "profiles", "traffic_step_kernel.json"), "w"), indent=1)
    open(os.path.join(ROOT, "profiles", f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(*sys.argv[1:2])
