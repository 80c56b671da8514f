"""Summarize a profiles/collect.sh run into profiles/<tag>_summary.md + traffic_step_kernel.json.

HBM bytes per launch follow MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE and WRITE_SIZE come
from separate --pmc passes, are in KiB (x1024), and gfx950's FETCH_SIZE counts wide reads at 1/2,
so the corrected figure is 2*FETCH + WRITE (the raw figure is reported beside it).

Usage: python profiles/summarize.py <tag> <precision> [n_envs] [timed_steps]
The resident-tier step kernel (``step_kernel<T, 27, ...>``) is summarized; the wide-tier launch
(``step_kernel_wide``) is listed in the stats table.  Per-launch figures average the last
``timed_steps`` launches before bench.py's 3 statistics steps (its timed window, after the
staggered-episode precondition).
traffic_step_kernel.json keeps one entry per precision (bench.py reads the one it runs).
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STATS_STEPS = 3     # bench.py's stats_of() steps after the timed window


def is_step(name):
    # the resident-tier step kernel: one wave per pair (step_kernel<...>) or the chunk-queue schedule
    # (step_kernel_queue<...>, the fp64 engine at 4096 envs)
    return ("step_kernel<" in name or "step_kernel_queue<" in name) and "wide" not in name


def main(tag="r2a", precision="fp64", n_envs=4096, timed=50, src=None):
    n_envs, timed = int(n_envs), int(timed)
    es = 8 if precision == "fp64" else 4
    algo_env = 83 * es + 21 * 4 + 436 * es + 2          # bench.algo_bytes_per_env_step
    src = src or os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_stats.csv"))))
    ktrace = [r for r in csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_trace.csv")))
              if is_step(r["Kernel_Name"])]
    ktrace.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in ktrace]
    win = durs[-timed - STATS_STEPS:-STATS_STEPS]

    def pmc(name):
        sub = name.split("_")[0].lower()
        rows = [r for r in csv.DictReader(open(os.path.join(src, sub, f"{sub}_counter_collection.csv")))
                if is_step(r["Kernel_Name"])]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        # (the timed window's kernel: the first dispatch is the reset launch, which is always the
        # one-wave-per-pair instance)
        return [float(r["Counter_Value"]) for r in rows][-timed - STATS_STEPS:-STATS_STEPS], rows[-1 - STATS_STEPS]
    fetch, row = pmc("FETCH_SIZE")
    write, _ = pmc("WRITE_SIZE")
    f_kib, w_kib = statistics.mean(fetch), statistics.mean(write)
    raw = (f_kib + w_kib) * 1024
    corrected = (2 * f_kib + w_kib) * 1024
    algo = algo_env * n_envs
    out = dict(tag=tag, n_envs=n_envs, precision=precision, kernel=row["Kernel_Name"][:80],
               avg_ms_timed=statistics.mean(win), timed_launches=len(win), avg_ms_all=statistics.mean(durs),
               launches=len(durs), fetch_kib_per_launch=f_kib, write_kib_per_launch=w_kib,
               hbm_bytes_per_launch_raw=raw, hbm_bytes_per_launch=corrected, algo_bytes_per_env_step=algo_env,
               algo_bytes_per_launch=algo, traffic_over_algo=corrected / algo,
               vgpr=int(row["VGPR_Count"]), agpr=int(row["Accum_VGPR_Count"]), sgpr=int(row["SGPR_Count"]),
               lds_bytes=int(row["LDS_Block_Size"]), scratch_bytes_per_lane=int(row["Scratch_Size"]),
               grid=int(row["Grid_Size"]), workgroup=int(row["Workgroup_Size"]))
    lines = [f"# rocprofv3 summary `{tag}` -- step kernel, {n_envs} envs, {precision}", "",
             f"Command: `bash profiles/collect.sh {tag} {precision}` (bench.py --steps {timed} --warmup 5, sim-only "
             "legs only, staggered-episode precondition)", "",
             "## Kernel stats (rocprofv3 --kernel-trace --stats)", "",
             "| kernel | calls | avg us | min us | max us | % |", "|---|---|---|---|---|---|"]
    for r in stats[:8]:
        name = r["Name"][:90].replace("|", "/")
        lines.append(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['MinNs']) / 1e3:.1f} | "
                     f"{float(r['MaxNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    lines += ["", f"Resident-tier step kernel, timed window (last {len(win)} launches): avg {out['avg_ms_timed']:.3f} ms "
                  f"(all {len(durs)} launches incl. reset / precondition episode: {out['avg_ms_all']:.3f} ms).", "",
              "## HBM traffic per launch (separate --pmc passes, timed window)", "",
              f"- FETCH_SIZE {f_kib:,.0f} KiB, WRITE_SIZE {w_kib:,.0f} KiB",
              f"- raw (FETCH+WRITE)*1024 = {raw / 1e6:,.2f} MB; gfx950-corrected (2*FETCH+WRITE)*1024 = "
              f"{corrected / 1e6:,.2f} MB",
              f"- algorithmic {algo / 1e6:,.2f} MB ({algo_env} B/env step x {n_envs}); traffic/algo = "
              f"{corrected / algo:.2f}x"] + ([
              f"- chunk-queue schedule: + the hand-off of each env between its two items (qpos, qvel, warm start, "
              f"time, 4 warning counters = 87 values written once and read once: {2 * 87 * es} B/env, "
              f"{2 * 87 * es * n_envs / 1e6:.2f} MB/launch) through UNCACHED memory, whose 8-byte lane accesses the "
              f"TCC counters report at ~4-5x (r2c: +16 MB WRITE_SIZE, +7 MB FETCH_SIZE vs the one-wave-per-pair "
              f"kernel r2a); traffic/(algo + hand-off) = {corrected / (algo + 2 * 87 * es * n_envs):.2f}x; "
              f"{corrected / (statistics.mean(win) * 1e-3) / 1e9:.0f} GB/s of the 8 TB/s HBM"]
              if "queue" in row["Kernel_Name"] else []) + ["",
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
            if is_step(r["Kernel_Name"]):
                by.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
        ids = sorted(by, key=int)[-timed - STATS_STEPS:-STATS_STEPS]
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
                             f"{life / kc:.0%}")
    path = os.path.join(ROOT, "profiles", "traffic_step_kernel.json")
    try:
        allp = json.load(open(path))
        if "precision" in allp:          # r1 single-entry layout
            allp = {allp["precision"]: allp}
    except (OSError, ValueError):
        allp = {}
    allp[precision] = out
    json.dump(allp, open(path, "w"), indent=1)
    open(os.path.join(ROOT, "profiles", f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(*sys.argv[1:])
