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
import re
import statistics
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STATS_STEPS = 3     # bench.py's stats_of() steps after the timed window


LLVM = "/opt/rocm/lib/llvm/bin"
CODE_OBJECTS = [os.path.join(ROOT, "build", "obj", f"hs_kernels_{p}.o") for p in ("f32", "f64")]   # make -C .../csrc


def code_object_resources(objs=None):
    """Per-kernel register / LDS / scratch figures from the gfx950 code object's own metadata
    (amdhsa.kernels notes of the object's .hip_fatbin offload bundle): the numbers the loader uses.
    vgpr_count is the unified register count (arch VGPRs + AGPRs); rocprofv3's VGPR_Count /
    Accum_VGPR_Count columns are granule-rounded allocations and do not split it the same way."""
    out = {}
    for obj in objs or CODE_OBJECTS:
        out.update(_code_object_resources(obj))
    return out


def _code_object_resources(obj):
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", obj, os.path.join(td, "o")])
        data = open(fat, "rb").read()
        out = {}
        pos = 0
        while True:
            pos = data.find(b"__CLANG_OFFLOAD_BUNDLE__", pos)
            if pos < 0: break
            n = struct.unpack_from("<Q", data, pos + 24)[0]
            p = pos + 32
            for _ in range(n):
                off, size, idl = struct.unpack_from("<QQQ", data, p); p += 24
                ident = data[p:p + idl].decode(); p += idl
                if "gfx950" in ident:
                    co = os.path.join(td, "co.elf")
                    open(co, "wb").write(data[pos + off: pos + off + size])
                    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
                    item = None
                    for line in notes.splitlines():
                        m = re.match(r"(\s*)(-?)\s*\.(\w+):\s+(.*)$", line)
                        if not m: continue
                        ind, dash, k, v = m.groups()
                        if dash and len(ind) == 2:   # a new entry of amdhsa.kernels
                            item = {}
                        if item is None: continue
                        if k == "name": out[v.strip()] = item
                        elif k in ("vgpr_count", "agpr_count", "sgpr_count", "private_segment_fixed_size", "group_segment_fixed_size", "vgpr_spill_count", "sgpr_spill_count"):
                            item[k] = int(v)
            pos += 24
        return out


def is_step(name):
    # the resident-tier step kernel: one wave per pair (step_kernel<...>) or the chunk-queue schedule
    # (step_kernel_queue<...>, the fp64 engine at 4096 envs)
    return ("step_kernel<" in name or "step_kernel_queue<" in name) and "wide" not in name


def resource_lines(kernel_name, out):
    """Registers from the code object's metadata (authoritative), rocprofv3's columns beside them."""
    lines = []
    try:
        res = code_object_resources()
        mangled = next((k for k in res if k in kernel_name), None)
        if mangled is None:   # rocprofv3 prints demangled names: match on the instance's template arguments
            # step_kernel_queue<T, 27, PGS, ROLL>: the per-step instance has ROLL = false (the fused-rollout
            # instance, ROLL = true, never runs in the profiled bench legs)
            queue = "queue" in kernel_name
            want = ("step_kernel_queue" if queue else "step_kernel") + ("Id" if "double" in kernel_name else "If") + \
                "Li27ELb" + ("1" if "true" in kernel_name.split(",")[2] else "0") + ("ELb0E" if queue else "E")
            mangled = next((k for k in res if want in k and "wide" not in k), None)
        r = res.get(mangled)
        if r:
            out["code_object"] = dict(r, kernel=mangled)
            lines.append(f"Code object ({mangled[:60]}...): arch VGPR {r['vgpr_count'] - r['agpr_count']} + AGPR "
                         f"{r['agpr_count']} (unified {r['vgpr_count']}), SGPR {r['sgpr_count']}, VGPRs spilled "
                         f"{r['vgpr_spill_count']}, SGPRs spilled to VGPR lanes {r['sgpr_spill_count']}, scratch "
                         f"{r['private_segment_fixed_size']} B/lane, LDS {r['group_segment_fixed_size']} B/workgroup.")
    except (OSError, subprocess.CalledProcessError, StopIteration) as e:
        lines.append(f"(code object metadata unavailable: {e})")
    lines.append(f"rocprofv3 columns (allocation granules, not the split above): VGPR_Count {out['vgpr']}, "
                 f"Accum_VGPR_Count {out['agpr']}, SGPR {out['sgpr']}, LDS {out['lds_bytes']} B/workgroup, scratch "
                 f"{out['scratch_bytes_per_lane']} B/lane, grid {out['grid']} threads x wg {out['workgroup']}.")
    return lines


def resources_report(path=None):
    """profiles/resources_<tag>.md: every step-kernel instance's registers from the code object."""
    res = code_object_resources()
    lines = ["# Step-kernel resources from the gfx950 code object metadata (build/obj/hs_kernels_{f32,f64}.o)", "",
             "| kernel | arch VGPR | AGPR | unified | VGPR spilled | SGPR | SGPR spills (to VGPR lanes) | scratch B/lane | LDS B/wg |",
             "|---|---|---|---|---|---|---|---|---|"]
    for k in sorted(res):
        if "kernel" not in k:
            continue
        r = res[k]
        lines.append(f"| `{k[:70]}` | {r['vgpr_count'] - r['agpr_count']} | {r['agpr_count']} | {r['vgpr_count']} | "
                     f"{r['vgpr_spill_count']} | {r['sgpr_count']} | {r['sgpr_spill_count']} | "
                     f"{r['private_segment_fixed_size']} | {r['group_segment_fixed_size']} |")
    text = "\n".join(lines) + "\n"
    if path:
        open(path, "w").write(text)
    return text


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
              f"time, 5 warning counters = 88 values written once and read once: {2 * 88 * es} B/env, "
              f"{2 * 88 * es * n_envs / 1e6:.2f} MB/launch) through UNCACHED memory, whose 8-byte lane accesses the "
              f"TCC counters report at ~4-5x (r2c: +16 MB WRITE_SIZE, +7 MB FETCH_SIZE vs the one-wave-per-pair "
              f"kernel r2a); traffic/(algo + hand-off) = {corrected / (algo + 2 * 88 * es * n_envs):.2f}x; "
              f"{corrected / (statistics.mean(win) * 1e-3) / 1e9:.0f} GB/s of the 8 TB/s HBM"]
              if "queue" in row["Kernel_Name"] else []) + ["",
              "## Resources", ""] + resource_lines(row["Kernel_Name"], out)
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
    if sys.argv[1:2] == ["--resources"]:      # python profiles/summarize.py --resources <tag>
        print(resources_report(os.path.join(ROOT, "profiles", f"resources_{sys.argv[2]}.md")))
    else:
        main(*sys.argv[1:])
