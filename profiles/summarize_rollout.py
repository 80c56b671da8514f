"""Summarize a profiles/collect_rollout.sh run (the train leg's fused rollout kernel) into
profiles/<tag>_summary.md + profiles/traffic_rollout_kernel.json (read by bench.py's train.roofline).

HBM bytes per launch as MI355X_MICROARCH.md (HBM/rocprofv3) prescribes: FETCH_SIZE and WRITE_SIZE from
separate --pmc passes, in KiB, gfx950's FETCH_SIZE counting wide reads at 1/2: 2*FETCH + WRITE.
TCP_TCC_READ_REQ_sum counts the CUs' read requests to L2; at 128 B per request (a wave's coalesced 1-KB
weight-row load is 8 of them) the count reproduces the pi-net weight stream's algorithmic bytes (r6c:
326 vs 323 KB per env step), so the L2 read bytes below are requests x 128 B.
Usage: python profiles/summarize_rollout.py <tag> [n_envs] [n_steps]
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KNAME = "step_kernel_queue<double, 27, false, true>"


def _rows(src, sub):
    f = os.path.join(src, sub, f"{sub}_counter_collection.csv")
    by = {}
    for r in csv.DictReader(open(f)):
        if KNAME in r["Kernel_Name"]:
            by.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    return [by[k] for k in sorted(by)]


def main(tag="r6_rollout", n_envs=4096, n_steps=32, keep=2):
    n_envs, n_steps = int(n_envs), int(n_steps)
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    kt = [r for r in csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_trace.csv"))) if KNAME in r["Kernel_Name"]]
    kt.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in kt][-keep:]
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_stats.csv"))))
    fetch = statistics.mean(r["FETCH_SIZE"] for r in _rows(src, "fetch")[-keep:])
    write = statistics.mean(r["WRITE_SIZE"] for r in _rows(src, "write")[-keep:])
    tcp = _rows(src, "tcp")[-keep:]
    l2req = statistics.mean(r["TCP_TCC_READ_REQ_sum"] for r in tcp)
    tcp_acc = statistics.mean(r["TCP_TOTAL_CACHE_ACCESSES_sum"] for r in tcp)
    sq = _rows(src, "sq")[-keep:]
    sqm = {k: statistics.mean(r[k] for r in sq) for k in sq[0]}
    env_steps = n_envs * n_steps
    hbm = (2 * fetch + write) * 1024
    ms = statistics.mean(durs)
    sys.path.insert(0, ROOT)
    from bench import L2_PEAK_GBS, rollout_algo_bytes
    algo_hbm, algo_l2 = rollout_algo_bytes(352, 21, n_steps)
    out = dict(source=f"profiles/{tag}_summary.md", kernel=KNAME, env_steps_per_launch=env_steps, kernel_ms=ms,
               fetch_kib_per_launch=fetch, write_kib_per_launch=write, hbm_bytes_per_launch=hbm,
               hbm_bytes_per_env_step=hbm / env_steps, algo_hbm_bytes_per_env_step=algo_hbm,
               l2_read_requests_per_launch=l2req, l2_read_bytes_per_launch=128 * l2req,
               l2_read_bytes_per_env_step=128 * l2req / env_steps, algo_l2_weight_bytes_per_env_step=algo_l2,
               tcp_cache_accesses_per_launch=tcp_acc,
               valu_busy_frac=sqm["SQ_ACTIVE_INST_VALU"] / sqm["SQ_WAVE_CYCLES"],
               wait_frac=sqm["SQ_WAIT_ANY"] / sqm["SQ_WAVE_CYCLES"],
               issue_any_frac=sqm["SQ_ACTIVE_INST_ANY"] / sqm["SQ_WAVE_CYCLES"],
               valu_insts_per_env_step=sqm["SQ_INSTS_VALU"] / env_steps)
    json.dump(out, open(os.path.join(ROOT, "profiles", "traffic_rollout_kernel.json"), "w"), indent=1)
    L = [f"# rocprofv3 summary `{tag}` -- the train leg's fused rollout kernel", "",
         f"Command: `bash profiles/collect_rollout.sh {tag}` (bench.py train leg only: 4096 fp64 envs, PPO n_steps "
         f"{n_steps}, batch 32768, 4 epochs, MLP[256,256] ReLU, staggered clocks; warm-up + 2 timed iterations). "
         f"Per-launch figures average the last {keep} `{KNAME}` launches ({n_steps} env steps x {n_envs} envs each).", "",
         "## Kernel stats (rocprofv3 --kernel-trace --stats, top 8)", "",
         "| kernel | calls | avg us | % |", "|---|---|---|---|"]
    for r in stats[:8]:
        L.append(f"| `{r['Name'][:90].replace('|', '/')}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                 f"{float(r['Percentage']):.2f} |")
    L += ["", "## The fused rollout kernel", "",
          f"- duration {ms:.3f} ms per launch = {ms / n_steps * 1e3:.1f} us per env step of {n_envs} envs",
          f"- HBM (separate --pmc passes, gfx950-corrected 2*FETCH+WRITE): {hbm / 1e6:,.1f} MB per launch = "
          f"{hbm / env_steps:,.0f} B per env step (algorithmic {algo_hbm:,.0f} B: rollout rows + per-launch state, "
          f"bench.rollout_algo_bytes) = {hbm / env_steps / algo_hbm:.2f}x; {hbm / (ms * 1e-3) / 1e9:,.0f} GB/s",
          f"- L2 read requests from the CUs (TCP_TCC_READ_REQ_sum): {l2req:,.0f} per launch x 128 B = "
          f"{128 * l2req / 1e9:,.1f} GB = {128 * l2req / env_steps / 1e3:,.0f} KB per env step (pi-net weight stream, "
          f"algorithmic {algo_l2 / 1e3:,.0f} KB: the f32 weights once per wave for its two envs); "
          f"{128 * l2req / (ms * 1e-3) / 1e12:,.2f} TB/s = {128 * l2req / (ms * 1e-3) / 1e9 / L2_PEAK_GBS:.2f} of the "
          f"{L2_PEAK_GBS / 1e3:.1f} TB/s shared-row L2 rate (MI355X_MICROARCH.md)",
          f"- the excess HBM traffic over the algorithmic rows is the chunk queue's hand-off: each env step of a pair "
          f"passes its state, action and return through UNCACHED rows (~93 values written and read, 1.5 KB per env "
          f"step), which the TCC counters over-report (DESIGN.md 3.1)",
          f"- SQ: VALU busy {out['valu_busy_frac']:.3f}, waiting {out['wait_frac']:.3f}, issuing {out['issue_any_frac']:.3f} "
          f"of wave cycles; {out['valu_insts_per_env_step']:,.0f} VALU wave instructions per env step", ""]
    open(os.path.join(ROOT, "profiles", f"{tag}_summary.md"), "w").write("\n".join(L) + "\n")
    print("\n".join(L))


if __name__ == "__main__":
    main(*sys.argv[1:])
