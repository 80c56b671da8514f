"""Markdown table of gpu_learning_curve_ref.py logs (one column per seed).

python tools/probes/lc_report.py gpurun_out/r4l/lc_seed0.log gpurun_out/r4l/lc_seed1.log ... [--every 2e6]
Rows: env steps (the first log line at or past each multiple of --every); cells: SB3's ep_rew_mean (mean
return of the last 100 finished episodes) / upright fraction of the rollout's steps (torso above 1.0 m)."""
import re
import sys

PAT = re.compile(r"seed (\d+) iter\s+(\d+) steps\s+([\d.]+)M ep_rew_mean\s+([-\d.naninf]+) episodes\s+(\d+) "
                 r"upright ([\d.]+) height ([\d.]+) vf_loss ([-\d.naninf]+) log_std ([-\d.]+) "
                 r"rollout ([\d.]+)s train ([\d.]+)s per iter\s+([\d.]+)s")


def parse(path):
    rows = []
    for line in open(path):
        m = PAT.search(line)
        if m:
            rows.append(dict(seed=int(m.group(1)), it=int(m.group(2)), steps=float(m.group(3)) * 1e6,
                             ret=float(m.group(4)), episodes=int(m.group(5)), upright=float(m.group(6)),
                             height=float(m.group(7)), log_std=float(m.group(9)), t_roll=float(m.group(10)),
                             t_train=float(m.group(11)), wall=float(m.group(12))))
    return rows


def main(argv):
    every = 2e6
    paths = []
    i = 0
    while i < len(argv):
        if argv[i] == "--every":
            every = float(argv[i + 1])
            i += 2
        else:
            paths.append(argv[i])
            i += 1
    runs = [parse(p) for p in paths]
    top = max((r[-1]["steps"] for r in runs if r), default=0)
    marks = []
    k = every
    while k <= top + every:
        marks.append(k)
        k += every
    hdr = ["env steps"] + [f"seed {r[0]['seed']}" if r else p for r, p in zip(runs, paths)]
    print("| " + " | ".join(hdr) + " |")
    print("|" + "---|" * len(hdr))
    for mk in marks:
        cells = []
        for r in runs:
            hit = next((x for x in r if x["steps"] >= mk), None)
            cells.append(f"{hit['ret']:.1f} / {hit['upright']:.2f}" if hit else "")
        if any(cells):
            print(f"| {mk / 1e6:.0f} M | " + " | ".join(cells) + " |")
    print()
    for r, p in zip(runs, paths):
        if not r:
            print(f"- {p}: no progress lines")
            continue
        best = max(r, key=lambda x: x["ret"])
        last = r[-1]
        print(f"- seed {last['seed']}: {last['steps'] / 1e6:.2f} M env steps, {last['episodes']} episodes in "
              f"{last['wall']:.0f} s; final ep_rew_mean {last['ret']:.1f}, upright {last['upright']:.2f}, "
              f"log_std {last['log_std']:.2f}; best {best['ret']:.1f} at {best['steps'] / 1e6:.1f} M "
              f"(rollout {last['t_roll']:.3f} s + update {last['t_train']:.3f} s per iteration)")


if __name__ == "__main__":
    main(sys.argv[1:])
