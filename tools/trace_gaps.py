"""GPU busy time and idle gaps per env step from a rocprofv3 kernel trace (headline bench steps and the last PPO
rollout steps of a `bench.py ... --ppo-epochs K` run):
    python tools/trace_gaps.py gpurun_out/<tag>/trace/run_kernel_trace.csv [--steps 20]
Per step: wall (pd_step start to the next pd_step start), busy (sum of kernel durations), and the mean gap before
each kernel kind."""
import argparse
import collections
import csv
import re


def short(n):
    m = re.search(r"(k_\w+|copyBuffer\w*|fillBuffer\w*|distribution_\w+|\w+Functor\w*)", n)
    return (m.group(1) if m else n[:40])[:40]


def window(rows, a, b, nsteps):
    gap = collections.defaultdict(float)
    busy, prev = 0.0, None
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        if prev is not None:
            gap[short(r["Kernel_Name"])] += max(0, s - prev)
        prev = e
    wall = int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])
    return wall / 1e3 / nsteps, busy / 1e3 / nsteps, {k: v / 1e3 / nsteps for k, v in gap.items() if v > 0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "k_pd_step" in r["Kernel_Name"]]
    n = a.steps
    for name, (i0, i1) in (("headline", (idx[15], idx[15 + n])), ("ppo rollout", (idx[-n - 1], idx[-1]))):
        wall, busy, gaps = window(rows, i0, i1, n)
        print(f"{name}: per step wall {wall:.1f} us, busy {busy:.1f} us, idle {wall - busy:.1f} us; gaps before: "
              + ", ".join(f"{k} {v:.1f}" for k, v in sorted(gaps.items(), key=lambda kv: -kv[1])))


if __name__ == "__main__":
    main()
