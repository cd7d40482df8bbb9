"""Print the per-step kernel timeline (durations and idle gaps) from a rocprofv3 kernel trace.

    python tools/timeline.py gpurun_out/<tag>/stats/run_kernel_trace.csv [--steps 150 153]
"""
import argparse
import csv
import re


def short(n):
    m = re.search(r"(k_\w+|copyBuffer\w*|fillBuffer\w*|distribution_\w+|partition_kernel|direct_copy|\w+Functor\w*)", n)
    return m.group(1) if m else n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, nargs=2, default=[150, 153])
    ap.add_argument("--key", default="k_pd_step")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.key in r["Kernel_Name"]]
    i0, i1 = idx[a.steps[0]], idx[a.steps[1]]
    prev = None
    busy = 0.0
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += (e - s) / 1e3
        print(f"{short(r['Kernel_Name']):44s} {(e - s) / 1e3:8.2f} us  gap {((s - prev) / 1e3 if prev else 0):7.2f} us")
        prev = e
    span = (int(rows[i1]["Start_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1e3 / (a.steps[1] - a.steps[0])
    print(f"per step: {span:.1f} us, kernels busy {busy / (a.steps[1] - a.steps[0]):.1f} us")


if __name__ == "__main__":
    main()
