"""Reduce a counter session (tools/counters_round.sh) to per-kernel medians, on the GPU box.

    python tools/counter_summary.py gpurun_out/<tag> [--keep-raw]

Writes <dir>/summary.json: {pass: {kernel: {counter: median per dispatch, "dispatches": n}}} for the
physics / task kernels and the calibration kernels (torch's own kernels are dropped), then deletes
the raw per-dispatch CSVs (they run to hundreds of MB) unless --keep-raw.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import shutil
import statistics
import sys
from collections import defaultdict

KEEP = ("k_pd_step", "k_simulate", "k_post_", "k_reset", "k_kinematics", "k_hound", "k_ant", "k_measure",
        "k_refresh", "k_set_", "soa_rw", "aos_dof_rw", "aos13_write", "stream_copy", "gae")


def short(name: str) -> str:
    m = re.search(r"(k_\w+|soa_rw|aos_dof_rw|aos13_write|stream_copy|\w*gae\w*)(<[^>]*>|I[0-9]+\w+?E)?", name)
    base = m.group(1) if m else name[:60]
    t = re.search(r"Topo_(\w+?)[,>E ]", name)
    terr = ", true" in name or "Lb1E" in name
    return base + (f"<{t.group(1)}{', terr' if terr else ''}>" if t else "")


def main():
    d = sys.argv[1]
    keep_raw = "--keep-raw" in sys.argv
    out = {}
    for f in sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv"))):
        pas = os.path.basename(os.path.dirname(f))
        vals = defaultdict(lambda: defaultdict(list))
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", r.get("Kernel", ""))
                if not any(k in name for k in KEEP):
                    continue
                vals[short(name)][r["Counter_Name"]].append(float(r["Counter_Value"]))
        out[pas] = {k: dict({c: statistics.median(v) for c, v in cs.items()},
                            dispatches=max(len(v) for v in cs.values())) for k, cs in vals.items()}
    with open(os.path.join(d, "summary.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    if not keep_raw:
        for sub in glob.glob(os.path.join(d, "*")):
            if os.path.isdir(sub):
                shutil.rmtree(sub)
    print(f"{len(out)} passes summarised into {d}/summary.json")


if __name__ == "__main__":
    main()
