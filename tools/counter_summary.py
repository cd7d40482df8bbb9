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
    if name.startswith("_Z"):  # mangled: ...14k_pd_step_teamI13Topo_anymal_cLb1ELb0EE...
        m = re.search(r"\d(k_[a-z0-9_]+?)(?:I\d|E|v)", name)
        t = re.search(r"Topo_([a-z0-9_]+?)(?=[A-Z])", name)
    else:
        m = re.search(r"(k_\w+|soa_rw|aos_dof_rw|aos13_write|stream_copy|\w*gae\w*)(<[^>]*>)?", name)
        t = re.search(r"Topo_(\w+?)[,> ]", name)
    base = m.group(1) if m else name[:60]
    if not t:
        return base
    # the template's bool arguments in order (demangled ", true" / mangled "Lb1E"): k_pd_step_team<T, TERR, TGS>
    # is "k_pd_step_team<anymal_c,0,1>" for the headline (plane, TGS)
    tail = name[t.end() - 1:]
    bits = re.findall(r"(?:, (true|false))|(?:Lb([01])E)", tail.split("(")[0] if "<" in name else tail)
    flags = "".join(("1" if a == "true" or b == "1" else "0") for a, b in bits)
    return base + f"<{t.group(1)}{',' + ','.join(flags) if flags else ''}>"


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
