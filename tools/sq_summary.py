"""Per-wave SQ counter summary of a kernel from tools/sq_counters.sh output.

    python tools/sq_summary.py gpurun_out/<tag> [--kernel k_pd_step]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="k_pd_step")
    ap.add_argument("--json", default=None, help="write the VALU summary (profiles/valu_pd_step.json)")
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--round", type=int, default=1)
    a = ap.parse_args()
    tot = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(a.dir, "sq_*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", r.get("Kernel", ""))
            if a.kernel in name:
                tot[r["Counter_Name"]].append(float(r["Counter_Value"]))
    med = {k: sorted(v)[len(v) // 2] for k, v in tot.items()}
    waves = med.get("SQ_WAVES", 1.0)
    print(f"{a.kernel}: {int(waves)} waves per dispatch (median of {len(tot.get('SQ_WAVES', []))} dispatches)")
    for k in sorted(med):
        print(f"  {k:28s} {med[k]:16.0f}  per wave {med[k] / waves:12.1f}")
    if a.json:
        import json
        # SQ_INSTS_VALU_FLOPS_FP32 counts FLOPs per lane summed over wave instructions (FMA = 2);
        # x64 lanes = FP32 FLOPs executed per launch (replicated team work included)
        flops = med["SQ_INSTS_VALU_FLOPS_FP32"] * 64
        out = {"kernel": a.kernel, "num_envs": a.num_envs, "round": a.round,
               "counters": "rocprofv3 --pmc SQ_* passes with --kernel-trace (tools/sq_counters.sh)",
               "waves_per_launch": waves,
               "valu_insts_per_wave": med["SQ_INSTS_VALU"] / waves,
               "wave_cycles_per_wave_x4": med["SQ_WAVE_CYCLES"] / waves,
               "busy_frac_valu": med["SQ_ACTIVE_INST_VALU"] / med["SQ_WAVE_CYCLES"],
               "wait_frac": med["SQ_WAIT_ANY"] / med["SQ_WAVE_CYCLES"],
               "fp32_flops_per_launch": flops,
               "fp32_flops_per_env_step": flops / a.num_envs}
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
