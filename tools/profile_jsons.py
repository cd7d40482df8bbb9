"""Write profiles/pmc_pd_step.json and profiles/valu_pd_step.json (read by bench.py) from a counter
session summary (tools/counters_round.sh -> gpurun_out/<tag>/summary.json), and copy the summary into
profiles/<round>_counters_summary.json.

    python tools/profile_jsons.py gpurun_out/<tag>/summary.json --round r02h

FETCH_SIZE is converted to bytes with the factor CALIBRATED in the same session on the kernel's own
access shapes (tools/hbm_calib: the SoA state read and the AoS dof read, both dword per lane, known
byte counts), not with the guide's 16-B streaming rule alone; the streaming control is reported beside.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_pd_step_team<anymal_c,0,1>"  # <T, TERR, TGS>: the headline (plane, TGS)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("summary")
    ap.add_argument("--round", required=True)
    ap.add_argument("--num-envs", type=int, default=4096)
    a = ap.parse_args()
    s = json.load(open(a.summary))
    calib_bytes = json.load(open(os.path.join(os.path.dirname(a.summary), "calib_bytes.json")))
    cf, cw = s["calib_FETCH_SIZE"], s["calib_WRITE_SIZE"]

    def factor(kernel, which, counter, src):
        return calib_bytes[kernel][which] / (src[kernel][counter] * 1024.0)

    fetch_factors = {k: factor(k, "read", "FETCH_SIZE", cf) for k in ("soa_rw", "aos_dof_rw", "stream_copy")}
    write_factors = {k: factor(k, "write", "WRITE_SIZE", cw) for k in ("soa_rw", "aos_dof_rw", "aos13_write",
                                                                       "stream_copy")}
    # the kernel's reads are mostly the SoA state: use that shape's factor
    ff, wf = fetch_factors["soa_rw"], write_factors["soa_rw"]
    fk = s["bench_FETCH_SIZE"][KERNEL]["FETCH_SIZE"]
    wk = s["bench_WRITE_SIZE"][KERNEL]["WRITE_SIZE"]
    import bench  # noqa: E402  (the kernel-scoped algorithmic bytes)
    alg = bench.physics_kernel_bytes_per_env() * a.num_envs
    pmc = {"kernel": "k_pd_step_team<Topo_anymal_c> (gs_sim_pd_step)", "num_envs": a.num_envs, "round": a.round,
           "counters": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, --kernel-trace "
                       "(tools/counters_round.sh)",
           "dispatches": s["bench_FETCH_SIZE"][KERNEL]["dispatches"],
           "fetch_size_kb_per_launch": fk, "write_size_kb_per_launch": wk,
           "fetch_factor_calibrated": ff, "write_factor_calibrated": wf,
           "calibration": {"fetch_bytes_per_counted_byte": fetch_factors,
                           "write_bytes_per_counted_byte": write_factors,
                           "program": "tools/hbm_calib.hip (known byte counts, same session)"},
           "hbm_bytes_per_launch": fk * 1024.0 * ff + wk * 1024.0 * wf,
           "algorithmic_bytes_per_launch": alg,
           "note": "traffic = FETCH_SIZE x calibrated factor (SoA dword reads) + WRITE_SIZE x calibrated factor"}
    with open(os.path.join(ROOT, "profiles", "pmc_pd_step.json"), "w") as f:
        json.dump(pmc, f, indent=1)
    sq = {}
    for p, d in s.items():
        if p.startswith("sq") and KERNEL in d:
            sq.update(d[KERNEL])
    waves = sq["SQ_WAVES"]
    flops = sq["SQ_INSTS_VALU_FLOPS_FP32"] * 64
    valu = {"kernel": "k_pd_step", "num_envs": a.num_envs, "round": a.round,
            "counters": "rocprofv3 --pmc SQ_* passes with --kernel-trace (tools/counters_round.sh)",
            "waves_per_launch": waves, "valu_insts_per_wave": sq["SQ_INSTS_VALU"] / waves,
            "wave_cycles_per_wave_x4": sq["SQ_WAVE_CYCLES"] / waves,
            "busy_frac_valu": sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_WAVE_CYCLES"],
            "wait_frac": sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"],
            "fp32_flops_per_launch": flops, "fp32_flops_per_env_step": flops / a.num_envs}
    with open(os.path.join(ROOT, "profiles", "valu_pd_step.json"), "w") as f:
        json.dump(valu, f, indent=1)
    shutil.copy(a.summary, os.path.join(ROOT, "profiles", f"{a.round}_counters_summary.json"))
    shutil.copy(os.path.join(os.path.dirname(a.summary), "calib_bytes.json"),
                os.path.join(ROOT, "profiles", f"{a.round}_calib_bytes.json"))
    print(json.dumps(pmc, indent=1))
    print(json.dumps(valu, indent=1))


if __name__ == "__main__":
    import sys
    sys.path.insert(0, ROOT)
    main()
