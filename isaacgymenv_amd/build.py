"""Build the native libraries in-tree (hipcc, gfx950).

    python -m isaacgymenv_amd.build          # all libraries
Outputs ``isaacgymenv_amd/_lib/libgymsim.so`` (physics + tensor API) and
``isaacgymenv_amd/_lib/libgymtask.so`` (fused task kernels).  Built .so files
are git-ignored but travel to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
ARCH = os.environ.get("GS_OFFLOAD_ARCH", "gfx950")

LIBS = {
    "libgymsim.so": ["gs_physics.hip", "gs_phys_inst.hip", "gs_team.hip", "gs_kinematics.hip", "gs_host.hip",
                     "gs_generic.hip", "gs_capi.hip"],
    "libgymtask.so": ["gt_anymal.hip", "gt_hound.hip", "gt_ant.hip"],
    "libgymrl.so": ["rl_gae.hip", "rl_grad.hip", "rl_rollout.hip", "rl_ppo_loss.hip", "rl_rms.hip", "rl_adam.hip", "rl_linear.hip",
                   "rl_policy.hip"],
}
# phase-profiling build of the simulator (tools/phase_profile.py); never loaded by default, built only
# on request (`python -m isaacgymenv_amd.build --prof`)
PROF_LIBS = {"libgymsim_prof.so": LIBS["libgymsim.so"]}
# the task kernels mirror torch's unfused elementwise arithmetic
# -fno-slp-vectorize: the SLP vectorizer packs the scalar spatial algebra into v_pk_* pairs and
# then spends ~1700 v_mov_b32 (and AGPR copies) arranging register pairs in the physics kernels
SIM_FLAGS = ["-fno-slp-vectorize"]
EXTRA_FLAGS = {"libgymtask.so": ["-ffp-contract=off"], "libgymrl.so": ["-ffp-contract=off"], "libgymsim.so": SIM_FLAGS,
               "libgymsim_prof.so": SIM_FLAGS + ["-DGS_PHASE_PROFILE"]}
HEADERS = ["gs_internal.h", "gs_topologies.h", "gs_math.h", "gs_terrain.h", "gs_pairs.h", "gs_solver.h", "gs_kinematics.h", "gs_host_impl.h",
           "gs_physics_impl.h", "torch_philox.h"]
# gs_phys_inst.hip is compiled once per (topology, kernel form): 0 simulate plane, 1 simulate terrain-mesh,
# 2 fused PD step plane, 3 fused PD step terrain-mesh (gs_physics_impl.h)
INST_SRC = "gs_phys_inst.hip"
INST_FORMS = (0, 1, 2, 3)


def topologies() -> list:
    """Topology struct names in GS_FOR_EACH_TOPOLOGY order (gs_topologies.h, tools/gen_topologies.py)."""
    import re
    text = open(os.path.join(CSRC, "gs_topologies.h")).read()
    body = text[text.index("#define GS_FOR_EACH_TOPOLOGY"):]
    return re.findall(r"X\((Topo_\w+),", body)


def _units(src: str) -> list:
    """(object suffix, extra flags) of each compile of one source."""
    if src != INST_SRC:
        return [("", [])]
    return [(f"_{t[5:]}_{f}", [f"-DGS_INST_TOPO={t}", f"-DGS_INST_FORM={f}"]) for t in topologies() for f in INST_FORMS]
OBJDIR = os.path.join(LIBDIR, "obj")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _stale(out: str, srcs) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = [os.path.join(CSRC, s) for s in srcs] + [os.path.join(CSRC, h) for h in HEADERS]
    # each library implements one public header (the others do not affect it)
    header = {"gs_": "gymsim.h", "gt_": "gymtask.h", "rl_": "gymrl.h"}[srcs[0][:3]]
    deps.append(os.path.join(os.path.dirname(HERE), "include", header))
    deps.append(os.path.abspath(__file__))  # flags live here
    return any(os.path.exists(d) and os.path.getmtime(d) > t for d in deps)


def _deps_newer(out: str, deps) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.exists(d) and os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True, prof: bool = False, variant=None) -> None:
    """Compile every stale library.  Each source is its own hipcc job (objects under _lib/obj/<lib>/,
    all jobs of all libraries in parallel: the physics sources dominate and compile independently),
    then each library is linked from its objects."""
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(LIBDIR, exist_ok=True)
    cc = hipcc()
    inc = ["-I", os.path.join(os.path.dirname(HERE), "include"), "-I", CSRC]
    compile_jobs, link_jobs = [], []
    libs = dict(LIBS, **PROF_LIBS) if prof else LIBS
    if variant:  # (name, defines): an A/B build libgymsim_<name>.so with extra -D flags, never loaded by default
        vname, vdefs = variant
        libs = {f"libgymsim_{vname}.so": LIBS["libgymsim.so"]}
        EXTRA_FLAGS[f"libgymsim_{vname}.so"] = SIM_FLAGS + [f"-D{d}" for d in vdefs]
    for lib, srcs in libs.items():
        if not all(os.path.exists(os.path.join(CSRC, s)) for s in srcs):
            raise RuntimeError(f"missing sources for {lib}: {srcs}")
        out = os.path.join(LIBDIR, lib)
        if not force and not _stale(out, srcs):
            continue
        odir = os.path.join(OBJDIR, lib.replace(".so", ""))
        os.makedirs(odir, exist_ok=True)
        header = {"gs_": "gymsim.h", "gt_": "gymtask.h", "rl_": "gymrl.h"}[srcs[0][:3]]
        common = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.abspath(__file__),
                                                              os.path.join(os.path.dirname(HERE), "include", header)]
        objs = []
        for src in srcs:
            for suffix, defs in _units(src):
                obj = os.path.join(odir, src.replace(".hip", suffix + ".o"))
                objs.append(obj)
                if force or _deps_newer(obj, [os.path.join(CSRC, src)] + common):
                    cmd = [cc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c"] + inc + defs
                    cmd += EXTRA_FLAGS.get(lib, []) + ["-o", obj, os.path.join(CSRC, src)]
                    compile_jobs.append((f"{lib}:{src}{suffix}", cmd))
        link_jobs.append((lib, [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + ["-lpthread"]))

    def run(job):
        name, cmd = job
        if verbose:
            print("[build]", " ".join(cmd), flush=True)
        return name, subprocess.run(cmd, capture_output=True, text=True)

    def run_all(jobs):
        if not jobs:
            return
        workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", "8") or 8)))
        with ThreadPoolExecutor(max_workers=workers) as ex:
            for name, r in ex.map(run, jobs):
                if r.returncode != 0:
                    raise RuntimeError(f"hipcc failed for {name}:\n{r.stdout}\n{r.stderr}")
                if verbose and r.stderr.strip():
                    print(r.stderr[-4000:], file=sys.stderr)

    # the slowest sources first so they overlap everything else
    compile_jobs.sort(key=lambda j: 0 if "hound" in j[0] else (1 if ("gs_team" in j[0] or "gs_phys" in j[0]
                                                                     or "gs_host" in j[0]) else 2))
    run_all(compile_jobs)
    run_all(link_jobs)


if __name__ == "__main__":
    # python -m isaacgymenv_amd.build [--force] [--prof] [--variant NAME DEFINE ...]
    var = None
    if "--variant" in sys.argv:
        k = sys.argv.index("--variant")
        var = (sys.argv[k + 1], [d for d in sys.argv[k + 2:] if not d.startswith("--")])
    build(force="--force" in sys.argv, prof="--prof" in sys.argv, variant=var)
