"""The C-ABI libraries load and export every entry point include/*.h declares (no GPU calls)."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBS = {"gymsim.h": "isaacgymenv_amd/_lib/libgymsim.so", "gymtask.h": "isaacgymenv_amd/_lib/libgymtask.so",
        "gymrl.h": "isaacgymenv_amd/_lib/libgymrl.so"}


def _declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b((?:gs|gt|rl)_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module", autouse=True)
def built():
    from isaacgymenv_amd import build
    build.build(verbose=False)


@pytest.mark.parametrize("header", sorted(LIBS))
def test_library_exports_declared_symbols(header):
    path = os.path.join(ROOT, LIBS[header])
    lib = ctypes.CDLL(path)  # loads without a GPU
    names = _declared(header)
    assert names, header
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"{LIBS[header]} lacks {missing}"


def test_python_bindings_cover_the_abi():
    from isaacgymenv_amd.isaacgym import _lib
    from isaacgymenv_amd import gymtask
    assert sorted(_lib.EXPORTED_SYMBOLS) == _declared("gymsim.h")
    assert sorted(gymtask.EXPORTED_SYMBOLS) == _declared("gymtask.h")
    from isaacgymenv_amd.rl import gae
    assert sorted(gae.EXPORTED_SYMBOLS) == _declared("gymrl.h")
    assert gae.lib().rl_abi_version() == 7


def test_abi_version_and_topology_query():
    from isaacgymenv_amd.isaacgym import _lib
    from tests import helpers as H
    L = _lib.lib()
    assert L.gs_abi_version() == 9
    for make in (H.anymal, H.cartpole, H.hound):
        art, flat = make()
        d, keep = _lib.model_desc(flat)
        assert L.gs_topology_supported(d) == 1


def test_sim_create_fails_cleanly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("has a GPU")
    from isaacgymenv_amd.isaacgym import _lib
    L = _lib.lib()
    p = _lib.GsSimParams()
    p.dt = 0.005
    assert not L.gs_sim_create(0, p)
    assert b"gs_sim_create" in L.gs_last_error()


def test_topology_header_is_current():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_topologies.py"), "--check"])
    assert r.returncode == 0, "run tools/gen_topologies.py"


def test_ctypes_struct_layouts_match_the_headers(tmp_path):
    """Every ctypes mirror has the C struct's size and field offsets (gcc on include/*.h)."""
    import shutil
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    from isaacgymenv_amd.isaacgym import _lib
    from isaacgymenv_amd import gymtask
    from isaacgymenv_amd.rl import gae
    mirrors = {"gs_model_desc": _lib.GsModelDesc, "gs_sim_params": _lib.GsSimParams, "gs_pd_args": _lib.GsPdArgs,
               "gt_torch_rand_plan": gymtask.GtTorchRandPlan, "gt_anymal_params": gymtask.GtAnymalParams,
               "gt_anymal_buffers": gymtask.GtAnymalBuffers, "gt_anymal_reset_draws": gymtask.GtAnymalResetDraws,
               "gt_hound_control_params": gymtask.GtHoundControlParams, "gt_ant_params": gymtask.GtAntParams,
               "gt_ant_buffers": gymtask.GtAntBuffers, "gt_anymal_terrain_reset": gymtask.GtAnymalTerrainReset,
               "gt_anymal_hound": gymtask.GtAnymalHound, "rl_linear_groups": gae.LinearGroups,
               "rl_opt_hyper": gae.OptHyper}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "gymsim.h"', '#include "gymtask.h"', '#include "gymrl.h"',
             "int main(void) {"]
    expect = []
    for cname, py in mirrors.items():
        lines.append(f'  printf("%zu\\n", sizeof({cname}));')
        expect.append(C_sizeof(py))
        for f in py._fields_:
            lines.append(f'  printf("%zu\\n", offsetof({cname}, {f[0]}));')
            expect.append(getattr(py, f[0]).offset)
    lines.append("  return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == expect


def C_sizeof(py):
    return ctypes.sizeof(py)


def test_linear_bwd_rejects_bias_partials_without_weight_partials():
    """rl_linear_bwd computes the bias partials in the weight-gradient pass, so bpart without wpart
    is refused before any launch (no GPU needed) instead of returning 0 with bpart unwritten."""
    from isaacgymenv_amd.rl import gae
    L = gae.lib()
    buf = (ctypes.c_double * 4096)()
    p = ctypes.addressof(buf)
    rc = L.rl_linear_bwd(p, p, 128, 128, p, 128, 128, p, None, 1, None, p, 0, None)
    assert rc != 0
    assert b"wpart" in L.rl_last_error()
