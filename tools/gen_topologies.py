#!/usr/bin/env python3
"""Generate isaacgymenv_amd/csrc/gs_topologies.h from the packed models.

Every articulation the kernels support gets a struct of compile-time tables
(body parents, generalized-DOF tree, ancestor lists, contact candidates and
their LDS slot offsets).  With these as ``constexpr`` the kernels fully unroll
their tree walks and keep per-body state in VGPRs (no runtime-indexed arrays,
no scratch).  The registry at the end maps a model's topology signature
(``_model.topology_signature``) to its kernel instantiation.

Run:  python tools/gen_topologies.py   (build() checks the file is current)
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from isaacgymenv_amd.isaacgym._assets import RawModel, build_articulation, PACKED_DIR  # noqa: E402
from isaacgymenv_amd.isaacgym._model import flatten, topology_signature  # noqa: E402

# (struct name, packed model, asset options as the reference task sets them, force sensors compiled in)
# Force sensors (gym.create_asset_force_sensor) keep every body's pose and motion subspace live until
# the end of the substep; only the topologies whose tasks create sensors (Ant, ant.py:174-178) pay for it.
MODELS = [
    ("anymal_c", "anymal_c.model.json", dict(collapse_fixed_joints=True, replace_cylinder_with_capsule=True), False),
    ("cartpole", "cartpole.model.json", dict(fix_base_link=True), False),
    ("nv_ant", "nv_ant.model.json", dict(), True),
    ("hound", "hound.model.json", dict(collapse_fixed_joints=False), False),
]

OUT = os.path.join(ROOT, "isaacgymenv_amd", "csrc", "gs_topologies.h")


def topo_tables(flat: dict) -> dict:
    nb, nd, nc = flat["nb"], flat["nd"], flat["nc"]
    fixed = flat["fixed_base"]
    nbase = 0 if fixed else 6
    nv = nbase + nd
    parent = [int(p) for p in flat["parent"]]
    bdof = [int(d) for d in flat["bdof"]]
    dpar = []
    for k in range(nbase):
        dpar.append(k - 1)
    body_of_dof = {bdof[b]: b for b in range(nb) if bdof[b] >= 0}
    for j in range(nd):
        b = body_of_dof[j]
        pb = parent[b]
        if pb == 0:
            dpar.append(nbase - 1)
        else:
            dpar.append(nbase + bdof[pb])
    anc = []
    for k in range(nv):
        lst, a = [], dpar[k]
        while a >= 0:
            lst.append(a)
            a = dpar[a]
        anc.append(lst)
    maxdep = max(1, max(len(a) for a in anc))
    # generalized dof that moves each body (root: last base dof or -1 when fixed)
    bgdof = [(nbase - 1) if b == 0 else nbase + bdof[b] for b in range(nb)]
    cbody = [int(b) for b in flat["cbody"]]
    cleaf = [bgdof[b] for b in cbody]
    csupp = [0 if l < 0 else len(anc[l]) + 1 for l in cleaf]
    # LDS slots per candidate: scaled Z rows (3 x supp) + J.nu_free (3) + Delassus diagonal (3)
    cslot, off = [], 0
    for s in csupp:
        cslot.append(off)
        off += 3 * s + 6
    # joint-limit rows, one potential row per dof (node nbase + j): scaled Z (supp) + c + 1/diag
    lleaf = [nbase + j for j in range(nd)]
    lsupp = [len(anc[l]) + 1 for l in lleaf]
    lslot = []
    for s in lsupp:
        lslot.append(off)
        off += s + 2
    gbody = [0] * nbase + [body_of_dof[j] for j in range(nd)]
    # last body (DFS order) of each body's subtree: where its subtree sums are complete
    subend = list(range(nb))
    for b in range(nb - 1, 0, -1):
        subend[parent[b]] = max(subend[parent[b]], subend[b])
    cshape = [int(s) for s in flat["cshape"]]
    ns = int(flat["ns"])
    # candidates of shape s are contiguous (body, shape, point order): [sh_c0[s], sh_c1[s]) on body sh_body[s]
    sh_c0 = [min([c for c in range(nc) if cshape[c] == s] or [nc]) for s in range(ns)]
    sh_c1 = [max([c + 1 for c in range(nc) if cshape[c] == s] or [nc]) for s in range(ns)]
    sh_body = [cbody[sh_c0[s]] if sh_c0[s] < nc else 0 for s in range(ns)]
    jkind = [int(k) for k in flat["jkind"]]
    team = team_tables(flat, parent, bdof, nbase)
    return dict(pair_a=[int(x) for x in flat["pair_a"]], pair_b=[int(x) for x in flat["pair_b"]],
                pair_k=[int(x) for x in flat["pair_kind"]],
                cdyn=[int(k) for k in flat["cdyn"]], shkind=[int(k) for k in flat["shkind"]],
                NPK=int(flat["npool"]), NPAIR=int(flat["npair"]),
                NR=int(flat["nr"]), clink=[int(l) for l in flat["clink"]], TEAM=team, NB=nb, ND=nd, NC=nc, NS=int(flat["ns"]), FIXED=fixed, NBASE=nbase, NV=nv, MAXDEP=maxdep,
                parent=parent, bdof=bdof, jkind=jkind, dpar=dpar, depth=[len(a) for a in anc],
                anc=[a + [-1] * (maxdep - len(a)) for a in anc], bgdof=bgdof, cbody=cbody, cleaf=cleaf,
                csupp=csupp, cslot=cslot, NSLOT=max(off, 1), gbody=gbody, cshape=cshape, subend=subend,
                lleaf=lleaf, lsupp=lsupp, lslot=lslot, sh_c0=sh_c0, sh_c1=sh_c1, sh_body=sh_body)


def team_tables(flat, parent, bdof, nbase):
    """Lane-team layout for a floating 'uniform star': root + NCH identical-structure serial chains.

    Returns None when the topology does not qualify (the one-env-per-lane kernel is used)."""
    nb = len(parent)
    if nbase != 6 or nb < 2:
        return None
    kids = {}
    for b in range(1, nb):
        kids.setdefault(parent[b], []).append(b)
    chains = []
    for top in kids.get(0, []):
        ch, cur = [top], top
        while cur in kids:
            if len(kids[cur]) != 1:
                return None
            cur = kids[cur][0]
            ch.append(cur)
        chains.append(ch)
    nch, cl = len(chains), len(chains[0])
    if any(len(c) != cl for c in chains) or nch > 8 or cl != 3:  # the team PGS distributes 6 + 3 components
        return None
    # chains must be contiguous in body order with dofs in the same order
    for c, ch in enumerate(chains):
        if ch != list(range(1 + c * cl, 1 + (c + 1) * cl)) or [bdof[b] for b in ch] != list(range(c * cl, (c + 1) * cl)):
            return None
    cbody = [int(b) for b in flat["cbody"]]
    cshape = [int(s) for s in flat["cshape"]]
    rc = sum(1 for b in cbody if b == 0)
    if cbody[:rc] != [0] * rc:
        return None
    rest = list(zip(cbody[rc:], cshape[rc:]))
    if len(rest) % nch:
        return None
    cc = len(rest) // nch
    per = [rest[c * cc:(c + 1) * cc] for c in range(nch)]
    loc_b = [b - 1 - 0 * cl for b, _ in per[0]]
    root_shapes = max(cshape[:rc]) + 1 if rc else 0
    shapes_per_chain = (max(s for _, s in rest) + 1 - root_shapes) // nch if rest else 0
    loc_s = [s - root_shapes for _, s in per[0]]
    for c in range(nch):
        if [b - 1 - c * cl for b, _ in per[c]] != loc_b:
            return None
        if [s - root_shapes - c * shapes_per_chain for _, s in per[c]] != loc_s:
            return None
    lanes = 1
    while lanes < nch:
        lanes *= 2
    if lanes > 4:  # quad-DPP reductions: up to 4 lanes per env
        return None
    return dict(LANES=lanes, NCH=nch, CL=cl, RC=rc, CC=cc, RS=root_shapes, SPC=shapes_per_chain,
                ccb=loc_b, ccs=loc_s, rcs=cshape[:rc] or [0])


def carr(v) -> str:
    if isinstance(v[0], list):
        return "{" + ", ".join(carr(x) for x in v) + "}"
    return "{" + ", ".join(str(int(x)) for x in v) + "}"


def emit() -> str:
    lines = [
        "// GENERATED by tools/gen_topologies.py -- do not edit by hand.",
        "// Compile-time articulation topologies for the specialised physics kernels.",
        "#pragma once",
        "",
    ]
    reg = []
    for name, packed, opts, sens in MODELS:
        with open(os.path.join(PACKED_DIR, packed)) as f:
            art = build_articulation(RawModel.from_json(json.load(f)), opts)
        flat = flatten(art)
        t = topo_tables(flat)
        sig = topology_signature(flat)
        lines.append(f"struct Topo_{name} {{")
        lines.append(f'  static constexpr const char* kName = "{name}";')
        for k in ("NB", "NR", "ND", "NC", "NS", "FIXED", "NBASE", "NV", "MAXDEP", "NSLOT", "NPAIR", "NPK"):
            lines.append(f"  static constexpr int {k} = {t[k]};")
        for k, n in (("parent", "NB"), ("bdof", "NB"), ("jkind", "NB"), ("bgdof", "NB"), ("subend", "NB"), ("dpar", "NV"),
                     ("depth", "NV"), ("gbody", "NV"), ("cbody", "NC"), ("clink", "NC"), ("cshape", "NC"), ("cleaf", "NC"), ("csupp", "NC"), ("cslot", "NC"),
                     ("lleaf", "ND"), ("lsupp", "ND"), ("lslot", "ND"), ("sh_c0", "NS"), ("sh_c1", "NS"),
                     ("sh_body", "NS"), ("cdyn", "NC"), ("shkind", "NS"), ("pair_a", "NPAIR"), ("pair_b", "NPAIR"),
                     ("pair_k", "NPAIR")):
            vals = t[k] if len(t[k]) else [0]
            dim = n if len(t[k]) else "1"
            lines.append(f"  static constexpr int {k}[{dim}] = {carr(vals)};")
        lines.append(f"  static constexpr int anc[NV][MAXDEP] = {carr(t['anc'])};")
        lines.append(f"  static constexpr bool SENS = {'true' if sens else 'false'};  // force sensors compiled in")
        tm = t["TEAM"]
        if tm:
            lines.append("  // lane-team layout (gs_team.hip): LANES lanes per env, lane c owns chain c")
            lines.append("  static constexpr bool HAS_TEAM = true;")
            for k in ("LANES", "NCH", "CL", "RC", "CC", "RS", "SPC"):
                lines.append(f"  static constexpr int T_{k} = {tm[k]};")
            for k in ("ccb", "ccs", "rcs"):
                vals = tm[k] if tm[k] else [0]
                lines.append(f"  static constexpr int T_{k}[{len(vals)}] = {carr(vals)};")
        else:
            lines.append("  static constexpr bool HAS_TEAM = false;")
        lines.append("};")
        lines.append("")
        reg.append((sig, name))
    lines.append("#define GS_FOR_EACH_TOPOLOGY(X) \\")
    lines.append(" \\\n".join(f'  X(Topo_{n}, "{s}")' for s, n in reg))
    lines.append("")
    return "\n".join(lines)


def main(check: bool = False) -> int:
    text = emit()
    if check:
        cur = open(OUT).read() if os.path.exists(OUT) else ""
        return 0 if cur == text else 1
    with open(OUT, "w") as f:
        f.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main("--check" in sys.argv))
