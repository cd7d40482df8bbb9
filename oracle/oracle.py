"""ctypes wrapper of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module.  It never backs a product code path.

Physics parity vs the reference (PhysX inside Isaac Gym) is UNPINNED; see the
header of physics_oracle.c and DESIGN.md section 4.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


class OModel(C.Structure):
    _fields_ = [("nb", C.c_int32), ("nd", C.c_int32), ("nc", C.c_int32), ("ns", C.c_int32),
                ("fixed_base", C.c_int32)] + [
        (n, C.c_void_p) for n in ("parent", "jkind", "bdof", "jorigin", "jaxis", "mass", "com", "inertia",
                                  "cbody", "cpoint", "cradius", "cshape", "effort", "vmax", "armature",
                                  "lower", "upper", "has_limits")] + [
        ("nsens", C.c_int32), ("sens_body", C.c_void_p), ("nr", C.c_int32), ("clink", C.c_void_p),
        ("dkp", C.c_void_p), ("dkd", C.c_void_p)] + [
        (n, C.c_void_p) for n in ("cdyn", "shkind", "shbody", "shlink", "shpose", "shsize", "shmargin", "shsphere",
                                  "hverts", "shv0", "shv1")] + [
        ("npair", C.c_int32), ("pair_a", C.c_void_p), ("pair_b", C.c_void_p), ("pair_kind", C.c_void_p),
        ("npool", C.c_int32), ("self_collide", C.c_int32), ("pverts", C.c_void_p), ("shp0", C.c_void_p),
        ("shp1", C.c_void_p), ("pool_policy", C.c_int32)]


class OParams(C.Structure):
    _fields_ = [("dt", C.c_double), ("substeps", C.c_int32), ("gravity", C.c_double * 3),
                ("pos_iters", C.c_int32), ("vel_iters", C.c_int32), ("contact_offset", C.c_double),
                ("rest_offset", C.c_double), ("max_depen_vel", C.c_double), ("collect_contacts", C.c_int32),
                ("has_ground", C.c_int32), ("ground_friction", C.c_double), ("limit_margin", C.c_double),
                ("has_terrain", C.c_int32), ("trows", C.c_int32), ("tcols", C.c_int32), ("tverts", C.c_void_p),
                ("tx0", C.c_double), ("ty0", C.c_double), ("ths", C.c_double), ("terrain_friction", C.c_double),
                ("solver_type", C.c_int32)]


def build(quiet: bool = True) -> None:
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)


_LIBS = {}


def _lib(real_bits: int):
    if real_bits not in _LIBS:
        path = os.path.join(HERE, f"liboracle{real_bits}.so")
        if not os.path.exists(path):
            build()
        lib = C.CDLL(path)
        lib.oracle_simulate.restype = C.c_int
        lib.oracle_simulate.argtypes = [C.POINTER(OModel), C.POINTER(OParams), C.c_int] + [C.c_void_p] * 6 + [C.c_int]
        lib.oracle_simulate_targets.restype = C.c_int
        lib.oracle_simulate_targets.argtypes = [C.POINTER(OModel), C.POINTER(OParams), C.c_int] + \
            [C.c_void_p] * 6 + [C.c_int, C.c_void_p, C.c_void_p]
        lib.oracle_self_contacts.restype = C.c_int
        lib.oracle_self_contacts.argtypes = [C.POINTER(OModel), C.POINTER(OParams), C.c_int] + [C.c_void_p] * 5
        lib.oracle_hull_select.restype = C.c_int
        lib.oracle_hull_select.argtypes = [C.POINTER(OModel), C.POINTER(OParams), C.c_int] + [C.c_void_p] * 2 + \
            [C.c_double if real_bits == 64 else C.c_float, C.c_void_p]
        lib.oracle_terrain_query.restype = C.c_int
        lib.oracle_terrain_query.argtypes = [C.POINTER(OParams), C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        _LIBS[real_bits] = lib
    return _LIBS[real_bits]


class OracleSim:
    """Holds the model arrays alive and steps numpy state in place."""

    def __init__(self, flat: dict, params: dict, real_bits: int = 64, sensor_bodies=(), terrain=None, drives=None,
                 self_collide=None, pool_policy: int = 0):
        """terrain: optional dict(vertices float32 [rows*cols, 3] world coordinates, rows, cols, x0, y0,
        hs, friction) -- the heightfield-grid mesh of gym.add_triangle_mesh.
        drives: optional (kp [nd], kd [nd]) joint-drive gains.
        self_collide: the actor's collision filter is 0 (self-collision pairs); None follows
        flat["self_collide"] (absent: off).
        pool_policy: 0 the product's self-contact rules; see OModel.pool_policy."""
        self.flat = flat
        self.real = np.float64 if real_bits == 64 else np.float32
        self.lib = _lib(real_bits)
        keep = {}
        m = OModel()
        for k in ("nb", "nd", "nc", "ns", "fixed_base"):
            setattr(m, k, int(flat[k]))
        m.nr = int(flat.get("nr", flat["nb"]))
        for k in ("parent", "jkind", "bdof", "cbody", "cshape", "has_limits", "clink", "cdyn", "shkind", "shbody",
                  "shlink", "shv0", "shv1", "pair_a", "pair_b", "pair_kind", "shp0", "shp1"):
            a = np.ascontiguousarray(flat[k], dtype=np.int32)
            keep[k] = a
            setattr(m, k, a.ctypes.data)
        for k in ("jorigin", "jaxis", "mass", "com", "inertia", "cpoint", "cradius", "effort", "vmax", "armature",
                  "lower", "upper", "shpose", "shsize", "shmargin", "shsphere", "hverts", "pverts"):
            a = np.ascontiguousarray(flat[k], dtype=np.float64)
            keep[k] = a
            setattr(m, k, a.ctypes.data)
        if drives is not None:
            for k, a in zip(("dkp", "dkd"), drives):
                a = np.ascontiguousarray(a, dtype=np.float64)
                assert a.shape == (int(flat["nd"]),)
                keep[k] = a
                setattr(m, k, a.ctypes.data)
        m.npair = int(flat["npair"])
        m.npool = int(flat["npool"])
        m.self_collide = int(bool(flat.get("self_collide", 0) if self_collide is None else self_collide))
        # DESIGN.md 3.12's self-contact departures as switches (tools/pool_policy_study.py): bit 0 overlapping cores
        # make a contact, bit 1 no MIN_RESPONSE bound; 0 = the product's rules
        m.pool_policy = int(pool_policy)
        sb = np.ascontiguousarray(list(sensor_bodies) or [0], dtype=np.int32)
        keep["sens_body"] = sb
        m.nsens = len(sensor_bodies)
        m.sens_body = sb.ctypes.data
        self.nsens = len(sensor_bodies)
        self._keep = keep
        self.model = m
        p = OParams()
        p.dt = params["dt"]
        p.substeps = params["substeps"]
        for i in range(3):
            p.gravity[i] = params["gravity"][i]
        p.pos_iters = params["pos_iters"]
        p.vel_iters = params["vel_iters"]
        p.solver_type = int(params.get("solver_type", 0))
        p.contact_offset = params["contact_offset"]
        p.rest_offset = params["rest_offset"]
        p.max_depen_vel = params["max_depen_vel"]
        p.collect_contacts = params.get("collect_contacts", 1)
        p.has_ground = params.get("has_ground", 1)
        p.ground_friction = params.get("ground_friction", 1.0)
        p.limit_margin = params.get("limit_margin", 0.1)
        if terrain is not None:
            tv = np.ascontiguousarray(terrain["vertices"], dtype=np.float32).reshape(-1)
            keep["tverts"] = tv
            p.has_terrain = 1
            p.trows, p.tcols = int(terrain["rows"]), int(terrain["cols"])
            p.tverts = tv.ctypes.data
            p.tx0, p.ty0, p.ths = float(terrain["x0"]), float(terrain["y0"]), float(terrain["hs"])
            p.terrain_friction = float(terrain.get("friction", 1.0))
        self.params = p

    def terrain_query(self, centres, radii):
        """The mesh contact query alone: [n][5] = (found, separation, normal xyz)."""
        c = np.ascontiguousarray(centres, dtype=self.real)
        r = np.ascontiguousarray(radii, dtype=self.real)
        out = np.zeros((c.shape[0], 5), dtype=self.real)
        if self.lib.oracle_terrain_query(C.byref(self.params), c.shape[0], c.ctypes.data, r.ctypes.data,
                                         out.ctypes.data) != 0:
            raise RuntimeError("oracle_terrain_query: no terrain")
        return out

    def hull_select(self, shape: int, R, P, rootz: float):
        """Indices (into flat["hverts"]) of hull shape `shape`'s ground contact vertices for body pose R, P
        (relative to the root origin) and root height rootz (test hook)."""
        Ra = np.ascontiguousarray(R, dtype=self.real).reshape(9)
        Pa = np.ascontiguousarray(P, dtype=self.real).reshape(3)
        sel = np.zeros(4, dtype=np.int32)
        n = self.lib.oracle_hull_select(C.byref(self.model), C.byref(self.params), shape, Ra.ctypes.data,
                                        Pa.ctypes.data, rootz, sel.ctypes.data)
        if n < 0:
            raise RuntimeError("oracle_hull_select: not a hull shape")
        return sel[:n].copy()

    def self_contacts(self, root, dof, mu):
        """The self-contact pool of each env's state (test hook): (contacts [n, npool, 10] = x xyz, n xyz,
        separation, friction, body a, body b; counts [n])."""
        n = root.shape[0]
        npool = max(1, int(self.model.npool))
        out = np.zeros((n, npool, 10), dtype=self.real)
        cnt = np.zeros(n, dtype=np.int32)
        args = [np.ascontiguousarray(a, dtype=self.real) for a in (root, dof, mu)]
        if self.lib.oracle_self_contacts(C.byref(self.model), C.byref(self.params), n, *(a.ctypes.data for a in args),
                                         out.ctypes.data, cnt.ctypes.data) != 0:
            raise RuntimeError("oracle_self_contacts failed")
        return out, cnt

    def simulate(self, root, dof, tau, mu, cf=None, num_threads: int = 1, sens=None, pos_targets=None,
                 vel_targets=None) -> None:
        opt = tuple(a for a in (cf, sens, pos_targets, vel_targets) if a is not None)
        for a in (root, dof, tau, mu) + opt:
            assert a.dtype == self.real and a.flags.c_contiguous
        n = root.shape[0]
        rc = self.lib.oracle_simulate_targets(C.byref(self.model), C.byref(self.params), n, root.ctypes.data,
                                              dof.ctypes.data, tau.ctypes.data, mu.ctypes.data,
                                              cf.ctypes.data if cf is not None else None,
                                              sens.ctypes.data if sens is not None else None, num_threads,
                                              pos_targets.ctypes.data if pos_targets is not None else None,
                                              vel_targets.ctypes.data if vel_targets is not None else None)
        if rc != 0:
            raise RuntimeError(f"oracle_simulate failed rc={rc}")
