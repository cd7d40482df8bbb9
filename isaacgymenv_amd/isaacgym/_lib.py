"""ctypes binding of libgymsim.so (include/gymsim.h).

There is no fallback: if the library is missing every call raises, and a GPU
sim without a GPU fails at gs_sim_create.  The library's host backend
(gs_sim_create with device < 0, gs_host.hip) is the product's sim_device=cpu
pipeline -- the same solver source on host buffers, not a fallback.  (The CPU
oracle under oracle/ is test infrastructure and is never loaded from here.)
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# GS_LIBGYMSIM=libgymsim_prof.so selects the phase-profiling build (tools/phase_profile.py)
LIB_PATH = os.path.join(_HERE, "_lib", os.environ.get("GS_LIBGYMSIM", "libgymsim.so"))


class GsModelDesc(C.Structure):
    _fields_ = [("num_bodies", C.c_int32), ("num_dofs", C.c_int32), ("num_candidates", C.c_int32),
                ("num_shapes", C.c_int32), ("fixed_base", C.c_int32)] + [
        (n, C.c_void_p) for n in ("parent", "joint_kind", "body_dof", "joint_origin", "joint_axis", "mass",
                                  "com", "inertia", "cand_body", "cand_point", "cand_radius", "cand_shape",
                                  "dof_effort", "dof_velocity", "dof_armature", "dof_lower", "dof_upper",
                                  "dof_has_limits")] + [
        ("num_links", C.c_int32)] + [(n, C.c_void_p) for n in ("cand_link", "link_body", "link_pose", "link_com")] + [
        (n, C.c_void_p) for n in ("cand_dyn", "shape_kind", "shape_body", "shape_link", "shape_pose", "shape_size",
                                  "shape_margin", "shape_sphere")] + [
        ("num_hull_verts", C.c_int32), ("hull_verts", C.c_void_p), ("shape_hv0", C.c_void_p),
        ("shape_hv1", C.c_void_p), ("num_pairs", C.c_int32), ("pair_a", C.c_void_p), ("pair_b", C.c_void_p),
        ("pair_kind", C.c_void_p), ("pair_pool", C.c_int32), ("num_pair_verts", C.c_int32), ("pair_verts", C.c_void_p),
        ("shape_pv0", C.c_void_p), ("shape_pv1", C.c_void_p)]


class GsSimParams(C.Structure):
    _fields_ = [("dt", C.c_double), ("substeps", C.c_int32), ("gravity", C.c_double * 3),
                ("num_position_iterations", C.c_int32), ("num_velocity_iterations", C.c_int32),
                ("contact_offset", C.c_double), ("rest_offset", C.c_double),
                ("bounce_threshold_velocity", C.c_double), ("max_depenetration_velocity", C.c_double),
                ("contact_collection", C.c_int32), ("kernel_variant", C.c_int32),
                ("joint_limit_margin", C.c_double), ("num_threads", C.c_int32),
                ("solver_type", C.c_int32)]


class GsPdArgs(C.Structure):
    _fields_ = [("actions", C.c_void_p), ("default_pos", C.c_void_p), ("kp", C.c_float), ("kd", C.c_float),
                ("action_scale", C.c_float), ("torque_limit", C.c_float), ("decimation", C.c_int32),
                ("extra_simulates", C.c_int32), ("torques_out", C.c_void_p), ("dof_state_out", C.c_void_p),
                ("root_state_out", C.c_void_p), ("contact_out", C.c_void_p), ("actions_copy_out", C.c_void_p),
                # ABI 9: the AnymalTerrain tail (gymtask.h gt_anymal_params / gt_anymal_buffers) or NULL
                ("tail_params", C.c_void_p), ("tail_buffers", C.c_void_p)]


_lib = None


GS_ABI = 9  # include/gymsim.h GS_ABI_VERSION this binding's structs follow


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m isaacgymenv_amd.build` "
                               "(hipcc, gfx950). There is no CPU fallback.")
        L = C.CDLL(LIB_PATH)
        L.gs_abi_version.restype = C.c_int
        if L.gs_abi_version() != GS_ABI:
            raise RuntimeError(f"{LIB_PATH} has gymsim ABI {L.gs_abi_version()}, this binding needs {GS_ABI}: "
                               "rebuild it with `python -m isaacgymenv_amd.build`")
        vp, i, f, d = C.c_void_p, C.c_int, C.c_float, C.c_double
        sig = {
            "gs_abi_version": (i, []),
            "gs_last_error": (C.c_char_p, []),
            "gs_topology_supported": (i, [C.POINTER(GsModelDesc)]),
            "gs_sim_create": (vp, [i, C.POINTER(GsSimParams)]),
            "gs_sim_destroy": (None, [vp]),
            "gs_sim_add_ground": (i, [vp, d, d, d]),
            "gs_sim_set_model": (i, [vp, C.POINTER(GsModelDesc)]),
            "gs_sim_prepare": (i, [vp, i, vp, vp, vp]),
            "gs_sim_simulate": (i, [vp, vp, vp]),
            "gs_sim_refresh_root": (i, [vp, vp, vp]),
            "gs_sim_refresh_dof": (i, [vp, vp, vp]),
            "gs_sim_refresh_contact": (i, [vp, vp, vp]),
            "gs_sim_refresh_rigid_body": (i, [vp, vp, vp]),
            "gs_sim_refresh_jacobian": (i, [vp, vp, vp]),
            "gs_sim_refresh_mass_matrix": (i, [vp, vp, vp]),
            "gs_sim_set_root": (i, [vp, vp, vp, i, vp]),
            "gs_sim_set_dof": (i, [vp, vp, vp, i, vp]),
            "gs_sim_pd_step": (i, [vp, C.POINTER(GsPdArgs), vp]),
            "gs_sim_kernel_variant": (i, [vp]),
            "gs_sim_enable_timing": (i, [vp, i]),
            "gs_sim_last_kernel_ms": (f, [vp]),
            "gs_debug_phase_cycles": (i, [vp, i, i]),
            "gs_sim_set_force_sensors": (i, [vp, i, vp]),
            "gs_sim_bind_force_sensors": (i, [vp, vp]),
            "gs_sim_set_dof_drives": (i, [vp, vp, vp, vp]),
            "gs_sim_bind_dof_targets": (i, [vp, vp, vp]),
            "gs_sim_bind_dof_properties_env": (i, [vp, vp, i, i]),
            "gs_sim_pd_tail_supported": (i, [vp]),
            "gs_sim_set_root_and_dof": (i, [vp, vp, vp, vp, i, vp]),
            "gs_sim_set_self_collision": (i, [vp, i]),
            "gs_sim_refresh_force_sensor": (i, [vp, vp, vp]),
            "gs_sim_add_triangle_mesh": (i, [vp, vp, C.c_int64, vp, C.c_int64, vp, d, d, d]),
            "gs_debug_terrain_query": (i, [vp, vp, vp, i, vp, vp]),
            "gs_debug_self_contacts": (i, [vp, i, vp, vp, vp]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed: {lib().gs_last_error().decode()}")


EXPORTED_SYMBOLS = [
    "gs_abi_version", "gs_last_error", "gs_topology_supported", "gs_sim_create", "gs_sim_destroy",
    "gs_sim_add_ground", "gs_sim_set_model", "gs_sim_prepare", "gs_sim_simulate", "gs_sim_refresh_root",
    "gs_sim_refresh_dof", "gs_sim_refresh_contact", "gs_sim_set_root", "gs_sim_set_dof", "gs_sim_pd_step",
    "gs_sim_kernel_variant", "gs_sim_enable_timing", "gs_sim_last_kernel_ms", "gs_debug_phase_cycles",
    "gs_sim_set_force_sensors", "gs_sim_bind_force_sensors", "gs_sim_refresh_force_sensor",
    "gs_sim_add_triangle_mesh", "gs_debug_terrain_query", "gs_sim_refresh_rigid_body", "gs_sim_refresh_jacobian",
    "gs_sim_refresh_mass_matrix", "gs_sim_set_dof_drives", "gs_sim_bind_dof_targets", "gs_sim_set_self_collision",
    "gs_debug_self_contacts", "gs_sim_bind_dof_properties_env", "gs_sim_pd_tail_supported", "gs_sim_set_root_and_dof",
]


def model_desc(flat: dict):
    """Build a GsModelDesc over the numpy arrays of ``_model.flatten``; returns (desc, keepalive)."""
    import numpy as np
    keep = {}
    m = GsModelDesc()
    m.num_bodies, m.num_dofs, m.num_candidates = flat["nb"], flat["nd"], flat["nc"]
    m.num_shapes, m.fixed_base = flat["ns"], flat["fixed_base"]
    pairs = [("parent", "parent", np.int32), ("joint_kind", "jkind", np.int32), ("body_dof", "bdof", np.int32),
             ("joint_origin", "jorigin", np.float64), ("joint_axis", "jaxis", np.float64),
             ("mass", "mass", np.float64), ("com", "com", np.float64), ("inertia", "inertia", np.float64),
             ("cand_body", "cbody", np.int32), ("cand_point", "cpoint", np.float64),
             ("cand_radius", "cradius", np.float64), ("cand_shape", "cshape", np.int32),
             ("dof_effort", "effort", np.float64), ("dof_velocity", "vmax", np.float64),
             ("dof_armature", "armature", np.float64), ("dof_lower", "lower", np.float64),
             ("dof_upper", "upper", np.float64), ("dof_has_limits", "has_limits", np.int32),
             ("cand_link", "clink", np.int32), ("link_body", "lbody", np.int32),
             ("link_pose", "lpose", np.float64), ("link_com", "lcom", np.float64),
             ("cand_dyn", "cdyn", np.int32), ("shape_kind", "shkind", np.int32), ("shape_body", "shbody", np.int32),
             ("shape_link", "shlink", np.int32), ("shape_pose", "shpose", np.float64),
             ("shape_size", "shsize", np.float64), ("shape_margin", "shmargin", np.float64),
             ("shape_sphere", "shsphere", np.float64), ("hull_verts", "hverts", np.float64),
             ("shape_hv0", "shv0", np.int32), ("shape_hv1", "shv1", np.int32), ("pair_a", "pair_a", np.int32),
             ("pair_b", "pair_b", np.int32), ("pair_kind", "pair_kind", np.int32), ("pair_verts", "pverts", np.float64),
             ("shape_pv0", "shp0", np.int32), ("shape_pv1", "shp1", np.int32)]
    m.num_links = flat["nr"]
    m.num_hull_verts = len(flat["hverts"])
    m.num_pairs = int(flat["npair"])
    m.pair_pool = int(flat["npool"])
    m.num_pair_verts = len(flat["pverts"])
    for field, key, dt in pairs:
        a = np.ascontiguousarray(flat[key], dtype=dt)
        if a.size == 0:
            a = np.zeros(1, dtype=dt)
        keep[field] = a
        setattr(m, field, a.ctypes.data)
    return m, keep
