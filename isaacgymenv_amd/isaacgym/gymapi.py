"""Drop-in ``isaacgym.gymapi`` for the MI355X simulator.

The reference imports the closed Isaac Gym binding as
``from isaacgym import gymapi, gymtorch`` (vec_task.py:37) and drives the
simulator only through ``self.gym = gymapi.acquire_gym()`` (vec_task.py:247).
This module keeps that Python surface -- the constants, parameter classes and
``Gym`` methods the reference's task layer calls -- and
implements it over libgymsim.so (include/gymsim.h).  Env/actor bookkeeping is
host Python (cold path); everything per step is a HIP launch on the torch
stream of the sim device.

Scope notes:
  * one articulation actor per env, every env the same asset;
  * z-up ground plane contacts (trimesh/heightfield terrain is the next row);
  * ``sim_device=cpu`` (``physx.use_gpu`` False, vec_task.py:82-88 / the task YAMLs'
    ``use_gpu: ${contains:"cuda",${....sim_device}}``) runs the host backend of libgymsim --
    the same solver source on a thread pool of ``physx.num_threads`` threads, host tensors,
    no GPU needed; ``sim_device=cuda:k pipeline=cpu`` runs the GPU solver behind host-side
    tensors (staged copies), as Isaac Gym's PhysX GPU + CPU pipeline does.
"""
from __future__ import annotations

import ctypes as C
import enum
import math
import os
import warnings
from typing import List, Optional

import numpy as np

from . import _assets
from ._assets import build_articulation, load_raw, mat_to_quat_xyzw, quat_xyzw_to_mat
from ._model import flatten
from . import _lib
from isaacgymenv_amd._stream import raw_stream


class PhysicsDeviationWarning(UserWarning):
    """A requested PhysX feature the MI355X solver does not reproduce (DESIGN.md sections 3 and 6)."""


# ------------------------------------------------------------------ constants
SIM_PHYSX = 0
SIM_FLEX = 1
UP_AXIS_Y = 0
UP_AXIS_Z = 1
DOF_MODE_NONE = 0
DOF_MODE_POS = 1
DOF_MODE_VEL = 2
DOF_MODE_EFFORT = 3
DOF_INVALID = 0
DOF_ROTATION = 1
DOF_TRANSLATION = 2
STATE_NONE, STATE_POS, STATE_VEL, STATE_ALL = 0, 1, 2, 3
DOMAIN_SIM, DOMAIN_ENV, DOMAIN_ACTOR = 0, 1, 2
MESH_NONE, MESH_COLLISION, MESH_VISUAL, MESH_VISUAL_AND_COLLISION = 0, 1, 2, 3
IMAGE_COLOR, IMAGE_DEPTH = 0, 1
KEY_ESCAPE, KEY_V, KEY_R = 0, 1, 2
INVALID_HANDLE = -1


class ContactCollection(enum.IntEnum):
    CC_NEVER = 0
    CC_LAST_SUBSTEP = 1
    CC_ALL_SUBSTEPS = 2


# ------------------------------------------------------------------ value types
class Vec3:
    __slots__ = ("x", "y", "z")

    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x, self.y, self.z = float(x), float(y), float(z)

    def __iter__(self):
        return iter((self.x, self.y, self.z))

    def __repr__(self):
        return f"Vec3({self.x}, {self.y}, {self.z})"


class Quat:
    __slots__ = ("x", "y", "z", "w")

    def __init__(self, x=0.0, y=0.0, z=0.0, w=1.0):
        self.x, self.y, self.z, self.w = float(x), float(y), float(z), float(w)

    def __iter__(self):
        return iter((self.x, self.y, self.z, self.w))

    @staticmethod
    def from_axis_angle(axis: Vec3, angle: float) -> "Quat":
        s = math.sin(angle / 2)
        n = math.sqrt(axis.x ** 2 + axis.y ** 2 + axis.z ** 2) or 1.0
        return Quat(axis.x / n * s, axis.y / n * s, axis.z / n * s, math.cos(angle / 2))

    @staticmethod
    def from_euler_zyx(roll, pitch, yaw) -> "Quat":
        q = mat_to_quat_xyzw(_assets.rpy_to_mat([roll, pitch, yaw]))
        return Quat(*q)


class Transform:
    def __init__(self, p: Optional[Vec3] = None, r: Optional[Quat] = None):
        self.p = p if p is not None else Vec3()
        self.r = r if r is not None else Quat()


class PlaneParams:
    def __init__(self):
        self.normal = Vec3(0.0, 0.0, 1.0)
        self.distance = 0.0
        self.static_friction = 1.0
        self.dynamic_friction = 1.0
        self.restitution = 0.0
        self.segmentation_id = 0


class TriangleMeshParams:
    def __init__(self):
        self.nb_vertices = 0
        self.nb_triangles = 0
        self.transform = Transform()
        self.static_friction = 1.0
        self.dynamic_friction = 1.0
        self.restitution = 0.0


class PhysXParams:
    def __init__(self):
        self.num_threads = 4
        self.solver_type = 1
        self.use_gpu = True
        self.num_position_iterations = 4
        self.num_velocity_iterations = 1
        self.contact_offset = 0.02
        self.rest_offset = 0.001
        self.bounce_threshold_velocity = 0.2
        self.max_depenetration_velocity = 100.0
        self.default_buffer_size_multiplier = 2.0
        self.max_gpu_contact_pairs = 1024 * 1024
        self.num_subscenes = 0
        self.contact_collection = ContactCollection.CC_LAST_SUBSTEP
        self.friction_offset_threshold = 0.04
        self.friction_correlation_distance = 0.025
        self.always_use_articulations = False


class FlexParams:
    def __init__(self):
        self.__dict__["_values"] = {}

    def __setattr__(self, k, v):
        self._values[k] = v

    def __getattr__(self, k):
        try:
            return self.__dict__["_values"][k]
        except KeyError:
            raise AttributeError(k)


class SimParams:
    def __init__(self):
        self.dt = 1.0 / 60.0
        self.substeps = 2
        self.up_axis = UP_AXIS_Y
        self.gravity = Vec3(0.0, -9.8, 0.0)
        self.use_gpu_pipeline = False
        self.num_client_threads = 0
        self.enable_actor_creation_warning = False
        self.physx = PhysXParams()
        self.flex = FlexParams()


class AssetOptions:
    def __init__(self):
        d = _assets.DEFAULT_ASSET_OPTIONS
        self.default_dof_drive_mode = DOF_MODE_POS
        self.collapse_fixed_joints = d["collapse_fixed_joints"]
        self.replace_cylinder_with_capsule = d["replace_cylinder_with_capsule"]
        self.flip_visual_attachments = False
        self.fix_base_link = False
        self.density = d["density"]
        self.angular_damping = d["angular_damping"]
        self.linear_damping = d["linear_damping"]
        self.max_angular_velocity = d["max_angular_velocity"]
        self.max_linear_velocity = d["max_linear_velocity"]
        self.armature = 0.0
        self.thickness = d["thickness"]
        self.disable_gravity = False
        self.use_mesh_materials = False
        self.override_com = False
        self.override_inertia = False
        self.vhacd_enabled = False
        self.use_physx_armature = True
        self.slices_per_cylinder = 20

    def as_dict(self):
        return {k: getattr(self, k) for k in vars(self)}


class CameraProperties:
    def __init__(self):
        self.width, self.height, self.horizontal_fov, self.enable_tensors = 1920, 1080, 90.0, False


class RigidShapeProperties:
    def __init__(self, friction=1.0):
        self.friction = friction
        self.rolling_friction = 0.0
        self.torsion_friction = 0.0
        self.restitution = 0.0
        self.compliance = 0.0
        self.thickness = 0.0
        self.contact_offset = 0.0
        self.rest_offset = 0.0
        self.filter = 0


class ActuatorProperties:
    def __init__(self, motor_effort=0.0):
        self.motor_effort = motor_effort
        self.control_limited = False
        self.lower_control_limit = 0.0
        self.upper_control_limit = 0.0
        self.lower_force_limit = 0.0
        self.upper_force_limit = 0.0
        self.kp = 0.0
        self.kv = 0.0


DofPropertiesDtype = np.dtype([("hasLimits", "?"), ("lower", "<f4"), ("upper", "<f4"), ("driveMode", "<i4"),
                               ("velocity", "<f4"), ("effort", "<f4"), ("stiffness", "<f4"),
                               ("damping", "<f4"), ("friction", "<f4"), ("armature", "<f4")])


# ------------------------------------------------------------------ handles
class Asset:
    def __init__(self, art: _assets.Articulation, options: AssetOptions):
        self.art = art
        self.options = options
        self.flat = flatten(art, armature=options.armature)
        self.shape_props = [RigidShapeProperties(art.default_friction) for _ in range(art.num_shapes)]
        self.dof_props = self._default_dof_props()
        self.sensors = []

    def _default_dof_props(self):
        p = np.zeros(self.art.num_dofs, dtype=DofPropertiesDtype)
        for i, d in enumerate(self.art.dofs):
            p[i]["hasLimits"] = d.has_limits
            p[i]["lower"] = d.lower if d.has_limits else -3.4028235e38
            p[i]["upper"] = d.upper if d.has_limits else 3.4028235e38
            p[i]["driveMode"] = self.options.default_dof_drive_mode
            p[i]["velocity"] = d.velocity
            p[i]["effort"] = d.effort
            p[i]["friction"] = d.friction
            p[i]["damping"] = d.damping
            p[i]["armature"] = self.options.armature if d.armature is None else d.armature
        return p


class Env:
    def __init__(self, sim: "Sim", index: int, origin):
        self.sim = sim
        self.index = index
        self.origin = np.asarray(origin, dtype=np.float64)
        self.actors: List["Actor"] = []


class Actor:
    def __init__(self, env: Env, asset: Asset, pose: Transform, name: str, group: int, filter: int):
        self.env = env
        self.asset = asset
        self.pose = pose
        self.name = name
        self.group = group
        self.filter = filter
        self.shape_friction = np.array([sp.friction for sp in asset.shape_props], dtype=np.float32)
        self.dof_props = asset.dof_props.copy()


class GymTensor:
    """Descriptor handed out by ``acquire_*_tensor`` / ``gymtorch.unwrap_tensor``."""

    def __init__(self, tensor, kind: str = "user"):
        self.tensor = tensor
        self.kind = kind


JOINT_LIMIT_MARGIN = 0.1


def torch_empty_like_on(t, device):
    import torch
    return torch.empty(t.shape, dtype=t.dtype, device=device)


# ------------------------------------------------------------------ the sim
class Sim:
    def __init__(self, gym: "Gym", compute_device: int, params: SimParams):
        import torch
        self.gym = gym
        self.params = params
        self.compute_device = compute_device
        self.gpu_pipeline = bool(params.use_gpu_pipeline)
        # host backend: sim_device=cpu (physx.use_gpu False), or no HIP device to run on
        self.host = not bool(params.physx.use_gpu)
        if self.host and self.gpu_pipeline:
            # as Isaac Gym, which cannot keep GPU-pipeline tensors with CPU PhysX: GPU physics
            print("*** the GPU pipeline needs GPU physics: ignoring physx.use_gpu=False")
            self.host = False
        if not self.host and not self.gpu_pipeline and not torch.cuda.is_available():
            print("*** no HIP device: running the physics on the CPU (host backend, physx.num_threads threads)")
            self.host = True
        self.sim_device = torch.device("cpu") if self.host else torch.device("cuda", compute_device)
        self.tensor_device = self.sim_device if self.gpu_pipeline else torch.device("cpu")
        self.envs: List[Env] = []
        self.asset: Optional[Asset] = None
        self.ground: Optional[PlaneParams] = None
        self.mesh = None
        self.prepared = False
        self.drives_dirty = False
        self.handle = None
        self._pd_args, self._pd_key = None, None  # Gym.amd_pd_decimation_step's cached argument struct
        px = params.physx
        p = _lib.GsSimParams()
        p.dt = params.dt
        p.substeps = max(1, int(params.substeps))
        g = params.gravity
        p.gravity[0], p.gravity[1], p.gravity[2] = g.x, g.y, g.z
        p.num_position_iterations = int(px.num_position_iterations)
        p.num_velocity_iterations = int(px.num_velocity_iterations)
        p.contact_offset = float(px.contact_offset)
        p.rest_offset = float(px.rest_offset)
        p.bounce_threshold_velocity = float(px.bounce_threshold_velocity)
        p.max_depenetration_velocity = float(px.max_depenetration_velocity)
        p.contact_collection = int(px.contact_collection)
        # GS_PHYSICS_KERNEL=auto|lane|team selects the physics kernel form
        # (generic: the runtime-sized kernel even where a compiled topology exists -- gymsim.h kernel_variant 4)
        p.kernel_variant = {"auto": 0, "lane": 1, "team": 2, "generic": 4}[os.environ.get("GS_PHYSICS_KERNEL", "auto")]
        # a joint-limit row is generated within this distance of a limit (rad / m)
        p.joint_limit_margin = JOINT_LIMIT_MARGIN
        # PhysX CPU worker threads (cfg/config.yaml:30 num_threads: 4); 0 = the calling thread only
        p.num_threads = max(1, int(getattr(px, "num_threads", 0) or 0))
        # physx.solver_type (cfg/config.yaml:31): 1 = TGS (position iterations as sub-steps), 0 = PGS with split
        # impulse -- every kernel form and the host backend solve both
        p.solver_type = 1 if int(getattr(px, "solver_type", 0)) == 1 else 0
        self.cparams = p
        L = _lib.lib()
        h = L.gs_sim_create(-1 if self.host else int(compute_device), p)
        if not h:
            raise RuntimeError(L.gs_last_error().decode())
        self.handle = h

    def __del__(self):
        try:
            if self.handle:
                _lib.lib().gs_sim_destroy(self.handle)
        except Exception:
            pass

    # -------- stream of the sim device
    def stream(self):
        if self.host:
            return None  # host backend: every call completes before it returns
        import torch
        return raw_stream(self.sim_device)

    # -------- prepare: allocate + bind tensors, initial state
    def prepare(self):
        import torch
        if self.asset is None or not self.envs:
            raise RuntimeError("prepare_sim: no actors were created")
        for e in self.envs:
            if len(e.actors) != 1 or e.actors[0].asset is not self.asset:
                raise RuntimeError("prepare_sim: the MI355X simulator supports exactly one actor of one asset "
                                   "per env (DESIGN.md section 6)")
        art, flat = self.asset.art, self.asset.flat
        L = _lib.lib()
        desc, keep = _lib.model_desc(flat)
        if self.mesh is not None:
            v, t, tp, smu, dmu, rest = self.mesh
            tpa = (C.c_double * 3)(*tp)
            _lib.check(L.gs_sim_add_triangle_mesh(self.handle, v.ctypes.data, v.size // 3, t.ctypes.data, t.size // 3,
                                                  tpa, smu, dmu, rest), "gs_sim_add_triangle_mesh")
        _lib.check(L.gs_sim_set_model(self.handle, desc), "gs_sim_set_model")
        # collision filter 0: Isaac Gym collides the actor's own shapes
        filters = {a.filter == 0 for e in self.envs for a in e.actors}
        if len(filters) > 1:
            raise NotImplementedError("actors with and without self-collision (collision filter 0) in one sim "
                                      "(DESIGN.md section 6)")
        # (GS_SELF_COLLIDE=0 turns the pairs off: an A/B knob for measurements, not a product setting)
        self.self_collide = bool(filters.pop()) and int(flat["npair"]) > 0 and os.environ.get("GS_SELF_COLLIDE", "1") != "0"
        _lib.check(L.gs_sim_set_self_collision(self.handle, int(self.self_collide)), "gs_sim_set_self_collision")
        sens = [b for b, _ in self.asset.sensors]
        if sens:
            sb = np.ascontiguousarray(sens, dtype=np.int32)
            _lib.check(L.gs_sim_set_force_sensors(self.handle, len(sens), sb.ctypes.data), "gs_sim_set_force_sensors")
        if self.ground is not None:
            _lib.check(L.gs_sim_add_ground(self.handle, self.ground.static_friction, self.ground.dynamic_friction,
                                           self.ground.restitution), "gs_sim_add_ground")
        self._tensors()
        N, nd, nb, ns = self.num_envs, self.num_dofs, self.num_bodies, max(1, art.num_shapes)
        dev, tdev = self.sim_device, self.tensor_device
        f32 = torch.float32
        # SoA sim state (device), initial values from the actors' start poses
        st = np.zeros((13 + 2 * nd, N), dtype=np.float32)
        for i, e in enumerate(self.envs):
            a = e.actors[0]
            st[0:3, i] = e.origin + np.array(list(a.pose.p))
            q = np.array(list(a.pose.r), dtype=np.float64)
            st[3:7, i] = q / np.linalg.norm(q)
            # dof positions start at 0, clamped into their limits
            lo = a.dof_props["lower"].astype(np.float64)
            hi = a.dof_props["upper"].astype(np.float64)
            st[13:13 + nd, i] = np.clip(0.0, lo, hi)
        self.state = torch.from_numpy(st).to(dev)
        mu = np.ones((ns, N), dtype=np.float32)
        for i, e in enumerate(self.envs):
            mu[:art.num_shapes, i] = e.actors[0].shape_friction
        self.shape_mu = torch.from_numpy(mu).to(dev)
        self.cf_soa = torch.zeros(3 * nb, N, dtype=f32, device=dev)
        _lib.check(L.gs_sim_prepare(self.handle, N, self.state.data_ptr(), self.shape_mu.data_ptr(),
                                    self.cf_soa.data_ptr()), "gs_sim_prepare")
        self._keep = keep
        self.kernel_variant = L.gs_sim_kernel_variant(self.handle)
        self.num_sensors = len(sens)
        self.sens_soa = torch.zeros(max(1, 6 * len(sens)), N, dtype=f32, device=dev)
        if sens:
            _lib.check(L.gs_sim_bind_force_sensors(self.handle, self.sens_soa.data_ptr()), "gs_sim_bind_force_sensors")
        self.sensor_tensor = torch.zeros(N * len(sens), 6, dtype=f32, device=tdev)
        self.dof_force = torch.zeros(N * nd, dtype=f32, device=dev)
        # joint-drive targets (set_dof_position/velocity_target_tensor), bound once; the gains come
        # from the actors' dof properties (DOF_MODE_POS / DOF_MODE_VEL with stiffness / damping)
        self.pos_target = torch.zeros(N * nd, dtype=f32, device=dev)
        self.vel_target = torch.zeros(N * nd, dtype=f32, device=dev)
        _lib.check(L.gs_sim_bind_dof_targets(self.handle, self.pos_target.data_ptr(), self.vel_target.data_ptr()),
                   "gs_sim_bind_dof_targets")
        self.apply_drives()
        # device mirrors used when the pipeline is on the CPU and the physics on the GPU
        if not self.gpu_pipeline and not self.host:
            self._root_dev = torch.zeros(N, 13, dtype=f32, device=dev)
            self._dof_dev = torch.zeros(N * nd, 2, dtype=f32, device=dev)
            self._cf_dev = torch.zeros(N * nb, 3, dtype=f32, device=dev)
            self._sens_dev = torch.zeros(N * len(sens), 6, dtype=f32, device=dev)
        self.prepared = True
        self.refresh("root")
        self.refresh("dof")
        self.refresh("contact")
        for kind in ("rigid_body", "jacobian", "mass_matrix"):  # acquired before prepare_sim
            self.refresh(kind)

    def _effective_dof_props(self, p):
        """(kp, kd, effort, lower, upper, velocity) float64 [nd] of one actor's dof properties as the solver reads
        them: stiffness only where driveMode is POS, damping where it is POS or VEL (EFFORT / NONE dofs ignore
        both, as gs_sim_set_dof_drives does); a dof without limits has lower = upper = 0."""
        mode = p["driveMode"].astype(np.int32)
        pos, vel = mode == int(DOF_MODE_POS), mode == int(DOF_MODE_VEL)
        lim = p["hasLimits"].astype(bool) & (p["upper"].astype(np.float64) > p["lower"].astype(np.float64))
        return (np.where(pos, p["stiffness"].astype(np.float64), 0.0),
                np.where(pos | vel, p["damping"].astype(np.float64), 0.0),
                p["effort"].astype(np.float64),
                np.where(lim, p["lower"].astype(np.float64), 0.0),
                np.where(lim, p["upper"].astype(np.float64), 0.0),
                p["velocity"].astype(np.float64))

    def _asset_dof_props(self):
        """The asset's values the model was built with (gs_sim_set_model), in _effective_dof_props' layout."""
        flat = self.asset.flat
        nd = int(flat["nd"])
        lim = np.asarray(flat["has_limits"], dtype=bool)[:nd] & (np.asarray(flat["upper"])[:nd] > np.asarray(flat["lower"])[:nd])
        return (np.asarray(flat["effort"], dtype=np.float64)[:nd],
                np.where(lim, np.asarray(flat["lower"], dtype=np.float64)[:nd], 0.0),
                np.where(lim, np.asarray(flat["upper"], dtype=np.float64)[:nd], 0.0),
                np.asarray(flat["vmax"], dtype=np.float64)[:nd])

    def drive_tables(self):
        """(mode int32 [nd], stiffness [nd], damping [nd]) of the first actor's dof properties: the asset-wide
        drive setting (gs_sim_set_dof_drives).  Actors whose properties differ get the per-actor table on top
        (dof_property_table)."""
        p = self.envs[0].actors[0].dof_props
        return (p["driveMode"].astype(np.int32), p["stiffness"].astype(np.float64), p["damping"].astype(np.float64))

    def dof_property_table(self):
        """[GS_DOFP_FIELDS = 6][nd][N] float32 of the actors' properties (gymsim.h gs_sim_bind_dof_properties_env),
        or None when every actor's effective drive gains equal the first actor's and its effort, limits and
        velocity limit the asset's (the uniform path: the asset model + gs_sim_set_dof_drives).  Isaac Gym keeps
        dof properties per actor (set_actor_dof_properties, anymal_terrain.py:283, useful_hound.py:422)."""
        props = [self._effective_dof_props(e.actors[0].dof_props) for e in self.envs]
        asset = self._asset_dof_props()
        first = props[0]
        uniform = all(all(np.array_equal(x, y) for x, y in zip(first[:2], q[:2])) for q in props[1:]) and \
            all(np.array_equal(np.float32(x), np.float32(y)) for q in props for x, y in zip(q[2:], asset))
        if uniform:
            return None
        tab = np.stack([np.stack(q, axis=0) for q in props], axis=-1).astype(np.float32)  # [6][nd][N]
        return np.ascontiguousarray(tab)

    def apply_drives(self):
        """Upload the drive gains (gs_sim_set_dof_drives) and, where actors differ, the per-actor property table
        (gs_sim_bind_dof_properties_env); called at prepare_sim and whenever dof properties change afterwards
        (set_actor_dof_properties)."""
        import torch
        self.drives_dirty = False
        mode, kp, kd = self.drive_tables()
        mode, kp, kd = (np.ascontiguousarray(x) for x in (mode, kp, kd))
        L = _lib.lib()
        _lib.check(L.gs_sim_set_dof_drives(self.handle, mode.ctypes.data, kp.ctypes.data, kd.ctypes.data),
                   "gs_sim_set_dof_drives")
        tab = self.dof_property_table()
        if tab is None:
            self.dof_env_table = None
            _lib.check(L.gs_sim_bind_dof_properties_env(self.handle, None, 0, 0), "gs_sim_bind_dof_properties_env")
        else:
            any_drive = int(bool(np.any(tab[0] > 0) or np.any(tab[1] > 0)))
            any_limits = int(bool(np.any(tab[3] < tab[4])))
            if not self.host:
                torch.cuda.synchronize(self.sim_device)  # (a launch still queued may read the previous table)
            self.dof_env_table = torch.from_numpy(tab).to(self.sim_device)
            _lib.check(L.gs_sim_bind_dof_properties_env(self.handle, self.dof_env_table.data_ptr(), any_drive,
                                                        any_limits), "gs_sim_bind_dof_properties_env")
        self.kernel_variant = L.gs_sim_kernel_variant(self.handle)

    def set_targets(self, kind: str, src, idx=None, n: int = 0):
        """Copy (or scatter, for the listed actor indices) a [N*nd] target tensor into the bound buffer."""
        import torch
        dst = self.pos_target if kind == "pos" else self.vel_target
        src = src.reshape(self.num_envs, self.num_dofs).to(self.sim_device, dtype=torch.float32)
        if idx is None:
            dst.view(self.num_envs, self.num_dofs).copy_(src)
            return
        ids = idx[:n].to(self.sim_device, dtype=torch.long) if n else idx.to(self.sim_device, dtype=torch.long)
        dst.view(self.num_envs, self.num_dofs)[ids] = src[ids]

    def _tensors(self):
        """Reference-layout tensors (sim owned; wrap_tensor shares them), sized from the created envs.
        Isaac Gym lets a task acquire them before prepare_sim (useful_hound.py:438-455 does, inside
        _create_envs) and they are the same buffers afterwards, so they are allocated once, here."""
        import torch
        if getattr(self, "root_tensor", None) is not None:
            return
        if self.asset is None or not self.envs:
            raise RuntimeError("tensors are available once the envs and actors exist")
        art = self.asset.art
        # num_bodies = reported rigid bodies (links); the dynamics may weld fixed-joint links
        N, nd, nb = len(self.envs), art.num_dofs, art.num_links
        self.num_envs, self.num_dofs, self.num_bodies = N, nd, nb
        self.nv = nd + (0 if art.fixed_base else 6)
        f32, tdev = torch.float32, self.tensor_device
        self.root_tensor = torch.zeros(N, 13, dtype=f32, device=tdev)
        self.dof_tensor = torch.zeros(N * nd, 2, dtype=f32, device=tdev)
        self.contact_tensor = torch.zeros(N * nb, 3, dtype=f32, device=tdev)
        self.rb_tensor = self.jac_tensor = self.mm_tensor = None

    # -------- tensor API
    def kinematics_tensor(self, kind: str):
        """Sim-owned rigid-body-state / jacobian / mass-matrix tensors, allocated on first acquire
        and filled once (Isaac Gym's acquired tensors hold the prepared state)."""
        import torch
        self._tensors()
        f32, tdev = torch.float32, self.tensor_device
        N, nr, nv = self.num_envs, self.num_bodies, self.nv
        if kind == "rigid_body" and self.rb_tensor is None:
            self.rb_tensor = torch.zeros(N * nr, 13, dtype=f32, device=tdev)
        elif kind == "jacobian" and self.jac_tensor is None:
            self.jac_tensor = torch.zeros(N, nr, 6, nv, dtype=f32, device=tdev)
        elif kind == "mass_matrix" and self.mm_tensor is None:
            self.mm_tensor = torch.zeros(N, nv, nv, dtype=f32, device=tdev)
        else:
            return {"rigid_body": self.rb_tensor, "jacobian": self.jac_tensor, "mass_matrix": self.mm_tensor}[kind]
        if self.prepared:
            self.refresh(kind)
        return {"rigid_body": self.rb_tensor, "jacobian": self.jac_tensor, "mass_matrix": self.mm_tensor}[kind]

    def refresh(self, kind: str):
        L, s = _lib.lib(), self.stream()
        if kind in ("rigid_body", "jacobian", "mass_matrix"):
            dst = {"rigid_body": self.rb_tensor, "jacobian": self.jac_tensor, "mass_matrix": self.mm_tensor}[kind]
            if dst is None:
                return  # never acquired: nothing to fill
            out = dst if self.gpu_pipeline or self.host else torch_empty_like_on(dst, self.sim_device)
            fn = {"rigid_body": L.gs_sim_refresh_rigid_body, "jacobian": L.gs_sim_refresh_jacobian,
                  "mass_matrix": L.gs_sim_refresh_mass_matrix}[kind]
            _lib.check(fn(self.handle, out.data_ptr(), s), f"refresh {kind}")
            if out is not dst:
                dst.copy_(out.cpu())
            return
        dst = {"root": self.root_tensor, "dof": self.dof_tensor, "contact": self.contact_tensor,
               "sensor": self.sensor_tensor}[kind]
        out = dst if self.gpu_pipeline or self.host else {"root": self._root_dev, "dof": self._dof_dev,
                                                          "contact": self._cf_dev, "sensor": self._sens_dev}[kind]
        fn = {"root": L.gs_sim_refresh_root, "dof": L.gs_sim_refresh_dof, "contact": L.gs_sim_refresh_contact,
              "sensor": L.gs_sim_refresh_force_sensor}[kind]
        _lib.check(fn(self.handle, out.data_ptr(), s), f"refresh {kind}")
        if out is not dst:
            dst.copy_(out.cpu())

    def set_state(self, kind: str, src, idx=None, n: int = 0):
        import torch
        L, s = _lib.lib(), self.stream()
        dev = self.sim_device
        # (the per-reset call: tensors already on the sim's device, typed and contiguous skip the conversions)
        if not (src.dtype == torch.float32 and src.device == dev and src.is_contiguous()):
            src = src.to(dev, dtype=torch.float32).contiguous()
        idx_ptr = None
        if idx is not None:
            if not (idx.dtype == torch.int32 and idx.device == dev and idx.is_contiguous()):
                idx = idx.to(dev, dtype=torch.int32).contiguous()
            n = int(n) if n else idx.numel()
            idx_ptr = idx.data_ptr()
            if n == 0:
                return
        fn = L.gs_sim_set_root if kind == "root" else L.gs_sim_set_dof
        _lib.check(fn(self.handle, src.data_ptr(), idx_ptr, n, s), f"set {kind}")
        self._hold = (src, idx)  # keep alive until the launch consumed them (stream ordered)

    def set_root_and_dof(self, root, dof, idx, n: int = 0):
        """set_state("root", root, idx, n) then set_state("dof", dof, idx, n), one host call (a reset's pair)."""
        import torch
        L, s = _lib.lib(), self.stream()
        dev = self.sim_device
        if not (root.dtype == torch.float32 and root.device == dev and root.is_contiguous()):
            root = root.to(dev, dtype=torch.float32).contiguous()
        if not (dof.dtype == torch.float32 and dof.device == dev and dof.is_contiguous()):
            dof = dof.to(dev, dtype=torch.float32).contiguous()
        if not (idx.dtype == torch.int32 and idx.device == dev and idx.is_contiguous()):
            idx = idx.to(dev, dtype=torch.int32).contiguous()
        n = int(n) if n else idx.numel()
        if n == 0:
            return
        _lib.check(L.gs_sim_set_root_and_dof(self.handle, root.data_ptr(), dof.data_ptr(), idx.data_ptr(), n, s),
                   "set root and dof")
        self._hold = (root, dof, idx)

    def simulate(self):
        L = _lib.lib()
        if self.drives_dirty:
            self.apply_drives()
        _lib.check(L.gs_sim_simulate(self.handle, self.dof_force.data_ptr(), self.stream()), "gs_sim_simulate")


# ------------------------------------------------------------------ Gym
class Gym:
    """The object returned by ``acquire_gym()`` (vec_task.py:247)."""

    # ---- sim lifecycle
    def create_sim(self, compute_device: int = 0, graphics_device: int = -1, type: int = SIM_PHYSX,
                   params: Optional[SimParams] = None):
        if type != SIM_PHYSX:
            raise ValueError("only SIM_PHYSX semantics are implemented")
        try:
            return Sim(self, compute_device, params or SimParams())
        except Exception as exc:  # reference callers test for None (vec_task.py:338)
            print(f"*** gs_sim_create failed: {exc}")
            return None

    def destroy_sim(self, sim: Sim):
        sim.__del__()
        sim.handle = None

    def get_sim_params(self, sim: Sim) -> SimParams:
        return sim.params

    def set_sim_params(self, sim: Sim, params: SimParams):
        sim.params = params

    def prepare_sim(self, sim: Sim) -> bool:
        sim.prepare()
        return True

    def simulate(self, sim: Sim):
        sim.simulate()

    def fetch_results(self, sim: Sim, wait: bool = True):
        if wait and not sim.gpu_pipeline and not sim.host:
            import torch
            torch.cuda.synchronize(sim.sim_device)

    def get_sim_time(self, sim: Sim) -> float:
        return 0.0

    # ---- world geometry
    def add_ground(self, sim: Sim, params: PlaneParams):
        n = params.normal
        if abs(n.z - 1.0) > 1e-6 or abs(n.x) > 1e-6 or abs(n.y) > 1e-6 or params.distance != 0.0:
            raise NotImplementedError("only the z-up ground plane through the origin is supported")
        sim.ground = params

    def add_triangle_mesh(self, sim: Sim, vertices, triangles, params: TriangleMeshParams):
        """A static heightfield-grid mesh (terrain_utils.convert_heightfield_to_trimesh layout,
        anymal_terrain.py:196-208); translation-only transform.  Handed to libgymsim at prepare_sim."""
        r = params.transform.r
        if abs(r.x) > 1e-9 or abs(r.y) > 1e-9 or abs(r.z) > 1e-9 or abs(abs(r.w) - 1.0) > 1e-9:
            raise NotImplementedError("add_triangle_mesh: only translated (unrotated) meshes are supported")
        if sim.mesh is not None:
            raise NotImplementedError("add_triangle_mesh: one triangle mesh per sim")
        v = np.ascontiguousarray(np.asarray(vertices, dtype=np.float32).reshape(-1))
        t = np.ascontiguousarray(np.asarray(triangles, dtype=np.uint32).reshape(-1))
        if params.nb_vertices and v.size != 3 * params.nb_vertices:
            raise ValueError("add_triangle_mesh: vertex count does not match nb_vertices")
        if params.nb_triangles and t.size != 3 * params.nb_triangles:
            raise ValueError("add_triangle_mesh: triangle count does not match nb_triangles")
        p = params.transform.p
        sim.mesh = (v, t, (float(p.x), float(p.y), float(p.z)), float(params.static_friction),
                    float(params.dynamic_friction), float(params.restitution))
        return True

    # ---- assets
    def load_asset(self, sim: Sim, root: str, filename: str, options: Optional[AssetOptions] = None) -> Asset:
        options = options or AssetOptions()
        raw = load_raw(root, filename)
        meshes = [n for n in raw.link_order if raw.links[n].dropped_meshes]
        if meshes:
            warnings.warn(f"{filename}: collision meshes that are not readable STL files are not simulated "
                          f"(STL meshes collide as their convex hull, DESIGN.md section 6); links without "
                          f"contacts: {', '.join(meshes)}", PhysicsDeviationWarning, stacklevel=2)
        art = build_articulation(raw, options.as_dict())
        return Asset(art, options)

    def get_asset_dof_count(self, asset: Asset) -> int:
        return asset.art.num_dofs

    def get_asset_rigid_body_count(self, asset: Asset) -> int:
        return asset.art.num_links

    def get_asset_rigid_shape_count(self, asset: Asset) -> int:
        return asset.art.num_shapes

    def get_asset_joint_count(self, asset: Asset) -> int:
        return asset.art.num_dofs

    def get_asset_rigid_body_names(self, asset: Asset) -> List[str]:
        return asset.art.link_names()

    def get_asset_rigid_body_name(self, asset: Asset, index: int) -> str:
        return asset.art.link_names()[index]

    def get_asset_dof_names(self, asset: Asset) -> List[str]:
        return asset.art.dof_names()

    def get_asset_dof_name(self, asset: Asset, index: int) -> str:
        return asset.art.dof_names()[index]

    def find_asset_rigid_body_index(self, asset: Asset, name: str) -> int:
        names = asset.art.link_names()
        return names.index(name) if name in names else INVALID_HANDLE

    def find_asset_dof_index(self, asset: Asset, name: str) -> int:
        names = asset.art.dof_names()
        return names.index(name) if name in names else INVALID_HANDLE

    def get_asset_dof_properties(self, asset: Asset):
        return asset.dof_props.copy()

    def get_asset_rigid_shape_properties(self, asset: Asset):
        return [RigidShapeProperties(p.friction) for p in asset.shape_props]

    def set_asset_rigid_shape_properties(self, asset: Asset, props) -> bool:
        for dst, src in zip(asset.shape_props, props):
            dst.friction = float(src.friction)
            dst.restitution = float(getattr(src, "restitution", 0.0))
        return True

    def get_asset_actuator_properties(self, asset: Asset):
        # MJCF motors carry their gear (ant.py:160-162 reads it as motor_effort); URDF: the effort limit
        return [ActuatorProperties(d.motor_gear if d.motor_gear > 0 else d.effort) for d in asset.art.dofs]

    def get_asset_actuator_count(self, asset: Asset) -> int:
        return asset.art.num_dofs

    def create_asset_force_sensor(self, asset: Asset, body_idx: int, pose: Transform, props=None) -> int:
        """Sensor on a leaf body with identity pose (ant.py:174-178); reads the joint-reaction wrench
        the body receives from its parent."""
        p, r = np.array(list(pose.p)), np.array(list(pose.r))
        if np.any(np.abs(p) > 1e-9) or np.any(np.abs(r - np.array([0, 0, 0, 1.0])) > 1e-9):
            raise NotImplementedError("force sensors support the identity sensor pose only")
        asset.sensors.append((int(body_idx), pose))
        return len(asset.sensors) - 1

    # ---- envs / actors
    def create_env(self, sim: Sim, lower: Vec3, upper: Vec3, num_per_row: int) -> Env:
        i = len(sim.envs)
        num_per_row = max(1, int(num_per_row))
        row, col = divmod(i, num_per_row)
        sx, sy = upper.x - lower.x, upper.y - lower.y
        env = Env(sim, i, (col * sx, row * sy, 0.0))
        sim.envs.append(env)
        return env

    def get_env_origin(self, env: Env) -> Vec3:
        return Vec3(*env.origin)

    def get_env_count(self, sim: Sim) -> int:
        return len(sim.envs)

    def create_actor(self, env: Env, asset: Asset, pose: Transform, name: str = "", group: int = -1,
                     filter: int = -1, segmentation_id: int = 0) -> int:
        a = Actor(env, asset, pose, name, group, filter)
        env.actors.append(a)
        owner = env.sim
        if owner.asset is None:
            owner.asset = asset
        elif owner.asset is not asset:
            raise NotImplementedError("one asset type per sim (DESIGN.md section 6)")
        return len(env.actors) - 1

    def get_actor_count(self, env: Env) -> int:
        return len(env.actors)

    def get_sim_actor_count(self, sim: Sim) -> int:
        return sum(len(e.actors) for e in sim.envs)

    def get_actor_dof_properties(self, env: Env, actor: int):
        return env.actors[actor].dof_props.copy()

    def set_actor_dof_properties(self, env: Env, actor: int, props) -> bool:
        env.actors[actor].dof_props = np.array(props, dtype=DofPropertiesDtype).copy()
        if getattr(env.sim, "prepared", False):
            env.sim.drives_dirty = True  # uploaded before the next simulate (tasks update actor by actor)
        return True

    def get_actor_rigid_shape_properties(self, env: Env, actor: int):
        return [RigidShapeProperties(float(f)) for f in env.actors[actor].shape_friction]

    def set_actor_rigid_shape_properties(self, env: Env, actor: int, props) -> bool:
        env.actors[actor].shape_friction = np.array([p.friction for p in props], dtype=np.float32)
        return True

    def find_actor_rigid_body_handle(self, env: Env, actor: int, name: str) -> int:
        names = env.actors[actor].asset.art.link_names()
        return names.index(name) if name in names else INVALID_HANDLE

    def find_actor_rigid_body_index(self, env: Env, actor: int, name: str, domain: int = DOMAIN_ENV) -> int:
        return self.find_actor_rigid_body_handle(env, actor, name)

    def find_actor_dof_handle(self, env: Env, actor: int, name: str) -> int:
        names = env.actors[actor].asset.art.dof_names()
        return names.index(name) if name in names else INVALID_HANDLE

    def get_actor_dof_count(self, env: Env, actor: int) -> int:
        return env.actors[actor].asset.art.num_dofs

    def get_actor_rigid_body_count(self, env: Env, actor: int) -> int:
        return env.actors[actor].asset.art.num_links

    def get_actor_rigid_body_names(self, env: Env, actor: int):
        return env.actors[actor].asset.art.link_names()

    def get_actor_dof_names(self, env: Env, actor: int):
        return env.actors[actor].asset.art.dof_names()

    def get_actor_joint_dict(self, env: Env, actor: int):
        """Joints in link order, fixed joints included (joint i connects link i + 1 to its parent)."""
        return {n: i for i, n in enumerate(env.actors[actor].asset.art.joint_names())}

    def get_actor_dof_dict(self, env: Env, actor: int):
        return {n: i for i, n in enumerate(env.actors[actor].asset.art.dof_names())}

    def get_actor_rigid_body_dict(self, env: Env, actor: int):
        return {n: i for i, n in enumerate(env.actors[actor].asset.art.link_names())}

    def enable_actor_dof_force_sensors(self, env: Env, actor: int):
        return True

    def set_rigid_body_color(self, *args, **kwargs):
        return None

    # ---- tensor acquire (sim owned, zero copy)
    def acquire_actor_root_state_tensor(self, sim: Sim) -> GymTensor:
        sim._tensors()
        return GymTensor(sim.root_tensor, "root")

    def acquire_dof_state_tensor(self, sim: Sim) -> GymTensor:
        sim._tensors()
        return GymTensor(sim.dof_tensor, "dof")

    def acquire_net_contact_force_tensor(self, sim: Sim) -> GymTensor:
        sim._tensors()
        return GymTensor(sim.contact_tensor, "contact")

    def acquire_rigid_body_state_tensor(self, sim: Sim) -> GymTensor:
        """[num_envs * num_bodies, 13]: link origin, quat xyzw, COM linear velocity, angular velocity."""
        return GymTensor(sim.kinematics_tensor("rigid_body"), "rigid_body")

    def acquire_force_sensor_tensor(self, sim: Sim) -> GymTensor:
        """[num_envs * sensors_per_env, 6]: force (3) then torque (3) in the sensor frame (ant.py:80-83)."""
        return GymTensor(sim.sensor_tensor, "sensor")

    def acquire_jacobian_tensor(self, sim: Sim, name: str) -> GymTensor:
        """Floating base: [num_envs, num_bodies, 6, 6 + num_dofs]; fixed base: [num_envs, num_bodies - 1,
        6, num_dofs] (the welded root row dropped, as Isaac Gym does).  Rows: COM linear velocity (3),
        angular velocity (3); columns: root link COM linear / angular velocity, dof velocities."""
        self._check_actor_name(sim, name)
        t = sim.kinematics_tensor("jacobian")
        return GymTensor(t[:, 1:] if sim.asset.art.fixed_base else t, "jacobian")

    def acquire_mass_matrix_tensor(self, sim: Sim, name: str) -> GymTensor:
        """[num_envs, nv, nv] in the jacobian's generalized velocities (v^T M v / 2 = kinetic energy)."""
        self._check_actor_name(sim, name)
        return GymTensor(sim.kinematics_tensor("mass_matrix"), "mass_matrix")

    @staticmethod
    def _check_actor_name(sim: Sim, name: str):
        names = {a.name for e in sim.envs for a in e.actors}
        if name not in names:
            raise ValueError(f"no actor named {name!r} (actors: {sorted(names)})")

    # ---- refresh (sim -> tensors)
    def refresh_actor_root_state_tensor(self, sim: Sim):
        sim.refresh("root")

    def refresh_dof_state_tensor(self, sim: Sim):
        sim.refresh("dof")

    def refresh_net_contact_force_tensor(self, sim: Sim):
        sim.refresh("contact")

    def refresh_rigid_body_state_tensor(self, sim: Sim):
        sim.refresh("rigid_body")

    def refresh_jacobian_tensors(self, sim: Sim):
        sim.refresh("jacobian")

    def refresh_mass_matrix_tensors(self, sim: Sim):
        sim.refresh("mass_matrix")

    def refresh_force_sensor_tensor(self, sim: Sim):
        if sim.num_sensors:
            sim.refresh("sensor")

    def refresh_dof_force_tensor(self, sim: Sim):
        return None

    # ---- set (caller -> sim)
    def set_dof_actuation_force_tensor(self, sim: Sim, t: GymTensor) -> bool:
        sim.dof_force.copy_(t.tensor.reshape(-1).to(sim.sim_device))
        return True

    def set_dof_actuation_force_tensor_indexed(self, sim: Sim, t: GymTensor, idx: GymTensor, n: int) -> bool:
        import torch
        ids = idx.tensor[:n].to(sim.sim_device, dtype=torch.long)
        src = t.tensor.reshape(sim.num_envs, sim.num_dofs).to(sim.sim_device)
        sim.dof_force.view(sim.num_envs, sim.num_dofs)[ids] = src[ids]
        return True

    def set_actor_root_state_tensor(self, sim: Sim, t: GymTensor) -> bool:
        sim.set_state("root", t.tensor)
        return True

    def amd_set_root_and_dof_state_indexed(self, sim: Sim, root: GymTensor, dof: GymTensor, idx: GymTensor,
                                           n: int) -> bool:
        """set_actor_root_state_tensor_indexed + set_dof_state_tensor_indexed with the same indices, in one host
        call (the reset's pair, anymal_terrain.py:401-408): the same two launches, less Python per reset."""
        both = getattr(sim, "set_root_and_dof", None)
        if both is None:  # a sim object with only the per-kind setter (test doubles)
            return (self.set_actor_root_state_tensor_indexed(sim, root, idx, n)
                    and self.set_dof_state_tensor_indexed(sim, dof, idx, n))
        both(root.tensor, dof.tensor, idx.tensor, n)
        return True

    def set_actor_root_state_tensor_indexed(self, sim: Sim, t: GymTensor, idx: GymTensor, n: int) -> bool:
        sim.set_state("root", t.tensor, idx.tensor, n)
        return True

    def set_dof_state_tensor(self, sim: Sim, t: GymTensor) -> bool:
        sim.set_state("dof", t.tensor)
        return True

    def set_dof_state_tensor_indexed(self, sim: Sim, t: GymTensor, idx: GymTensor, n: int) -> bool:
        sim.set_state("dof", t.tensor, idx.tensor, n)
        return True

    def set_dof_position_target_tensor(self, sim: Sim, t: GymTensor) -> bool:
        """Targets of DOF_MODE_POS dofs (joint drives); other dofs ignore them."""
        sim.set_targets("pos", t.tensor)
        return True

    def set_dof_position_target_tensor_indexed(self, sim: Sim, t: GymTensor, idx: GymTensor, n: int) -> bool:
        """UsefulHound sets targets on reset (useful_hound.py:622-627); its dofs are DOF_MODE_EFFORT,
        where a target has no effect."""
        sim.set_targets("pos", t.tensor, idx.tensor, n)
        return True

    def set_dof_velocity_target_tensor(self, sim: Sim, t: GymTensor) -> bool:
        sim.set_targets("vel", t.tensor)
        return True

    def set_dof_velocity_target_tensor_indexed(self, sim: Sim, t: GymTensor, idx: GymTensor, n: int) -> bool:
        sim.set_targets("vel", t.tensor, idx.tensor, n)
        return True

    # ---- viewer / rendering (headless build: no-ops)
    def create_viewer(self, sim: Sim, props: CameraProperties):
        return None

    def subscribe_viewer_keyboard_event(self, *args, **kwargs):
        return None

    def viewer_camera_look_at(self, *args, **kwargs):
        return None

    def query_viewer_has_closed(self, viewer) -> bool:
        return False

    def query_viewer_action_events(self, viewer):
        return []

    def step_graphics(self, sim: Sim):
        return None

    def draw_viewer(self, *args, **kwargs):
        return None

    def sync_frame_time(self, sim: Sim):
        return None

    def poll_viewer_events(self, viewer):
        return None

    def clear_lines(self, viewer):
        return None

    def destroy_viewer(self, viewer):
        return None

    # ---- MI355X extensions (not part of the Isaac Gym API)
    def amd_pd_decimation_step(self, sim: Sim, actions, default_pos, kp: float, kd: float, action_scale: float,
                               torque_limit: float, decimation: int, extra_simulates: int, torques_out,
                               write_root: bool = True, write_contacts: bool = True, actions_copy_out=None,
                               tail=None):
        """Fused ``for i in decimation: PD torque; simulate; refresh dof`` + ``extra_simulates`` more
        simulates, + the root/contact refreshes of post_physics_step, in ONE kernel launch.  ``tail``: the
        AnymalTerrain post_physics_step part A run in the same launch, as (gt_anymal_params, gt_anymal_buffers)
        ctypes structs (gymtask.AnymalTailKernel.tail_for_launch; only where amd_pd_tail_supported)."""
        L = _lib.lib()
        assert sim.gpu_pipeline or sim.host, "the fused step needs the GPU pipeline or the host backend"
        # the argument struct is kept per sim and rebuilt only when a fixed field changes (a step changes the two
        # action pointers only): ~2 us of ctypes field stores off the host path before the launch
        key = (default_pos.data_ptr(), kp, kd, action_scale, torque_limit, decimation, extra_simulates,
               torques_out.data_ptr(), sim.dof_tensor.data_ptr(), sim.root_tensor.data_ptr() if write_root else None,
               sim.contact_tensor.data_ptr() if write_contacts else None)
        a = sim._pd_args
        if a is None or sim._pd_key != key:
            a = _lib.GsPdArgs()
            a.default_pos = key[0]
            a.kp, a.kd, a.action_scale, a.torque_limit = kp, kd, action_scale, torque_limit
            a.decimation, a.extra_simulates = int(decimation), int(extra_simulates)
            a.torques_out, a.dof_state_out, a.root_state_out, a.contact_out = key[7:]
            sim._pd_args, sim._pd_key = a, key
        a.actions = actions.data_ptr()
        a.actions_copy_out = actions_copy_out.data_ptr() if actions_copy_out is not None else None
        if tail is None:
            a.tail_params = a.tail_buffers = None
        else:
            a.tail_params, a.tail_buffers = C.addressof(tail[0]), C.addressof(tail[1])
        if sim.drives_dirty:
            sim.apply_drives()
        _lib.check(L.gs_sim_pd_step(sim.handle, a, sim.stream()), "gs_sim_pd_step")

    def amd_pd_tail_supported(self, sim: Sim) -> bool:
        """The fused step's kernel can run the AnymalTerrain tail (gs_sim_pd_tail_supported: the lane team)."""
        return bool(_lib.lib().gs_sim_pd_tail_supported(sim.handle))

    def amd_enable_kernel_timing(self, sim: Sim, enable: bool = True):
        _lib.check(_lib.lib().gs_sim_enable_timing(sim.handle, int(enable)), "gs_sim_enable_timing")

    def amd_kernel_variant(self, sim: Sim) -> int:
        """1: one env per lane, 2: lane team (4 lanes per env), 3 host backend, 4 runtime-sized (any topology); see
        gs_sim_kernel_variant."""
        return int(_lib.lib().gs_sim_kernel_variant(sim.handle))

    def amd_last_kernel_ms(self, sim: Sim) -> float:
        return float(_lib.lib().gs_sim_last_kernel_ms(sim.handle))


_GYM = None


def acquire_gym() -> Gym:
    global _GYM
    if _GYM is None:
        _GYM = Gym()
    return _GYM
