"""ctypes binding of libgymtask.so (include/gymtask.h) and the AnymalTerrain tail driver.

Loaded only on the GPU pipeline; there is no fallback -- a missing library is an
error (the torch statements in tasks/anymal_terrain.py serve the CPU pipeline).
"""
from __future__ import annotations

import ctypes as C
import os

import torch
from isaacgymenv_amd._stream import raw_stream

# GT_LIBGYMTASK names another build of the library in _lib/ (A/B runs)
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                        os.path.basename(os.environ.get("GT_LIBGYMTASK", "libgymtask.so")))


class GtTorchRandPlan(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("offset", C.c_uint64), ("threads", C.c_uint32), ("numel", C.c_uint32)]


class TorchRandPlanner:
    """Reserves torch.rand(n) draws on a device generator without launching torch's kernel.

    Mirrors ATen's calc_execution_policy + philox_cuda_state (DistributionTemplates.h): the
    kernel-side evaluation is isaacgymenv_amd/csrc/torch_philox.h.  After ``plan(n)`` the
    generator is exactly where ``torch.rand(n, device=...)`` would have left it."""

    def __init__(self, device):
        dev = torch.device(device)
        self.index = dev.index if dev.index is not None else torch.cuda.current_device()
        self.gen = torch.cuda.default_generators[self.index]
        props = torch.cuda.get_device_properties(self.index)
        self.grid_cap = props.multi_processor_count * (props.max_threads_per_multi_processor // 256)

    def plan(self, n: int) -> GtTorchRandPlan:
        return self.plan_many((n,))[0]

    def plan_many(self, sizes):
        """Plans for consecutive torch.rand calls of the given sizes (one generator update)."""
        g = self.gen
        seed, off = g.initial_seed(), g.get_offset()
        plans = []
        for n in sizes:
            threads = 256 * min(self.grid_cap, (n + 255) // 256)
            plans.append(GtTorchRandPlan(seed, off, threads, n))
            off += ((n - 1) // (4 * threads) + 1) * 4
        g.set_offset(off)
        return plans


class GtAnymalParams(C.Structure):
    _fields_ = [("num_envs", C.c_int32), ("num_dofs", C.c_int32), ("num_bodies", C.c_int32), ("num_obs", C.c_int32),
                ("base_index", C.c_int32), ("num_feet", C.c_int32), ("feet_idx", C.c_int32 * 4),
                ("num_knees", C.c_int32), ("knee_idx", C.c_int32 * 4), ("hip_dofs", C.c_int32 * 4),
                ("allow_knee_contacts", C.c_int32), ("max_episode_length", C.c_int64), ("dt", C.c_float)] + [
        (n, C.c_float) for n in ("s_termination", "s_lin_vel_xy", "s_lin_vel_z", "s_ang_vel_z", "s_ang_vel_xy",
                                 "s_orient", "s_torque", "s_joint_acc", "s_base_height", "s_air_time",
                                 "s_collision", "s_stumble", "s_action_rate", "s_hip", "lin_vel_scale",
                                 "ang_vel_scale", "dof_pos_scale", "dof_vel_scale", "height_meas_scale")] + [
        ("default_dof_pos", C.c_float * 16), ("base_init_state", C.c_float * 13)]


class GtAnymalBuffers(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("root_states", "contact_forces", "dof_state", "torques", "actions",
                                          "last_actions", "last_dof_vel", "commands", "feet_air_time",
                                          "progress_buf", "randomize_buf", "reset_buf", "timeout_buf")] + [
        ("timeout_is_int64", C.c_int32)] + [
        (n, C.c_void_p) for n in ("rew_buf", "episode_sums", "base_lin_vel", "base_ang_vel", "projected_gravity",
                                  "obs_buf", "noise_scale", "reset_count", "host_count")] + [
        ("seq", C.c_int32), ("reset_masks", C.c_void_p), ("obs_out", C.c_void_p), ("time_outs", C.c_void_p),
        ("clip_obs", C.c_float), ("measured_heights", C.c_void_p), ("hound", C.c_void_p), ("obs_mirror", C.c_void_p)]


class GtAnymalHound(C.Structure):
    """gt_anymal_hound (include/gymtask.h, ABI 3): UsefulHound's differences to the AnymalTerrain tail."""
    _fields_ = [("num_actions", C.c_int32), ("num_shoulders", C.c_int32), ("shoulder_idx", C.c_int32 * 4),
                ("eef_state", C.c_void_p), ("eef_stride", C.c_int32), ("arm_commands", C.c_void_p),
                ("pos_control", C.c_void_p), ("effort_control", C.c_void_p), ("arm_default", C.c_float * 6),
                ("arm_lower", C.c_float * 6), ("arm_upper", C.c_float * 6), ("arm_noise2", C.c_float),
                ("u_arm", C.c_void_p), ("plan_arm", GtTorchRandPlan)]


class GtAnymalResetDraws(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("u_pos", "u_vel", "u_cmd_x", "u_cmd_y", "u_cmd_h")] + [
        (n, GtTorchRandPlan) for n in ("plan_pos", "plan_vel", "plan_cmd_x", "plan_cmd_y", "plan_cmd_h")] + [
        (n, C.c_float) for n in ("pos_range", "pos_lower", "vel_range", "vel_lower", "cmd_x_range", "cmd_x_lower",
                                 "cmd_y_range", "cmd_y_lower", "cmd_h_range", "cmd_h_lower")]


class GtAnymalTerrainReset(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("terrain_levels", "terrain_types", "env_origins", "terrain_origins")] + [
        (n, C.c_int32) for n in ("env_rows", "env_cols", "update_levels")] + [
        ("env_length", C.c_float), ("max_episode_length_s", C.c_float), ("u_root_xy", C.c_void_p),
        ("plan_root_xy", GtTorchRandPlan), ("xy_range", C.c_float), ("xy_lower", C.c_float)]


class GtHoundControlParams(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("num_envs", "nv", "num_links", "jac_row", "eef_link", "arm_control_stride")] + [
        (n, C.c_float) for n in ("kp", "kd", "action_scale", "torque_limit", "arm_action_scale")] + [
        (n, C.c_float * 6) for n in ("arm_kp", "arm_kd", "arm_kp_null", "arm_kd_null", "arm_cmd_limit", "arm_default",
                                     "arm_effort")]


class GtAntParams(C.Structure):
    _fields_ = [("num_envs", C.c_int32), ("num_dofs", C.c_int32)] + [
        (n, C.c_float) for n in ("dt", "dof_vel_scale", "contact_force_scale", "heading_weight", "up_weight",
                                 "actions_cost_scale", "energy_cost_scale", "joints_at_limit_cost_scale",
                                 "termination_height", "death_cost", "max_episode_length")] + [
        ("dof_lower", C.c_float * 8), ("dof_upper", C.c_float * 8)]


class GtAntBuffers(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("root_states", "dof_state", "sensors", "actions", "targets",
                                          "inv_start_rot", "potentials", "prev_potentials", "up_vec",
                                          "heading_vec", "obs_buf", "rew_buf", "true_objective", "reset_buf",
                                          "progress_buf", "reset_count", "host_count")] + [("seq", C.c_int32),
                                                                                           ("reset_masks", C.c_void_p)]


class GtAntResetArgs(C.Structure):
    _fields_ = [("plan_pos", GtTorchRandPlan), ("plan_vel", GtTorchRandPlan), ("u_pos", C.c_void_p),
                ("u_vel", C.c_void_p)] + [(n, C.c_float) for n in ("pos_range", "pos_lower", "vel_range",
                                                                     "vel_lower")] + [
        (n, C.c_void_p) for n in ("initial_dof_pos", "initial_root_states", "dof_state", "progress_buf",
                                  "env_ids_out")]


_lib = None


class EpisodeExtras(dict):
    """extras["episode"] of a fused reset (anymal_terrain.py:416-421): {"rew_<term>": 0-d tensor, ...,
    "terrain_level": 0-d tensor}, the same keys, order and values as the dict of fresh torch.mean results the
    reference builds -- held as the reset's own fresh device buffer and split into its 0-d tensors when first read
    (splitting 14 views costs ~10-20 us of host time on every reset step, and a learner that never reads the meters,
    like the PPO rollout, never pays it).  Every read path of a dict materialises first, the C-level ones included
    (dict(x) / {**x} / copy go through the overridden __iter__ / keys)."""

    __slots__ = ("_src",)

    def __init__(self, keys, ep, terrain_level=None):
        super().__init__()
        self._src = (keys, ep, terrain_level)

    def _m(self):
        src = self._src
        if src is not None:
            self._src = None
            keys, ep, lvl = src
            n = len(keys)
            dict.update(self, zip(keys, ep[:n].unbind()))
            dict.__setitem__(self, "terrain_level", ep[n] if lvl is None else lvl)
        return self

    def __getitem__(self, k):
        return dict.__getitem__(self._m(), k)

    def __iter__(self):
        return dict.__iter__(self._m())

    def __len__(self):
        return dict.__len__(self._m())

    def __contains__(self, k):
        return dict.__contains__(self._m(), k)

    def __repr__(self):
        return dict.__repr__(self._m())

    def __eq__(self, other):
        return dict.__eq__(self._m(), other)

    def __reduce__(self):
        return (dict, (dict(self._m().items()),))

    def get(self, k, default=None):
        return dict.get(self._m(), k, default)

    def keys(self):
        return dict.keys(self._m())

    def values(self):
        return dict.values(self._m())

    def items(self):
        return dict.items(self._m())

    def copy(self):
        return dict(self._m().items())

    def pop(self, *a):
        return dict.pop(self._m(), *a)

    def popitem(self):
        return dict.popitem(self._m())

    def setdefault(self, *a):
        return dict.setdefault(self._m(), *a)

    def update(self, *a, **k):
        return dict.update(self._m(), *a, **k)

    def __setitem__(self, k, v):
        dict.__setitem__(self._m(), k, v)

    def __delitem__(self, k):
        dict.__delitem__(self._m(), k)

    def clear(self):
        self._src = None
        dict.clear(self)

    __hash__ = None


def _anymal_set_reset_state():
    """AnymalTerrain._set_reset_state (the one-call root + dof indexed set that gt_anymal_reset_observe replaces by
    its C callback); a task that overrides it keeps the Python sequence."""
    from isaacgymenv_amd.isaacgymenvs.tasks.anymal_terrain import AnymalTerrain
    return AnymalTerrain._set_reset_state


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m isaacgymenv_amd.build`. "
                               "The GPU pipeline has no torch fallback for the fused task kernels.")
        L = C.CDLL(LIB_PATH)
        P, B, vp, i = C.POINTER(GtAnymalParams), C.POINTER(GtAnymalBuffers), C.c_void_p, C.c_int
        for name, args in {"gt_anymal_post_physics_a": [P, B, vp],
                           "gt_anymal_reset": [P, B, vp, i, vp, vp, vp, vp, vp, vp, vp],
                           "gt_anymal_post_physics_b": [P, B, vp, C.POINTER(GtTorchRandPlan), vp],
                           "gt_anymal_post_physics_ab": [P, B, C.POINTER(GtTorchRandPlan), vp],
                           "gt_torch_rand": [C.POINTER(GtTorchRandPlan), vp, vp],
                           "gt_anymal_reset_flagged": [P, B, i, C.POINTER(GtAnymalResetDraws),
                                                       C.POINTER(GtAnymalTerrainReset), vp, vp, C.c_float, vp, vp],
                           "gt_host_alloc": [C.c_uint64, C.POINTER(vp), C.POINTER(vp)],
                           "gt_host_free": [vp],
                           "gt_wait_host_seq": [vp, C.c_int32, C.c_int32, C.POINTER(C.c_int32)],
                           "gt_measure_heights": [vp, i, i, C.c_float, C.c_float, C.c_float, vp, vp, i, i, vp,
                                                  vp],
                           "gt_hound_control": [C.POINTER(GtHoundControlParams), vp, vp, vp, vp, vp, vp, vp, vp,
                                                vp],
                           "gt_ant_post_physics": [C.POINTER(GtAntParams), C.POINTER(GtAntBuffers), vp],
                           "gt_ant_reset_flagged": [C.POINTER(GtAntParams), C.POINTER(GtAntBuffers), i,
                                                    C.POINTER(GtAntResetArgs), vp],
                           "gt_anymal_reset_observe": [P, B, i, C.POINTER(GtAnymalResetDraws), vp, vp, C.c_float, vp,
                                                       C.c_uint64, C.POINTER(C.c_uint64), C.c_uint32, i, vp, vp, vp,
                                                       vp, vp],
                           "gt_anymal_wait_reset_observe": [vp, C.c_int32, C.c_int32, C.POINTER(C.c_int32), P, B,
                                                            C.POINTER(GtAnymalResetDraws), vp, vp, C.c_float, vp,
                                                            C.c_uint64, C.POINTER(C.c_uint64), C.c_uint32, i, vp, vp,
                                                            vp, vp, vp]}.items():
            fn = getattr(L, name)
            fn.restype = C.c_int
            fn.argtypes = args
        L.gt_last_error.restype = C.c_char_p
        L.gt_abi_version.restype = C.c_int
        _lib = L
    return _lib


EXPORTED_SYMBOLS = ["gt_abi_version", "gt_last_error", "gt_anymal_post_physics_a", "gt_anymal_reset",
                    "gt_anymal_post_physics_b", "gt_anymal_reset_flagged", "gt_torch_rand", "gt_host_alloc",
                    "gt_host_free", "gt_wait_host_seq", "gt_measure_heights", "gt_hound_control",
                    "gt_ant_post_physics", "gt_ant_reset_flagged", "gt_anymal_reset_observe", "gt_anymal_post_physics_ab",
                    "gt_anymal_wait_reset_observe"]


class AntTailKernel:
    """gt_ant_post_physics bound to one Ant env (GPU pipeline): observations + reward + done mask in one
    launch, and the done count published to pinned host memory for the next step's reset."""

    def __init__(self, env):
        L = lib()
        t = self.env = env
        p = GtAntParams()
        p.num_envs, p.num_dofs = t.num_envs, t.num_dof
        p.dt, p.dof_vel_scale, p.contact_force_scale = float(t.dt), float(t.dof_vel_scale), float(t.contact_force_scale)
        p.heading_weight, p.up_weight = float(t.heading_weight), float(t.up_weight)
        p.actions_cost_scale, p.energy_cost_scale = float(t.actions_cost_scale), float(t.energy_cost_scale)
        p.joints_at_limit_cost_scale = float(t.joints_at_limit_cost_scale)
        p.termination_height, p.death_cost = float(t.termination_height), float(t.death_cost)
        p.max_episode_length = float(t.max_episode_length)
        p.dof_lower[:] = [float(v) for v in t.dof_limits_lower.cpu()]
        p.dof_upper[:] = [float(v) for v in t.dof_limits_upper.cpu()]
        self.p = p
        self.true_objective = torch.zeros(t.num_envs, dtype=torch.float32, device=t.device)
        self.reset_count = torch.zeros(3, dtype=torch.int32, device=t.device)
        h, d = C.c_void_p(), C.c_void_p()
        _check(L.gt_host_alloc(8, C.byref(h), C.byref(d)), "gt_host_alloc")
        self._host_words, self._host_words_dev = h.value, d.value
        self._seq = 0
        self._launched = False
        self._count = C.c_int32(0)
        self.reset_masks = torch.zeros((t.num_envs + 63) // 64, dtype=torch.int64, device=t.device)
        self.env_ids = torch.zeros(t.num_envs, dtype=torch.int32, device=t.device)
        self.planner = TorchRandPlanner(t.device)

    def __del__(self):
        if getattr(self, "_host_words", None) and _lib is not None:
            _lib.gt_host_free(self._host_words)
            self._host_words = None

    def done_count(self):
        """Envs the previous launch flagged (None before the first launch: the caller must look)."""
        if not self._launched:
            return None
        _check(lib().gt_wait_host_seq(C.c_void_p(self._host_words), self._seq, 10000, C.byref(self._count)),
               "gt_wait_host_seq")
        return int(self._count.value)

    def reset_flagged(self, k: int, u_pos=None, u_vel=None):
        """ant.py:252-279 reset_idx for the k envs the previous launch flagged, in one kernel: the two
        torch_rand_float draws evaluated in-kernel from the device generator (advanced exactly as torch.rand
        would be) or taken from u_pos / u_vel [k, 8], the clamped dof state, potentials, counters; then the
        reference's two indexed state sets.  Returns the flagged env ids (int32 [k])."""
        from .isaacgym import gymtorch
        t = self.env
        r = GtAntResetArgs()
        if u_pos is None:
            r.plan_pos, r.plan_vel = self.planner.plan_many((k * t.num_dof, k * t.num_dof))
        else:
            r.u_pos, r.u_vel = u_pos.contiguous().data_ptr(), u_vel.contiguous().data_ptr()
        # torch_rand_float(lower, upper): (upper - lower) * rand + lower, the range a Python double
        r.pos_range, r.pos_lower = 0.2 - (-0.2), -0.2
        r.vel_range, r.vel_lower = 0.1 - (-0.1), -0.1
        r.initial_dof_pos, r.initial_root_states = t.initial_dof_pos.data_ptr(), t.initial_root_states.data_ptr()
        r.dof_state, r.progress_buf, r.env_ids_out = t.dof_state.data_ptr(), t.progress_buf.data_ptr(), \
            self.env_ids.data_ptr()
        stream = raw_stream(t.root_states.device)
        _check(lib().gt_ant_reset_flagged(C.byref(self.p), C.byref(self._buffers()), k, C.byref(r),
                                          C.c_void_p(stream)), "gt_ant_reset_flagged")
        ids = self.env_ids[:k]
        t.gym.set_actor_root_state_tensor_indexed(t.sim, gymtorch.unwrap_tensor(t.initial_root_states),
                                                  gymtorch.unwrap_tensor(ids), k)
        t.gym.set_dof_state_tensor_indexed(t.sim, gymtorch.unwrap_tensor(t.dof_state), gymtorch.unwrap_tensor(ids), k)
        return ids

    def _buffers(self):
        t = self.env
        b = GtAntBuffers()
        for name, ten in (("root_states", t.root_states), ("dof_state", t.dof_state), ("sensors", t.vec_sensor_tensor),
                          ("actions", t.actions), ("targets", t.targets), ("inv_start_rot", t.inv_start_rot),
                          ("potentials", t.potentials), ("prev_potentials", t.prev_potentials),
                          ("up_vec", t.up_vec), ("heading_vec", t.heading_vec), ("obs_buf", t.obs_buf),
                          ("rew_buf", t.rew_buf), ("true_objective", self.true_objective),
                          ("reset_buf", t.reset_buf), ("progress_buf", t.progress_buf)):
            assert ten.is_contiguous() and ten.is_cuda, name
            setattr(b, name, ten.data_ptr())
        assert t.reset_buf.dtype == torch.int64 and t.progress_buf.dtype == torch.int64
        b.seq = self._seq
        b.reset_count = self.reset_count.data_ptr()
        b.host_count = self._host_words_dev
        b.reset_masks = self.reset_masks.data_ptr()
        return b

    def __call__(self):
        t = self.env
        self._seq += 1
        b = self._buffers()
        stream = raw_stream(t.root_states.device)
        _check(lib().gt_ant_post_physics(C.byref(self.p), C.byref(b), C.c_void_p(stream)), "gt_ant_post_physics")
        self._launched = True


class HoundControlKernel:
    """gt_hound_control bound to one UsefulHound env's tensors (the fused inner step of its decimation loop)."""

    def __init__(self, env):
        import torch
        self.env = env
        p = GtHoundControlParams()
        p.num_envs = env.num_envs
        p.nv = int(env._mm_full.shape[-1])
        p.num_links = int(env._jac_full.shape[1])
        p.jac_row = int(env._hand_joint_index)
        p.eef_link = int(env.eef_index)
        p.arm_control_stride = int(env._effort_control.stride(0))
        p.kp, p.kd = float(env.Kp), float(env.Kd)
        p.action_scale, p.torque_limit = float(env.action_scale), 80.0
        p.arm_action_scale = float(env.arm_action_scale)
        for name, t in (("arm_kp", env.arm_kp), ("arm_kd", env.arm_kd), ("arm_kp_null", env.arm_kp_null),
                        ("arm_kd_null", env.arm_kd_null), ("arm_cmd_limit", env.arm_cmd_limit.reshape(-1)),
                        ("arm_default", env.houndarm_default_dof_pos[:6]), ("arm_effort", env._houndarm_effort_limits[:6])):
            vals = [float(v) for v in t.detach().cpu().reshape(-1)[:6]]
            getattr(p, name)[:] = vals
        self.p = p
        self.leg_default = env.hound_default_dof_pos[0].contiguous()
        for t in (env.dof_state, env._mm_full, env._jac_full, env._rigid_body_state):
            assert t.is_contiguous() and t.dtype == torch.float32 and t.is_cuda
        assert env._effort_control.is_contiguous()

    def __call__(self, actions, torques_out):
        import torch
        env = self.env
        stream = raw_stream(actions.device)
        _check(lib().gt_hound_control(C.byref(self.p), actions.data_ptr(), env.dof_state.data_ptr(),
                                      self.leg_default.data_ptr(), env._mm_full.data_ptr(), env._jac_full.data_ptr(),
                                      env._rigid_body_state.data_ptr(), torques_out.data_ptr(),
                                      env._effort_control.data_ptr(), C.c_void_p(stream)), "gt_hound_control")


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {lib().gt_last_error().decode()}")


def _ptr(t):
    return t.data_ptr() if t is not None else None


class AnymalTailKernels:
    """Drives gt_anymal_* for an AnymalTerrain task on the GPU pipeline, and for UsefulHound (the same
    tail with the gt_anymal_hound differences: 12 leg dofs of 18, shoulder terminations, the arm's
    reset draw, end-effector observations)."""

    TERMS = ["lin_vel_xy", "lin_vel_z", "ang_vel_z", "ang_vel_xy", "orient", "torques", "joint_acc",
             "base_height", "air_time", "collision", "stumble", "action_rate", "hip"]

    def __init__(self, task):
        L = lib()
        self.task = t = task
        dev = t.device
        N = t.num_envs
        self.hound = hasattr(t, "hound_num_dof")
        nd = int(t.hound_num_dof) if self.hound else int(t.num_dof)
        self.nd = nd
        p = GtAnymalParams()
        p.num_envs, p.num_dofs, p.num_bodies, p.num_obs = N, nd, int(t.contact_forces.shape[1]), t.num_obs
        p.base_index = int(t.base_index)
        p.num_feet = len(t.feet_indices)
        p.num_knees = len(t.knee_indices)
        for k, v in enumerate(t.feet_indices.tolist()):
            p.feet_idx[k] = v
        for k, v in enumerate(t.knee_indices.tolist()):
            p.knee_idx[k] = v
        for k, v in enumerate([0, 3, 6, 9]):
            p.hip_dofs[k] = v
        p.allow_knee_contacts = int(bool(t.allow_knee_contacts))
        p.max_episode_length = int(t.max_episode_length)
        p.dt = float(t.dt)
        rs = t.rew_scales
        for field, key in (("s_termination", "termination"), ("s_lin_vel_xy", "lin_vel_xy"),
                           ("s_lin_vel_z", "lin_vel_z"), ("s_ang_vel_z", "ang_vel_z"),
                           ("s_ang_vel_xy", "ang_vel_xy"), ("s_orient", "orient"), ("s_torque", "torque"),
                           ("s_joint_acc", "joint_acc"), ("s_base_height", "base_height"),
                           ("s_air_time", "air_time"), ("s_collision", "collision"), ("s_stumble", "stumble"),
                           ("s_action_rate", "action_rate"), ("s_hip", "hip")):
            setattr(p, field, float(rs[key]))
        p.lin_vel_scale, p.ang_vel_scale = float(t.lin_vel_scale), float(t.ang_vel_scale)
        p.dof_pos_scale, p.dof_vel_scale = float(t.dof_pos_scale), float(t.dof_vel_scale)
        p.height_meas_scale = float(t.height_meas_scale)
        default = t.hound_default_dof_pos if self.hound else t.default_dof_pos
        for k, v in enumerate(default[0].tolist()):
            p.default_dof_pos[k] = v
        for k, v in enumerate(t.base_init_state.tolist()):
            p.base_init_state[k] = v
        self.p = p
        # fixed buffers the kernels write in place (the torch path rebinds these attributes instead)
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)  # noqa: E731
        t.base_lin_vel, t.base_ang_vel, t.projected_gravity = z(N, 3), z(N, 3), z(N, 3)
        self.reset_bool = torch.zeros(N, dtype=torch.bool, device=dev)
        self.sums = z(len(self.TERMS), N)
        for k, name in enumerate(self.TERMS):
            self.sums[k].copy_(t.episode_sums[name])
            t.episode_sums[name] = self.sums[k]
        self.ep_out = z(len(self.TERMS))
        self.noise_scale = t.noise_scale_vec.contiguous()
        self.reset_count = torch.zeros(3, dtype=torch.int32, device=dev)  # accumulator, wg counter, last count
        self.reset_masks = torch.zeros((N + 63) // 64, dtype=torch.int64, device=dev)
        # GT_ANYMAL_RESET_SCRATCH_WORDS: re-armed counter (16 words) + per-wave episode partial sums
        self.reset_scratch = torch.zeros(16 + (len(self.TERMS) + 1) * ((N + 63) // 64), dtype=torch.float32,
                                         device=dev)
        # {count, seq} published by post_a straight into pinned host memory (gt_wait_host_seq)
        h, d = C.c_void_p(), C.c_void_p()
        _check(L.gt_host_alloc(8, C.byref(h), C.byref(d)), "gt_host_alloc")
        self._host_words, self._host_words_dev = h.value, d.value
        self._seq = 0
        self._count_out = C.c_int32(0)
        # reference draws (reset offsets/commands, obs noise) evaluated inside the kernels from the
        # device generator's Philox stream (bit-identical to torch.rand); False: torch draws buffers
        self.inkernel_rng = True
        self.planner = TorchRandPlanner(dev)
        self._draws = None
        self._ep_keys = ["rew_" + name for name in self.TERMS]
        self._terrain_level = None
        self._pending_extras = None  # (episode buffer, terrain) of a reset whose extras are not built yet
        self._b = None
        self._bound = None
        # (struct field, task attribute) of the buffers whose storage the kernels use
        self._stable = [(n, "last_hound_dof_vel" if (self.hound and n == "last_dof_vel") else n) for n in self._STABLE]
        self._h = self._hound_struct() if self.hound else None

    def _hound_struct(self):
        t = self.task
        h = GtAnymalHound()
        h.num_actions = int(t.num_actions)
        h.num_shoulders = len(t.base_indices)
        for k, v in enumerate(t.base_indices.tolist()):
            h.shoulder_idx[k] = v
        rb = t._rigid_body_state
        for x in (rb, t.arm_commands, t._pos_control, t._effort_control):
            assert x.is_contiguous() and x.dtype == torch.float32 and x.device.type == "cuda"
        h.eef_state = rb[0, t.eef_index].data_ptr()
        h.eef_stride = int(rb.stride(0))
        h.arm_commands, h.pos_control, h.effort_control = (x.data_ptr() for x in (t.arm_commands, t._pos_control,
                                                                                   t._effort_control))
        h.arm_default[:] = [float(v) for v in t.houndarm_default_dof_pos[:6].tolist()]
        h.arm_lower[:] = [float(v) for v in t.houndarm_dof_lower_limits[:6].tolist()]
        h.arm_upper[:] = [float(v) for v in t.houndarm_dof_upper_limits[:6].tolist()]
        h.arm_noise2 = float(t.houndarm_dof_noise * 2.0)  # useful_hound.py:598, a Python double cast once
        self._h_keep = (rb, t.arm_commands, t._pos_control, t._effort_control)
        return h

    def __del__(self):
        if getattr(self, "_host_words", None) and _lib is not None:
            _lib.gt_host_free(self._host_words)
            self._host_words = None

    # task attributes whose storage the kernels use; rebuilt only when one of them is rebound
    _STABLE = ("root_states", "contact_forces", "dof_state", "last_actions", "last_dof_vel", "commands",
               "feet_air_time", "progress_buf", "randomize_buf", "rew_buf", "base_lin_vel", "base_ang_vel",
               "projected_gravity", "obs_buf")

    def _buffers(self, check: bool = True):
        """The gt_anymal_buffers struct; rebuilt only if the task rebound a buffer (cheap on the hot path).
        check=False skips the rebinding check (the later launches of one step's tail, after post_a checked)."""
        t = self.task
        b = self._b
        if b is None or check:
            cur = tuple(getattr(t, attr) for _, attr in self._stable)
        if b is None or (check and any(x is not y for x, y in zip(cur, self._bound))):
            b = GtAnymalBuffers()
            for (name, attr), v in zip(self._stable, cur):
                assert v.is_contiguous() and v.device.type == "cuda", attr
                setattr(b, name, v.data_ptr())
            b.hound = C.cast(C.pointer(self._h), C.c_void_p) if self._h is not None else None
            b.reset_buf = self.reset_bool.data_ptr()
            b.episode_sums = self.sums.data_ptr()
            b.noise_scale = self.noise_scale.data_ptr()
            b.reset_count = self.reset_count.data_ptr()
            b.host_count = self._host_words_dev
            b.reset_masks = self.reset_masks.data_ptr()
            self._b, self._bound = b, cur
        b.torques = t.torques.data_ptr()
        b.actions = t.actions.data_ptr()
        tb = t.timeout_buf
        b.timeout_buf = tb.data_ptr()
        b.timeout_is_int64 = int(tb.dtype == torch.int64)
        b.obs_out = None
        b.time_outs = None
        hb = getattr(t, "_heights_dev", None)
        b.measured_heights = hb.data_ptr() if hb is not None else None
        return b

    def _stream(self):
        return raw_stream(self.task.device)

    def post_a(self):
        t = self.task
        if not t.torques.is_contiguous():
            t.torques = t.torques.contiguous()
        if not t.actions.is_contiguous():
            t.actions = t.actions.contiguous()
        b = self._buffers()
        self._seq = (self._seq + 1) & 0x7FFFFFFF
        b.seq = self._seq
        _check(lib().gt_anymal_post_physics_a(self.p, b, self._stream()), "gt_anymal_post_physics_a")
        t.reset_buf = self.reset_bool  # check_termination makes reset_buf a bool tensor (anymal_terrain.py:295)

    def tail_for_launch(self):
        """post_a run by the fused physics launch instead of its own (gymsim ABI 9, gs_pd_args.tail_*): the
        (params, buffers) structs for amd_pd_decimation_step, with the next sequence number the count is
        published under; None where the lane team cannot run it (then call post_a after the launch).  Call after
        the step's actions copy is bound to the task (task.actions) and before the launch."""
        t = self.task
        ok = self._tail_ok
        if ok is None:
            # off by default (GS_FUSED_TAIL=1 turns it on): measured no faster than the separate launch -- the
            # physics kernel grew by what post_a took (0.1106 -> 0.1185 ms, 30.0 vs 29.8 M env-steps/s,
            # profiles/r06i_fused_tail_ab.txt): the tail's cost is its own dependent chain, not the launch
            ok = self._tail_ok = (os.environ.get("GS_FUSED_TAIL", "0") == "1" and not self.hound and self.nd % 4 == 0
                                  and t.gym.amd_pd_tail_supported(t.sim))
        if not ok or not (t.torques.is_contiguous() and t.actions.is_contiguous()):
            return None
        b = self._buffers()
        if any(x % 16 for x in (b.torques, b.actions, b.last_actions, b.last_dof_vel, b.dof_state)):
            return None
        self._seq = (self._seq + 1) & 0x7FFFFFFF
        b.seq = self._seq
        return self.p, b

    def after_fused_tail(self):
        """The host side of post_a once the fused launch ran it (check_termination's bool reset_buf)."""
        self.task.reset_buf = self.reset_bool

    _tail_ok = None
    _ids_buf = None

    def post_ab_applies(self) -> bool:
        """post_a and the (optimistic) observations can be one launch (gt_anymal_post_physics_ab): AnymalTerrain on
        the plane, 12 dofs, in-kernel noise draws (or none), fused observation outputs, post_a's vector rows.
        Opt-in (GT_POST_AB=1): measured slower than the two launches -- 0.170 vs 0.131 ms per headline step
        (profiles/r06zd_post_ab_ab.txt): the element loop must call k_post_b's body out of line (inlining it in a
        loop crashes this compiler), and the call's by-reference structs cost ~570 B of scratch per lane."""
        ok = self._ab_ok
        if ok is None:
            t = self.task
            ok = self._ab_ok = (os.environ.get("GT_POST_AB", "0") == "1" and not self.hound and self.nd == 12
                                and getattr(t, "_heights_dev", None) is None)
        t = self.task
        return (ok and (self.inkernel_rng or not t.add_noise) and not t.dr_randomizations.get("observations", None)
                and t.torques.is_contiguous() and t.actions.is_contiguous())

    _ab_ok = None

    def post_ab(self):
        """post_a() + observe() as one launch (gymtask ABI 5): the counters, termination, reward, the reset count
        and masks, then the observations with their noise, time_outs and the clamped copy."""
        t = self.task
        b = self._buffers()
        if any(x % 16 for x in (b.torques, b.actions, b.last_actions, b.last_dof_vel, b.dof_state)):
            self.post_a()
            self.observe()
            return
        self._seq = (self._seq + 1) & 0x7FFFFFFF
        b.seq = self._seq
        plan = self.planner.plan(t.obs_buf.numel()) if t.add_noise else None
        obs = torch.empty_like(t.obs_buf)
        time_outs = torch.empty(t.num_envs, dtype=torch.bool, device=t.device)
        b.obs_out, b.time_outs, b.clip_obs = obs.data_ptr(), time_outs.data_ptr(), float(t.clip_obs)
        b.obs_mirror = self._mirror_ptr
        _check(lib().gt_anymal_post_physics_ab(self.p, b, plan, self._stream()), "gt_anymal_post_physics_ab")
        t.reset_buf = self.reset_bool
        t._fused_outputs = (time_outs, obs)
        t._obs_mirrored = obs if self._mirror_ptr else None

    def num_resets(self) -> int:
        """Envs the last post_a flagged for reset, read back through the stream (synchronising)."""
        return int(self.reset_count[2].item())

    # The host learns the reset count from post_a's last workgroup, which stores it into pinned
    # host memory; meanwhile the GPU already builds the observations of the common no-reset step
    # (see AnymalTerrain.post_physics_step).
    WAIT_TIMEOUT_MS = 60000

    def wait_reset_count(self) -> int:
        _check(lib().gt_wait_host_seq(self._host_words, self._seq, self.WAIT_TIMEOUT_MS, C.byref(self._count_out)),
               "gt_wait_host_seq")
        self.last_reset_count = int(self._count_out.value)
        return self.last_reset_count

    def rng_snapshot(self):
        """Host-side generator position (the device generator's Philox offset; with torch-drawn
        buffers also the CPU generator, for callers that draw there).  Restoring it discards the
        draws made after the snapshot."""
        g = self.planner.gen
        return g.get_offset(), (None if self.inkernel_rng else torch.get_rng_state())

    def rng_restore(self, snap):
        off, cpu = snap
        self.planner.gen.set_offset(off)
        if cpu is not None:
            torch.set_rng_state(cpu)

    def observe(self, rand_like=None):
        """compute_observations + noise + history (anymal_terrain.py:477-485), one kernel.  The
        noise is torch.rand_like(obs_buf): evaluated in-kernel (inkernel_rng) or drawn by
        ``rand_like`` into a buffer; either way the generator advances as the reference's."""
        t = self.task
        if getattr(t, "_heights_dev", None) is not None:
            self.measure_heights()
        if not t.add_noise:
            self.post_b(None)
        elif self.inkernel_rng:
            self.post_b(None, self.planner.plan(t.obs_buf.numel()))
        else:
            self.post_b((rand_like or torch.rand_like)(t.obs_buf))

    def measure_heights(self):
        """get_heights for the trimesh terrain (anymal_terrain.py:515-538), one kernel into
        task._heights_dev (= task.measured_heights)."""
        t = self.task
        ter = t.terrain
        hs = t.height_samples
        pts = t.height_points
        assert hs.dtype == torch.int16 and hs.is_contiguous() and pts.is_contiguous()
        out = t._heights_dev
        _check(lib().gt_measure_heights(hs.data_ptr(), hs.shape[0], hs.shape[1], float(ter.border_size),
                                        float(ter.horizontal_scale), float(ter.vertical_scale),
                                        t.root_states.data_ptr(), pts.data_ptr(), t.num_envs, pts.shape[1],
                                        out.data_ptr(), self._stream()), "gt_measure_heights")
        t.measured_heights = out

    def reset(self, env_ids_int32, pos_offset, vel, cmd_x, cmd_y, cmd_h):
        t = self.task
        k = int(env_ids_int32.numel())
        cx, cy, ch = (x.reshape(-1).contiguous() for x in (cmd_x, cmd_y, cmd_h))
        ids = env_ids_int32.contiguous()
        _check(lib().gt_anymal_reset(self.p, self._buffers(), ids.data_ptr(), k, pos_offset.contiguous().data_ptr(),
                                     vel.contiguous().data_ptr(), cx.data_ptr(), cy.data_ptr(), ch.data_ptr(),
                                     self.ep_out.data_ptr(), self._stream()), "gt_anymal_reset")
        if t.reset_buf is not self.reset_bool:  # before the first step reset_buf is VecTask's int64 buffer
            t.reset_buf[ids.long()] = 1
        vals = self.ep_out / (k * t.max_episode_length_s)
        t.extras["episode"] = {"rew_" + name: vals[i] for i, name in enumerate(self.TERMS)}
        if self._terrain_level is None or t.custom_origins:
            self._terrain_level = torch.mean(t.terrain_levels.float())
        t.extras["episode"]["terrain_level"] = self._terrain_level
        self._keep = (ids, pos_offset, vel, cx, cy, ch)

    def reset_flagged(self, k: int, rand_unit=None, defer_extras: bool = False):
        """reset_idx for the k envs the last post_a flagged, in one kernel (plane and trimesh terrain).

        Draws u ~ U[0,1) with ``rand_unit(shape, device)`` in the reference's order and shapes
        (anymal_terrain.py:385-398: dof offsets, dof velocities, [trimesh: root x, y], cmd x, cmd y,
        cmd heading), so the RNG stream advances exactly as torch_rand_float's would; the kernel
        applies the affine maps, the trimesh curriculum (update_terrain_level, :427-435), ranks the
        flagged envs (nonzero order) and fills extras["episode"]."""
        t = self.task
        dev, nd = t.device, self.nd
        tr = self._terrain_reset() if t.custom_origins else None
        h = self._h
        d = self._draws
        if d is None:  # the affine maps are fixed per task
            d = self._draws = GtAnymalResetDraws()
            for name, (lo, hi) in (("pos", (0.5, 1.5)), ("vel", (-0.1, 0.1)), ("cmd_x", t.command_x_range),
                                   ("cmd_y", t.command_y_range), ("cmd_h", t.command_yaw_range)):
                setattr(d, name + "_range", float(hi - lo))
                setattr(d, name + "_lower", float(lo))
        # draw order (anymal_terrain.py:385-398, useful_hound.py:571-605): dof offsets, dof velocities,
        # [trimesh: root x, y], [UsefulHound: arm reset noise (k, 6)], command x, y, heading
        if self.inkernel_rng:
            u = None
            d.u_pos = d.u_vel = d.u_cmd_x = d.u_cmd_y = d.u_cmd_h = None
            sizes = [k * nd, k * nd] + ([2 * k] if tr is not None else []) + ([6 * k] if h is not None else [])
            plans = self.planner.plan_many(sizes + [k, k, k])
            d.plan_pos, d.plan_vel = plans[0], plans[1]
            d.plan_cmd_x, d.plan_cmd_y, d.plan_cmd_h = plans[-3:]
            rest = plans[2:-3]
            if tr is not None:
                tr.u_root_xy = None
                tr.plan_root_xy = rest.pop(0)
            if h is not None:
                h.u_arm = None
                h.plan_arm = rest.pop(0)
        else:
            u = [rand_unit((k, nd), dev), rand_unit((k, nd), dev)]
            if tr is not None:
                u.append(rand_unit((k, 2), dev))
            if h is not None:
                u.append(rand_unit((k, 6), dev))  # torch.rand((k, 6)), useful_hound.py:596
            u += [rand_unit((k, 1), dev) for _ in range(3)]
            d.u_pos, d.u_vel = u[0].data_ptr(), u[1].data_ptr()
            d.u_cmd_x, d.u_cmd_y, d.u_cmd_h = (x.data_ptr() for x in u[-3:])
            extra = u[2:-3]
            if tr is not None:
                tr.u_root_xy = extra.pop(0).data_ptr()
            if h is not None:
                h.u_arm = extra.pop(0).data_ptr()
        # the flagged env ids: a prefix of one persistent buffer (stream order keeps the previous reset's readers
        # ahead of this write); extras["episode"] gets a fresh buffer per reset, as the reference's torch.mean
        ids_buf = self._ids_buf
        if ids_buf is None or ids_buf.numel() < t.num_envs:
            ids_buf = self._ids_buf = torch.empty(t.num_envs, dtype=torch.int32, device=dev)
        ids = ids_buf[:k]
        ep = torch.empty(len(self.TERMS) + 1, dtype=torch.float32, device=dev)
        _check(lib().gt_anymal_reset_flagged(self.p, self._buffers(check=False), k, d, tr, ids.data_ptr(), ep.data_ptr(),
                                             float(t.max_episode_length_s), self.reset_scratch.data_ptr(),
                                             self._stream()), "gt_anymal_reset_flagged")
        t._set_reset_state(ids)
        self._keep = (u, ids)
        # extras["episode"] (fresh 0-d tensors per reset, as the reference's torch.mean results): with
        # defer_extras the caller builds it with finish_reset() once the next launches are queued
        self._pending_extras = (ep, tr is not None)
        if not defer_extras:
            self.finish_reset()

    def reset_observe_applies(self) -> bool:
        """The reset step's sequence can be one C call (gt_anymal_reset_observe): plane AnymalTerrain, in-kernel
        draws, fused observation outputs, and a sim whose indexed sets libgymsim does itself.  (The task-level
        conditions are fixed after construction and cached; inkernel_rng and the observation DR are re-read.)"""
        t = self.task
        if not self.inkernel_rng or t.dr_randomizations.get("observations", None):
            return False
        ok = self._ro_ok
        if ok is None:
            ok = self._ro_ok = self._reset_observe_static()
        return ok

    _ro_ok = None

    def _reset_observe_static(self) -> bool:
        t = self.task
        return (self.inkernel_rng and not self.hound and not t.custom_origins and getattr(t, "_heights_dev", None) is None
                and not t.dr_randomizations.get("observations", None) and hasattr(t.sim, "handle")
                and type(t)._set_reset_state is _anymal_set_reset_state())

    def reset_observe(self, k: int):
        """reset_flagged(k) + observe() of a reset step in one host call (gymtask ABI 5, gt_anymal_reset_observe:
        the reset draws' plans, k_reset_flagged, gymsim's one-launch root / dof indexed sets through a C callback,
        k_post_b with the noise plan); the generator ends where the Python sequence leaves it.  extras["episode"] is
        left pending for finish_reset()."""
        args, off, outs = self._ro_prepare()
        _check(lib().gt_anymal_reset_observe(self.p, args[0], k, *args[1:]), "gt_anymal_reset_observe")
        self._ro_done(off, outs)

    def wait_reset_observe(self, snap) -> int:
        """wait_reset_count() and, when the count is > 0, reset_observe(count) in the same C call (the reset's first
        launch follows the count with no Python in between).  snap: rng_snapshot() taken before the optimistic
        observation (None: the generator has not moved since).  Returns the count; a reset's extras["episode"] is
        left pending for finish_reset()."""
        # the reset draws start where the optimistic noise did (the rolled-back offset); with no reset the generator
        # stays after the optimistic draws
        args, off, outs = self._ro_prepare(None if snap is None else snap[0])
        cnt = self._count_out
        rc = lib().gt_anymal_wait_reset_observe(self._host_words, self._seq, self.WAIT_TIMEOUT_MS, C.byref(cnt),
                                                self.p, *args)
        _check(rc, "gt_anymal_wait_reset_observe")
        k = self.last_reset_count = int(cnt.value)
        if k > 0:
            self._ro_done(off, outs)
        return k

    def _ro_prepare(self, start_offset=None):
        t = self.task
        d = self._draws
        if d is None:
            d = self._draws = GtAnymalResetDraws()
            for name, (lo, hi) in (("pos", (0.5, 1.5)), ("vel", (-0.1, 0.1)), ("cmd_x", t.command_x_range),
                                   ("cmd_y", t.command_y_range), ("cmd_h", t.command_yaw_range)):
                setattr(d, name + "_range", float(hi - lo))
                setattr(d, name + "_lower", float(lo))
        ids_buf = self._ids_buf
        if ids_buf is None or ids_buf.numel() < t.num_envs:
            ids_buf = self._ids_buf = torch.empty(t.num_envs, dtype=torch.int32, device=t.device)
        # fresh outputs (extras["episode"], the observations, time_outs): allocated after the previous reset's call,
        # off the host path between the count and this one
        nxt = self._ro_next
        if nxt is None or nxt[1].shape != t.obs_buf.shape:
            nxt = self._ro_next = self._ro_alloc()
        ep, obs, time_outs = nxt
        b = self._buffers(check=False)
        b.obs_out, b.time_outs, b.clip_obs = obs.data_ptr(), time_outs.data_ptr(), float(t.clip_obs)
        b.obs_mirror = self._mirror_ptr
        cb = self._set_state_cb
        if cb is None:
            from isaacgymenv_amd.isaacgym import _lib as gs
            cb = self._set_state_cb = C.cast(gs.lib().gs_sim_set_root_and_dof, C.c_void_p).value
        g = self.planner.gen
        off = C.c_uint64(g.get_offset() if start_offset is None else start_offset)
        args = (b, self._draws, ids_buf.data_ptr(), ep.data_ptr(), float(t.max_episode_length_s),
                self.reset_scratch.data_ptr(), g.initial_seed(), C.byref(off), self.planner.grid_cap,
                int(bool(t.add_noise)), cb, t.sim.handle, t.root_states.data_ptr(), t.dof_state.data_ptr(),
                self._stream())
        return args, off, nxt

    def _ro_done(self, off, outs):
        t = self.task
        ep, obs, time_outs = outs
        self.planner.gen.set_offset(off.value)
        t._fused_outputs = (time_outs, obs)
        t._obs_mirrored = obs if self._mirror_ptr else None
        self._keep = (self._ids_buf, ep)
        self._pending_extras = (ep, False)
        self._ro_next = self._ro_alloc()

    def _ro_alloc(self):
        t = self.task
        return (torch.empty(len(self.TERMS) + 1, dtype=torch.float32, device=t.device), torch.empty_like(t.obs_buf),
                torch.empty(t.num_envs, dtype=torch.bool, device=t.device))

    _set_state_cb = None
    _ro_next = None
    _mirror_ptr = None  # set_obs_mirror

    def set_obs_mirror(self, buf):
        """A [num_envs][num_obs] float32 device buffer that also receives every step's observations (the tensor
        VecTask returns stays a fresh one); None stops it.  The task's _obs_mirrored names the returned tensor whose
        values the mirror holds."""
        t = self.task
        if buf is not None:
            assert buf.dtype == torch.float32 and buf.is_contiguous() and tuple(buf.shape) == tuple(t.obs_buf.shape) \
                and buf.device == t.obs_buf.device, "obs mirror: [num_envs][num_obs] float32 on the task's device"
        self._mirror_buf = buf
        self._mirror_ptr = buf.data_ptr() if buf is not None else None
        t._obs_mirrored = None

    def finish_reset(self):
        """extras["episode"] of the last reset_flagged(defer_extras=True); a no-op when none is pending."""
        pend, self._pending_extras = self._pending_extras, None
        if pend is None:
            return
        ep, has_terrain = pend
        t = self.task
        if has_terrain:
            last = None
        else:
            if self._terrain_level is None:
                self._terrain_level = torch.mean(t.terrain_levels.float())
            last = self._terrain_level
        t.extras["episode"] = EpisodeExtras(self._ep_keys, ep, last)

    def _terrain_reset(self):
        """gt_anymal_terrain_reset over the task's curriculum tensors (rebuilt when the task rebinds one)."""
        t = self.task
        cur = (t.terrain_levels, t.terrain_types, t.env_origins, t.terrain_origins)
        tr = getattr(self, "_tr", None)
        if tr is None or any(x is not y for x, y in zip(cur, self._tr_bound)):
            for x, dt in zip(cur, (torch.int64, torch.int64, torch.float32, torch.float32)):
                assert x.is_contiguous() and x.dtype == dt and x.device.type == "cuda"
            tr = GtAnymalTerrainReset()
            tr.terrain_levels, tr.terrain_types, tr.env_origins, tr.terrain_origins = (x.data_ptr() for x in cur)
            tr.env_rows, tr.env_cols = int(t.terrain.env_rows), int(t.terrain.env_cols)
            tr.env_length = float(t.terrain.env_length)
            tr.max_episode_length_s = float(t.max_episode_length_s)
            tr.xy_range, tr.xy_lower = 1.0, -0.5  # torch_rand_float(-0.5, 0.5, (k, 2)), :396
            self._tr, self._tr_bound = tr, cur
        tr.update_levels = int(bool(t.init_done and t.curriculum))
        return tr

    def post_b(self, noise, noise_plan=None):
        """Observations (+noise), history buffers, and VecTask's time_outs / clamped obs (vec_task.py:393-402)."""
        t = self.task
        b = self._buffers(check=False)
        fuse_outputs = not t.dr_randomizations.get("observations", None)
        if fuse_outputs:
            obs = torch.empty_like(t.obs_buf)
            time_outs = torch.empty(t.num_envs, dtype=torch.bool, device=t.device)
            b.obs_out, b.time_outs, b.clip_obs = obs.data_ptr(), time_outs.data_ptr(), float(t.clip_obs)
        b.obs_mirror = self._mirror_ptr if fuse_outputs else None
        _check(lib().gt_anymal_post_physics_b(self.p, b, _ptr(noise), noise_plan, self._stream()),
               "gt_anymal_post_physics_b")
        if fuse_outputs:
            t._fused_outputs = (time_outs, obs)
            t._obs_mirrored = obs if self._mirror_ptr else None
