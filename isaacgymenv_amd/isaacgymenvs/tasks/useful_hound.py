"""UsefulHound: quadruped + 6-DoF arm (reference ``tasks/useful_hound.py``), SURVEY.md section 8 row A14.

The task layer restates the reference's behaviour on our simulator; the physics (19 welded dynamic
bodies, 24 reported links, 84 plane-contact candidates) runs in the HIP lane kernel, and the
tensor API's link kinematics (rigid-body state, Jacobian, mass matrix) in gs_kinematics.hip.

* ``pre_physics_step`` (useful_hound.py:695-726): ``decimation`` x [arm OSC torques from the
  *step-start* Jacobian / mass matrix (they are refreshed once per env step, in post_physics_step)
  and the never-refreshed end-effector state; leg PD torques; set efforts; simulate; refresh dof];
* the OSC (:660-691) is the reference's: ``M_eef = (J M^-1 J^T)^-1``, ``u = J^T M_eef (kp dpose -
  kd v_eef) + (1 - J^T M_eef J M^-1) M u_null``, clamped to the arm's effort limits, with
  ``J = jacobian[:, joint_dict['joint6'], :, :6]`` and ``M = mass_matrix[:, -6:, -6:]`` exactly as
  the reference indexes them;
* ``post_physics_step`` (:728-760): refresh root / contacts / Jacobian / mass matrix, push every
  ``push_interval`` steps, base-frame velocities, heading command, termination on trunk, thigh and
  shoulder contacts, reward, same-step reset, observations (204 = AnymalTerrain's 188 with 18
  actions + end-effector position (3) + quaternion (4) + arm command (3)) and noise;
* RNG order: friction buckets, terrain levels / types at creation; per reset: leg dof offsets,
  leg dof velocities, [trimesh root xy], arm reset noise, command x, y, heading; per step: push
  draw and observation noise.
On the GPU pipeline the leg PD + arm OSC of each decimation step is one HIP kernel (gt_hound_control,
float64 6x6 algebra, one lane per env) instead of ~40 torch launches with two host-synchronising
batched inverses, and the post-physics tail is AnymalTerrain's fused kernels with the UsefulHound
extension (gt_anymal_hound: termination, reward, reset with the arm draw, 204-wide observations)
without a nonzero() / host sync; the torch statements remain the CPU-pipeline path (and the
golden-tested spec).
The end-effector state comes from the rigid-body state tensor, which the reference acquires but
never refreshes outside its debug-viz branch: it holds the prepared (initial) state, and so does
ours.
"""
from __future__ import annotations

import numpy as np
import torch

from isaacgym import gymapi, gymtorch

from ..utils.torch_jit_utils import (get_axis_params, quat_apply, quat_rotate_inverse, tensor_clamp, to_torch,
                                     torch_rand_float)
from .anymal_terrain import REWARD_TERMS, AnymalTerrain, torch_rand_unit, wrap_to_pi
from .base.vec_task import VecTask

HOUND_LEG_DOFS, HOUND_ARM_DOFS = 12, 6


class UsefulHound(AnymalTerrain):
    supports_fused_physics = False

    def __init__(self, cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture,
                 force_render):
        self.cfg = cfg
        env = cfg["env"]
        learn = env["learn"]
        self.height_samples = None
        self.custom_origins = False
        self.debug_viz = env["enableDebugVis"]
        self.init_done = False
        self.lin_vel_scale = learn["linearVelocityScale"]
        self.ang_vel_scale = learn["angularVelocityScale"]
        self.dof_pos_scale = learn["dofPositionScale"]
        self.dof_vel_scale = learn["dofVelocityScale"]
        self.height_meas_scale = learn["heightMeasurementScale"]
        self.action_scale = env["control"]["actionScale"]
        # arm (useful_hound.py:89-104)
        self.arm_action_scale = env["control"]["houndarmactionScale"]
        self.houndarm_dof_noise = env["houndarmDofNoise"]
        self.arm_reward_settings = {"r_dist_scale": learn["distRewardScale"], "r_vel_scale": learn["velRewardScale"]}
        self.arm_control_type = env["houndarmcontrolType"]
        arm_ranges = env["randomArmCommandPositionRanges"]
        self.arm_command_x_range = arm_ranges["x"]
        self.arm_command_y_range = arm_ranges["y"]
        self.arm_command_z_range = arm_ranges["z"]

        self.rew_scales = {
            "termination": learn["terminalReward"],
            "lin_vel_xy": learn["linearVelocityXYRewardScale"],
            "lin_vel_z": learn["linearVelocityZRewardScale"],
            "ang_vel_z": learn["angularVelocityZRewardScale"],
            "ang_vel_xy": learn["angularVelocityXYRewardScale"],
            "orient": learn["orientationRewardScale"],
            "torque": learn["torqueRewardScale"],
            "joint_acc": learn["jointAccRewardScale"],
            "base_height": learn["baseHeightRewardScale"],
            "air_time": learn["feetAirTimeRewardScale"],
            "collision": learn["kneeCollisionRewardScale"],
            "stumble": learn["feetStumbleRewardScale"],
            "action_rate": learn["actionRateRewardScale"],
            "hip": learn["hipRewardScale"],
        }
        ranges = env["randomCommandVelocityRanges"]
        self.command_x_range = ranges["linear_x"]
        self.command_y_range = ranges["linear_y"]
        self.command_yaw_range = ranges["yaw"]
        init = env["baseInitState"]
        self.base_init_state = init["pos"] + init["rot"] + init["vLinear"] + init["vAngular"]
        self.named_hound_default_joint_angles = env["defaultJointAngles"]
        self.decimation = env["control"]["decimation"]
        self.dt = self.decimation * cfg["sim"]["dt"]
        self.max_episode_length_s = learn["episodeLength_s"]
        self.max_episode_length = int(self.max_episode_length_s / self.dt + 0.5)
        self.push_interval = int(learn["pushInterval_s"] / self.dt + 0.5)
        self.allow_knee_contacts = learn["allowKneeContacts"]
        self.Kp = env["control"]["stiffness"]
        self.Kd = env["control"]["damping"]
        self.curriculum = env["terrain"]["curriculum"]
        for k in self.rew_scales:
            self.rew_scales[k] *= self.dt

        VecTask.__init__(self, config=cfg, rl_device=rl_device, sim_device=sim_device,
                         graphics_device_id=graphics_device_id, headless=headless,
                         virtual_screen_capture=virtual_screen_capture, force_render=force_render)

        root = self.gym.acquire_actor_root_state_tensor(self.sim)
        dofs = self.gym.acquire_dof_state_tensor(self.sim)
        contacts = self.gym.acquire_net_contact_force_tensor(self.sim)
        self.gym.refresh_dof_state_tensor(self.sim)
        self.gym.refresh_actor_root_state_tensor(self.sim)
        self.gym.refresh_net_contact_force_tensor(self.sim)
        self.root_states = gymtorch.wrap_tensor(root)
        self.dof_state = gymtorch.wrap_tensor(dofs)
        nd = self.total_num_dof
        self.hound_dof_pos = self.dof_state.view(self.num_envs, nd, 2)[:, 0:HOUND_LEG_DOFS, 0]
        self.hound_dof_vel = self.dof_state.view(self.num_envs, nd, 2)[:, 0:HOUND_LEG_DOFS, 1]
        self.contact_forces = gymtorch.wrap_tensor(contacts).view(self.num_envs, -1, 3)

        dev = self.device
        zeros = lambda *s: torch.zeros(*s, dtype=torch.float, device=dev, requires_grad=False)  # noqa: E731
        self.common_step_counter = 0
        self.extras = {}
        self.noise_scale_vec = self._get_noise_scale_vec(cfg)
        self.commands = zeros(self.num_envs, 4)
        self.commands_scale = torch.tensor([self.lin_vel_scale, self.lin_vel_scale, self.ang_vel_scale],
                                           device=dev, requires_grad=False)
        self.gravity_vec = to_torch(get_axis_params(-1.0, self.up_axis_idx), device=dev).repeat((self.num_envs, 1))
        self.forward_vec = to_torch([1.0, 0.0, 0.0], device=dev).repeat((self.num_envs, 1))
        self.torques = zeros(self.num_envs, self.num_actions)
        self.actions = zeros(self.num_envs, self.num_actions)
        self.last_actions = zeros(self.num_envs, self.num_actions)
        self.feet_air_time = zeros(self.num_envs, 4)
        self.last_hound_dof_vel = torch.zeros_like(self.hound_dof_vel)
        self.height_points = self.init_height_points()
        self.measured_heights = None
        self.hound_default_dof_pos = torch.zeros_like(self.hound_dof_pos, dtype=torch.float, device=dev,
                                                      requires_grad=False)
        for i in range(self.num_actions - HOUND_ARM_DOFS):
            self.hound_default_dof_pos[:, i] = self.named_hound_default_joint_angles[self.dof_names[i]]
        self.episode_sums = {k: zeros(self.num_envs) for k in REWARD_TERMS}
        # arm OSC gains and limits (useful_hound.py:229-246)
        self.houndarm_default_dof_pos = to_torch([0, 0, 0, 0, 0, 0], device=dev)
        self.arm_kp = to_torch([150.0] * 6, device=dev)
        self.arm_kd = 2 * torch.sqrt(self.arm_kp)
        self.arm_kp_null = to_torch([10.0] * 6, device=dev)
        self.arm_kd_null = 2 * torch.sqrt(self.arm_kp_null)
        self.arm_cmd_limit = to_torch([0.1, 0.1, 0.1, 0.5, 0.5, 0.5], device=dev).unsqueeze(0)
        self.arm_commands = zeros(self.num_envs, 3)
        self._fused_refreshed = False
        self._control = None
        self._kernels = None
        self._heights_dev = None
        if self.device != "cpu":
            # GPU pipeline: the leg PD + arm OSC of every decimation step is one kernel (gt_hound_control),
            # the post-physics tail the fused AnymalTerrain kernels with the UsefulHound extension
            from ...gymtask import AnymalTailKernels, HoundControlKernel  # fail loudly without libgymtask.so
            self._control = HoundControlKernel(self)
            self._torque_buf = zeros(self.num_envs, self.num_actions)
            self.torques = self._torque_buf
            if self.custom_origins:
                self._heights_dev = zeros(self.num_envs, self.num_height_points)
                self.height_points = self.height_points.contiguous()
            self._kernels = AnymalTailKernels(self)
        self.gym.refresh_actor_root_state_tensor(self.sim)
        self.gym.refresh_net_contact_force_tensor(self.sim)
        self.gym.refresh_jacobian_tensors(self.sim)
        self.gym.refresh_mass_matrix_tensors(self.sim)
        self.reset_idx(torch.arange(self.num_envs, device=self.device))
        self.init_done = True

    # the generic terms of AnymalTerrain read dof_pos / dof_vel / last_dof_vel: the leg dofs here
    @property
    def dof_pos(self):
        return self.hound_dof_pos

    @property
    def dof_vel(self):
        return self.hound_dof_vel

    # ------------------------------------------------------------------ creation
    def _create_envs(self, num_envs, spacing, num_per_row):
        """useful_hound.py:312-465."""
        asset_root, asset_file = self._asset_location()
        ua = self.cfg["env"]["urdfAsset"]
        opts = gymapi.AssetOptions()
        opts.default_dof_drive_mode = gymapi.DOF_MODE_EFFORT
        opts.collapse_fixed_joints = ua["collapseFixedJoints"]
        opts.replace_cylinder_with_capsule = False
        opts.flip_visual_attachments = False
        opts.fix_base_link = ua["fixBaseLink"]
        opts.density = 0.001
        opts.angular_damping = 0.0
        opts.linear_damping = 0.0
        opts.armature = 0.0
        opts.thickness = 0.01
        opts.disable_gravity = False
        asset = self.gym.load_asset(self.sim, asset_root, asset_file, opts)
        self.total_num_dof = self.gym.get_asset_dof_count(asset)
        self.hound_num_dof = self.total_num_dof - HOUND_ARM_DOFS
        self.arm_num_dof = self.total_num_dof - self.hound_num_dof
        self.num_dof = self.total_num_dof
        self.num_bodies = self.gym.get_asset_rigid_body_count(asset)

        shape_props = self.gym.get_asset_rigid_shape_properties(asset)
        fr = self.cfg["env"]["learn"]["frictionRange"]
        num_buckets = 100
        friction_buckets = torch_rand_float(fr[0], fr[1], (num_buckets, 1), device=self.device)

        self.base_init_state = to_torch(self.base_init_state, device=self.device, requires_grad=False)
        start_pose = gymapi.Transform()
        start_pose.p = gymapi.Vec3(*self.base_init_state[:3])
        body_names = self.gym.get_asset_rigid_body_names(asset)
        self.dof_names = self.gym.get_asset_dof_names(asset)
        feet_names = [s for s in body_names if ua["footName"] in s]
        knee_names = [s for s in body_names if ua["kneeName"] in s]
        base_names = [s for s in body_names if ua["baseName"] in s]
        self.feet_indices = torch.zeros(len(feet_names), dtype=torch.long, device=self.device, requires_grad=False)
        self.knee_indices = torch.zeros(len(knee_names), dtype=torch.long, device=self.device, requires_grad=False)
        self.base_indices = torch.zeros(len(base_names), dtype=torch.long, device=self.device, requires_grad=False)
        self.base_index = 0

        # arm dofs: effort drive, no PhysX gains; limits / efforts kept for the OSC (:356-374)
        dof_props = self.gym.get_asset_dof_properties(asset)
        lower, upper, effort = [], [], []
        for a in range(self.arm_num_dof):
            i = a + self.hound_num_dof
            dof_props["driveMode"][i] = gymapi.DOF_MODE_EFFORT
            dof_props["stiffness"][i] = 0.0
            dof_props["damping"][i] = 0.0
            lower.append(dof_props["lower"][i])
            upper.append(dof_props["upper"][i])
            effort.append(dof_props["effort"][i])
        self.houndarm_dof_lower_limits = to_torch(lower, device=self.device)
        self.houndarm_dof_upper_limits = to_torch(upper, device=self.device)
        self._houndarm_effort_limits = to_torch(effort, device=self.device)
        self.houndarm_dof_speed_scales = torch.ones_like(self.houndarm_dof_lower_limits)

        tcfg = self.cfg["env"]["terrain"]
        self.env_origins = torch.zeros(self.num_envs, 3, device=self.device, requires_grad=False)
        if not self.curriculum:
            tcfg["maxInitMapLevel"] = tcfg["numLevels"] - 1
        self.terrain_levels = torch.randint(0, tcfg["maxInitMapLevel"] + 1, (self.num_envs,), device=self.device)
        self.terrain_types = torch.randint(0, tcfg["numTerrains"], (self.num_envs,), device=self.device)
        if self.custom_origins:
            self.terrain_origins = torch.from_numpy(self.terrain.env_origins).to(self.device).to(torch.float)
            spacing = 0.0
        lower_v = gymapi.Vec3(-spacing, -spacing, 0.0)
        upper_v = gymapi.Vec3(spacing, spacing, spacing)
        self.anymal_handles = []
        self.envs = []
        friction_host = friction_buckets.cpu().numpy()[:, 0]
        for i in range(self.num_envs):
            env_handle = self.gym.create_env(self.sim, lower_v, upper_v, num_per_row)
            if self.custom_origins:
                self.env_origins[i] = self.terrain_origins[self.terrain_levels[i], self.terrain_types[i]]
                pos = self.env_origins[i].clone()
                pos[:2] += torch_rand_float(-1.0, 1.0, (2, 1), device=self.device).squeeze(1)
                start_pose.p = gymapi.Vec3(*pos.tolist())
            for sp in shape_props:
                sp.friction = friction_host[i % num_buckets]
            self.gym.set_asset_rigid_shape_properties(asset, shape_props)
            handle = self.gym.create_actor(env_handle, asset, start_pose, "UsefulHound", i, 0, 0)
            self.gym.set_actor_dof_properties(env_handle, handle, dof_props)
            self.envs.append(env_handle)
            self.anymal_handles.append(handle)
        find = lambda n: self.gym.find_actor_rigid_body_handle(self.envs[0], self.anymal_handles[0], n)  # noqa: E731
        for i, n in enumerate(feet_names):
            self.feet_indices[i] = find(n)
        for i, n in enumerate(knee_names):
            self.knee_indices[i] = find(n)
        for i, n in enumerate(base_names):
            self.base_indices[i] = find(n)
        self.eef_index = find("end_link")
        self.base_index = find("trunk")

        # arm tensors (useful_hound.py:438-464)
        rb = self.gym.acquire_rigid_body_state_tensor(self.sim)
        self._rigid_body_state = gymtorch.wrap_tensor(rb).view(self.num_envs, -1, 13)
        dof3 = gymtorch.wrap_tensor(self.gym.acquire_dof_state_tensor(self.sim)).view(self.num_envs, -1, 2)
        self._q = dof3[:, HOUND_LEG_DOFS:, 0]
        self._qd = dof3[:, HOUND_LEG_DOFS:, 1]
        self._eef_state = self._rigid_body_state[:, self.eef_index, :]
        jacobian = gymtorch.wrap_tensor(self.gym.acquire_jacobian_tensor(self.sim, "UsefulHound"))
        hand_joint_index = self.gym.get_actor_joint_dict(self.envs[0], self.anymal_handles[0])["joint6"]
        self._j_eef = jacobian[:, hand_joint_index, :, :6]
        mm = gymtorch.wrap_tensor(self.gym.acquire_mass_matrix_tensor(self.sim, "UsefulHound"))
        self._mm = mm[:, -6:, -6:]
        self._jac_full, self._mm_full, self._hand_joint_index = jacobian, mm, hand_joint_index
        self._pos_control = torch.zeros((self.num_envs, self.arm_num_dof), dtype=torch.float, device=self.device)
        self._effort_control = torch.zeros_like(self._pos_control)
        self._arm_control = self._effort_control[:, :6]
        self._global_indices = torch.arange(self.num_envs, dtype=torch.int32, device=self.device).view(self.num_envs, -1)

    # ------------------------------------------------------------------ terms
    def check_termination(self):
        """useful_hound.py:467-480: trunk, thigh or shoulder contact, or the episode limit."""
        cf = self.contact_forces
        self.reset_buf = torch.norm(cf[:, self.base_index, :], dim=1) > 1.0
        self.reset_buf = self.reset_buf | torch.any(torch.norm(cf[:, self.knee_indices, :], dim=2) > 1.0, dim=1)
        self.reset_buf = self.reset_buf | torch.any(torch.norm(cf[:, self.base_indices, :], dim=2) > 1.0, dim=1)
        time_out = self.progress_buf >= self.max_episode_length - 1
        self.reset_buf = self.reset_buf | time_out

    def compute_observations(self):
        self.measured_heights = self.get_heights()
        heights = torch.clip(self.root_states[:, 2].unsqueeze(1) - 0.5 - self.measured_heights, -1, 1.0) \
            * self.height_meas_scale
        self.obs_buf = torch.cat((self.base_lin_vel * self.lin_vel_scale,
                                  self.base_ang_vel * self.ang_vel_scale,
                                  self.projected_gravity,
                                  self.commands[:, :3] * self.commands_scale,
                                  self.hound_dof_pos * self.dof_pos_scale,
                                  self.hound_dof_vel * self.dof_vel_scale,
                                  heights,
                                  self.actions,
                                  self._eef_state[:, :3],
                                  self._eef_state[:, 3:7],
                                  self.arm_commands[:, :]), dim=-1)

    def compute_reward(self):
        """useful_hound.py:499-567 (AnymalTerrain's terms; collision also counts shoulder contacts)."""
        rs = self.rew_scales
        cf = self.contact_forces
        lin_vel_error = torch.sum(torch.square(self.commands[:, :2] - self.base_lin_vel[:, :2]), dim=1)
        ang_vel_error = torch.square(self.commands[:, 2] - self.base_ang_vel[:, 2])
        r = {}
        r["lin_vel_xy"] = torch.exp(-lin_vel_error / 0.25) * rs["lin_vel_xy"]
        r["ang_vel_z"] = torch.exp(-ang_vel_error / 0.25) * rs["ang_vel_z"]
        r["lin_vel_z"] = torch.square(self.base_lin_vel[:, 2]) * rs["lin_vel_z"]
        r["ang_vel_xy"] = torch.sum(torch.square(self.base_ang_vel[:, :2]), dim=1) * rs["ang_vel_xy"]
        r["orient"] = torch.sum(torch.square(self.projected_gravity[:, :2]), dim=1) * rs["orient"]
        r["base_height"] = torch.square(self.root_states[:, 2] - 0.52) * rs["base_height"]
        r["torques"] = torch.sum(torch.square(self.torques), dim=1) * rs["torque"]
        r["joint_acc"] = torch.sum(torch.square(self.last_hound_dof_vel - self.hound_dof_vel), dim=1) * rs["joint_acc"]
        knee_contact = torch.norm(cf[:, self.knee_indices, :], dim=2) > 1.0
        base_contact = torch.norm(cf[:, self.base_indices, :], dim=2) > 1.0
        r["collision"] = torch.sum(knee_contact, dim=1) * rs["collision"] + torch.sum(base_contact, dim=1) * \
            rs["collision"]
        stumble = (torch.norm(cf[:, self.feet_indices, :2], dim=2) > 5.0) * \
                  (torch.abs(cf[:, self.feet_indices, 2]) < 1.0)
        r["stumble"] = torch.sum(stumble, dim=1) * rs["stumble"]
        r["action_rate"] = torch.sum(torch.square(self.last_actions - self.actions), dim=1) * rs["action_rate"]
        contact = cf[:, self.feet_indices, 2] > 1.0
        first_contact = (self.feet_air_time > 0.0) * contact
        self.feet_air_time += self.dt
        air = torch.sum((self.feet_air_time - 0.5) * first_contact, dim=1) * rs["air_time"]
        air *= torch.norm(self.commands[:, :2], dim=1) > 0.1
        r["air_time"] = air
        self.feet_air_time *= ~contact
        r["hip"] = torch.sum(torch.abs(self.hound_dof_pos[:, [0, 3, 6, 9]] -
                                       self.hound_default_dof_pos[:, [0, 3, 6, 9]]), dim=1) * rs["hip"]
        self.rew_buf = r["lin_vel_xy"] + r["ang_vel_z"] + r["lin_vel_z"] + r["ang_vel_xy"] + r["orient"] + \
            r["base_height"] + r["torques"] + r["joint_acc"] + r["collision"] + r["action_rate"] + \
            r["air_time"] + r["hip"] + r["stumble"]
        self.rew_buf = torch.clip(self.rew_buf, min=0.0, max=None)
        self.rew_buf += rs["termination"] * self.reset_buf * ~self.timeout_buf
        for k in REWARD_TERMS:
            self.episode_sums[k] += r[k]

    def reset_idx(self, env_ids):
        """useful_hound.py:569-642."""
        k = len(env_ids)
        dev = self.device
        positions_offset = torch_rand_float(0.5, 1.5, (k, self.hound_num_dof), device=dev)
        velocities = torch_rand_float(-0.1, 0.1, (k, self.hound_num_dof), device=dev)
        self.hound_dof_pos[env_ids] = self.hound_default_dof_pos[env_ids] * positions_offset
        self.hound_dof_vel[env_ids] = velocities
        env_ids_int32 = env_ids.to(dtype=torch.int32)
        if self.custom_origins:
            self.update_terrain_level(env_ids)
            self.root_states[env_ids] = self.base_init_state
            self.root_states[env_ids, :3] += self.env_origins[env_ids]
            self.root_states[env_ids, :2] += torch_rand_float(-0.5, 0.5, (k, 2), device=dev)
        else:
            self.root_states[env_ids] = self.base_init_state
        reset_noise = torch.rand((k, 6), device=dev)
        pos = tensor_clamp(self.houndarm_default_dof_pos.unsqueeze(0) +
                           self.houndarm_dof_noise * 2.0 * (reset_noise - 0.5),
                           self.houndarm_dof_lower_limits.unsqueeze(0), self.houndarm_dof_upper_limits)
        self._q[env_ids, :] = pos
        self._qd[env_ids, :] = torch.zeros_like(self._qd[env_ids])
        self._pos_control[env_ids, :] = pos
        self._effort_control[env_ids, :] = torch.zeros_like(pos)
        self.commands[env_ids, 0] = torch_rand_float(self.command_x_range[0], self.command_x_range[1], (k, 1),
                                                     device=dev).squeeze()
        self.commands[env_ids, 1] = torch_rand_float(self.command_y_range[0], self.command_y_range[1], (k, 1),
                                                     device=dev).squeeze()
        self.commands[env_ids, 3] = torch_rand_float(self.command_yaw_range[0], self.command_yaw_range[1], (k, 1),
                                                     device=dev).squeeze()
        self.commands[env_ids] *= (torch.norm(self.commands[env_ids, :2], dim=1) > 0.25).unsqueeze(1)
        self._set_reset_state(env_ids_int32)
        self.last_actions[env_ids] = 0.0
        self.last_hound_dof_vel[env_ids] = 0.0
        self.feet_air_time[env_ids] = 0.0
        self.progress_buf[env_ids] = 0
        self.reset_buf[env_ids] = 1
        self.extras["episode"] = {}
        for key in self.episode_sums:
            self.extras["episode"]["rew_" + key] = torch.mean(self.episode_sums[key][env_ids]) / \
                self.max_episode_length_s
            self.episode_sums[key][env_ids] = 0.0
        self.extras["episode"]["terrain_level"] = torch.mean(self.terrain_levels.float())

    def _set_reset_state(self, env_ids_int32):
        """useful_hound.py:608-627: root and dof state, arm position targets and zero efforts of the reset envs."""
        n = len(env_ids_int32)
        self.gym.set_actor_root_state_tensor_indexed(self.sim, gymtorch.unwrap_tensor(self.root_states),
                                                     gymtorch.unwrap_tensor(env_ids_int32), n)
        self.gym.set_dof_state_tensor_indexed(self.sim, gymtorch.unwrap_tensor(self.dof_state),
                                              gymtorch.unwrap_tensor(env_ids_int32), n)
        total_pos = torch.cat([self.hound_dof_pos, self._pos_control], axis=1)
        total_effort = torch.zeros_like(total_pos)
        self.gym.set_dof_position_target_tensor_indexed(self.sim, gymtorch.unwrap_tensor(total_pos),
                                                        gymtorch.unwrap_tensor(env_ids_int32), n)
        self.gym.set_dof_actuation_force_tensor_indexed(self.sim, gymtorch.unwrap_tensor(total_effort),
                                                        gymtorch.unwrap_tensor(env_ids_int32), n)

    # ------------------------------------------------------------------ arm control
    def _compute_osc_torques(self, dpose):
        """Operational-space control of the arm (useful_hound.py:660-691)."""
        q, qd = self._q[:, :6], self._qd[:, :6]
        mm_inv = torch.inverse(self._mm)
        m_eef_inv = self._j_eef @ mm_inv @ torch.transpose(self._j_eef, 1, 2)
        m_eef = torch.inverse(m_eef_inv)
        u = torch.transpose(self._j_eef, 1, 2) @ m_eef @ (
            self.arm_kp * dpose - self.arm_kd * self._eef_state[:, 7:]).unsqueeze(-1)
        j_eef_inv = m_eef @ self._j_eef @ mm_inv
        u_null = self.arm_kd_null * -qd + self.arm_kp_null * (
            (self.houndarm_default_dof_pos[:6] - q + np.pi) % (2 * np.pi) - np.pi)
        u_null[:, 6:] *= 0
        u_null = self._mm @ u_null.unsqueeze(-1)
        u += (torch.eye(6, device=self.device).unsqueeze(0) - torch.transpose(self._j_eef, 1, 2) @ j_eef_inv) @ u_null
        return tensor_clamp(u.squeeze(-1), -self._houndarm_effort_limits[:6].unsqueeze(0),
                            self._houndarm_effort_limits[:6].unsqueeze(0))

    # ------------------------------------------------------------------ step
    def pre_physics_step(self, actions):
        self.actions = actions.clone().to(self.device)
        if self._control is not None:
            a = self.actions.contiguous()
            for _ in range(self.decimation):
                self._control(a, self._torque_buf)  # torques [N,18] and _arm_control, as the torch loop below
                self.gym.set_dof_actuation_force_tensor(self.sim, gymtorch.unwrap_tensor(self._torque_buf))
                self.torques = self._torque_buf
                self.gym.simulate(self.sim)
                self.gym.refresh_dof_state_tensor(self.sim)
            return
        for _ in range(self.decimation):
            u_arm = self.actions[:, 12:] * self.arm_cmd_limit / self.arm_action_scale
            u_arm = self._compute_osc_torques(dpose=u_arm)
            self._arm_control[:, :] = u_arm
            torques = torch.clip(self.Kp * (self.action_scale * self.actions[:, :12] + self.hound_default_dof_pos -
                                            self.hound_dof_pos) - self.Kd * self.hound_dof_vel, -80.0, 80.0)
            torques = torch.cat([torques, u_arm], axis=1)
            self.gym.set_dof_actuation_force_tensor(self.sim, gymtorch.unwrap_tensor(torques))
            self.torques = torques.view(self.torques.shape)
            self.gym.simulate(self.sim)
            if self.device == "cpu":
                self.gym.fetch_results(self.sim, True)
            self.gym.refresh_dof_state_tensor(self.sim)

    def post_physics_step(self):
        self.gym.refresh_actor_root_state_tensor(self.sim)
        self.gym.refresh_net_contact_force_tensor(self.sim)
        self.gym.refresh_jacobian_tensors(self.sim)
        self.gym.refresh_mass_matrix_tensors(self.sim)
        self.common_step_counter += 1
        push = self.common_step_counter % self.push_interval == 0
        if self._kernels is not None:
            # the fused tail (AnymalTerrain.post_physics_step's kernel path, UsefulHound extension)
            if push:
                self.push_robots()
            kern = self._kernels
            kern.post_a()
            snap = kern.rng_snapshot() if self.add_noise else None
            kern.observe()
            if kern.wait_reset_count() > 0:
                if snap is not None:
                    kern.rng_restore(snap)
                kern.reset_flagged(kern.last_reset_count, torch_rand_unit)
                kern.observe()
            return
        self.progress_buf += 1
        self.randomize_buf += 1
        if push:
            self.push_robots()
        self.base_quat = self.root_states[:, 3:7]
        self.base_lin_vel = quat_rotate_inverse(self.base_quat, self.root_states[:, 7:10])
        self.base_ang_vel = quat_rotate_inverse(self.base_quat, self.root_states[:, 10:13])
        self.projected_gravity = quat_rotate_inverse(self.base_quat, self.gravity_vec)
        forward = quat_apply(self.base_quat, self.forward_vec)
        heading = torch.atan2(forward[:, 1], forward[:, 0])
        self.commands[:, 2] = torch.clip(0.5 * wrap_to_pi(self.commands[:, 3] - heading), -1.0, 1.0)
        self.check_termination()
        self.compute_reward()
        env_ids = self.reset_buf.nonzero(as_tuple=False).flatten()
        if len(env_ids) > 0:
            self.reset_idx(env_ids)
        self.compute_observations()
        if self.add_noise:
            self.obs_buf += (2 * torch.rand_like(self.obs_buf) - 1) * self.noise_scale_vec
        self.last_actions[:] = self.actions[:]
        self.last_hound_dof_vel[:] = self.hound_dof_vel[:]
