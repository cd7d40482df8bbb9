"""AnymalTerrain: ANYmal-C velocity-tracking locomotion (reference ``tasks/anymal_terrain.py``).

The north-star task.  Behaviour (including the quirks listed in SURVEY.md
section 0.5) follows the reference line by line:

* ``pre_physics_step`` (anymal_terrain.py:441-451): ``decimation`` x
  [PD torque -> set efforts -> simulate -> refresh dof], and VecTask.step then
  simulates ``controlFrequencyInv`` more times with the last torques, so the sim
  advances 5 substeps per env step while ``self.dt`` is 4 substeps;
* ``post_physics_step`` (:453-501) refreshes root state and contacts only (the
  dof tensor keeps its post-decimation values), pushes every ``push_interval``
  steps, derives base-frame quantities, terminates, rewards, resets the
  terminated envs in the SAME step, then builds observations (+ noise);
* ``check_termination`` turns ``reset_buf`` into a bool tensor (:295);
* RNG call order is the reference's: friction buckets, terrain levels/types at
  env creation, then per reset: dof offsets, dof velocities, command x, y,
  heading; per step: push draw (every 750 steps) and the observation noise.

MI355X path (``sim_device=cuda:k``, GPU pipeline):
* ``fused_physics_step`` runs the whole decimation loop + the extra simulate +
  the root/contact refreshes as ONE kernel (libgymsim ``gs_sim_pd_step``);
* the post-physics tail runs as two fused kernels from libgymtask
  (``gt_anymal_post_physics_a`` before the reset, ``gt_anymal_post_physics_b``
  after it); ``reset_idx`` keeps its torch RNG draws (bit-exact resets with the
  reference's generator stream) and applies them with one kernel.
On the CPU pipeline the tail runs the torch statements below.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from isaacgym import gymapi, gymtorch, terrain_utils

from ..utils.torch_jit_utils import (get_axis_params, normalize, quat_apply, quat_rotate_inverse, to_torch,
                                     torch_rand_float)
from .base.vec_task import VecTask


def torch_rand_unit(shape, device):
    """The torch.rand draw inside torch_rand_float (torch_jit_utils.py); the fused reset applies
    torch_rand_float's affine map on the GPU, so the RNG stream advances identically."""
    return torch.rand(*shape, device=device)

REWARD_TERMS = ["lin_vel_xy", "lin_vel_z", "ang_vel_z", "ang_vel_xy", "orient", "torques", "joint_acc",
                "base_height", "air_time", "collision", "stumble", "action_rate", "hip"]


class AnymalTerrain(VecTask):
    supports_fused_physics = True

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
        self.named_default_joint_angles = env["defaultJointAngles"]

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

        super().__init__(config=cfg, rl_device=rl_device, sim_device=sim_device,
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
        self.dof_pos = self.dof_state.view(self.num_envs, self.num_dof, 2)[..., 0]
        self.dof_vel = self.dof_state.view(self.num_envs, self.num_dof, 2)[..., 1]
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
        self.last_dof_vel = torch.zeros_like(self.dof_vel)
        self.height_points = self.init_height_points()
        self.measured_heights = None
        self.default_dof_pos = torch.zeros_like(self.dof_pos, dtype=torch.float, device=dev, requires_grad=False)
        for i in range(self.num_actions):
            self.default_dof_pos[:, i] = self.named_default_joint_angles[self.dof_names[i]]
        self.episode_sums = {k: zeros(self.num_envs) for k in REWARD_TERMS}

        self._kernels = None
        self._heights_dev = None
        if self.custom_origins and self.device != "cpu":
            # trimesh: the fused tail measures the terrain under the probes in a kernel (gt_measure_heights)
            self._heights_dev = zeros(self.num_envs, self.num_height_points)
            self.height_points = self.height_points.contiguous()
        if self.device != "cpu":
            from ...gymtask import AnymalTailKernels  # fails loudly when libgymtask.so is missing
            self._kernels = AnymalTailKernels(self)
        self._fused_refreshed = False
        self.reset_idx(torch.arange(self.num_envs, device=self.device))
        self.init_done = True

    # ------------------------------------------------------------------ creation
    def create_sim(self):
        self.up_axis_idx = 2
        self.sim = super().create_sim(self.device_id, self.graphics_device_id, self.physics_engine, self.sim_params)
        terrain_type = self.cfg["env"]["terrain"]["terrainType"]
        if terrain_type == "plane":
            self._create_ground_plane()
        elif terrain_type == "trimesh":
            self._create_trimesh()
            self.custom_origins = True
        self._create_envs(self.num_envs, self.cfg["env"]["envSpacing"], int(np.sqrt(self.num_envs)))

    def _get_noise_scale_vec(self, cfg):
        learn = self.cfg["env"]["learn"]
        v = torch.zeros_like(self.obs_buf[0])
        self.add_noise = learn["addNoise"]
        lvl = learn["noiseLevel"]
        v[:3] = learn["linearVelocityNoise"] * lvl * self.lin_vel_scale
        v[3:6] = learn["angularVelocityNoise"] * lvl * self.ang_vel_scale
        v[6:9] = learn["gravityNoise"] * lvl
        v[9:12] = 0.0
        v[12:24] = learn["dofPositionNoise"] * lvl * self.dof_pos_scale
        v[24:36] = learn["dofVelocityNoise"] * lvl * self.dof_vel_scale
        v[36:176] = learn["heightMeasurementNoise"] * lvl * self.height_meas_scale
        v[176:188] = 0.0
        return v

    def _create_ground_plane(self):
        t = self.cfg["env"]["terrain"]
        plane = gymapi.PlaneParams()
        plane.normal = gymapi.Vec3(0.0, 0.0, 1.0)
        plane.static_friction = t["staticFriction"]
        plane.dynamic_friction = t["dynamicFriction"]
        plane.restitution = t["restitution"]
        self.gym.add_ground(self.sim, plane)

    def _create_trimesh(self):
        """anymal_terrain.py:196-209: the generated heightfield as a triangle mesh placed at
        (-border, -border, 0), and the raw int16 samples kept on the device for get_heights."""
        t = self.cfg["env"]["terrain"]
        self.terrain = Terrain(t, num_robots=self.num_envs)
        tm = gymapi.TriangleMeshParams()
        tm.nb_vertices = self.terrain.vertices.shape[0]
        tm.nb_triangles = self.terrain.triangles.shape[0]
        tm.transform.p.x = -self.terrain.border_size
        tm.transform.p.y = -self.terrain.border_size
        tm.transform.p.z = 0.0
        tm.static_friction = t["staticFriction"]
        tm.dynamic_friction = t["dynamicFriction"]
        tm.restitution = t["restitution"]
        self.gym.add_triangle_mesh(self.sim, self.terrain.vertices.flatten(order="C"),
                                   self.terrain.triangles.flatten(order="C"), tm)
        self.height_samples = torch.tensor(self.terrain.heightsamples).view(
            self.terrain.tot_rows, self.terrain.tot_cols).to(self.device)

    def _asset_location(self):
        here = os.path.dirname(os.path.abspath(__file__))
        asset_root = os.environ.get("ISAACGYMENVS_ASSET_ROOT", os.path.join(here, "../../assets"))
        path = os.path.join(asset_root, self.cfg["env"]["urdfAsset"]["file"])
        return os.path.dirname(path), os.path.basename(path)

    def _create_envs(self, num_envs, spacing, num_per_row):
        asset_root, asset_file = self._asset_location()
        opts = gymapi.AssetOptions()
        opts.default_dof_drive_mode = gymapi.DOF_MODE_EFFORT
        opts.collapse_fixed_joints = True
        opts.replace_cylinder_with_capsule = True
        opts.flip_visual_attachments = True
        opts.fix_base_link = self.cfg["env"]["urdfAsset"]["fixBaseLink"]
        opts.density = 0.001
        opts.angular_damping = 0.0
        opts.linear_damping = 0.0
        opts.armature = 0.0
        opts.thickness = 0.01
        opts.disable_gravity = False
        asset = self.gym.load_asset(self.sim, asset_root, asset_file, opts)
        self.num_dof = self.gym.get_asset_dof_count(asset)
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
        foot = self.cfg["env"]["urdfAsset"]["footName"]
        knee = self.cfg["env"]["urdfAsset"]["kneeName"]
        feet_names = [s for s in body_names if foot in s]
        knee_names = [s for s in body_names if knee in s]
        self.feet_indices = torch.zeros(len(feet_names), dtype=torch.long, device=self.device, requires_grad=False)
        self.knee_indices = torch.zeros(len(knee_names), dtype=torch.long, device=self.device, requires_grad=False)
        self.base_index = 0
        dof_props = self.gym.get_asset_dof_properties(asset)

        tcfg = self.cfg["env"]["terrain"]
        self.env_origins = torch.zeros(self.num_envs, 3, device=self.device, requires_grad=False)
        if not self.curriculum:
            tcfg["maxInitMapLevel"] = tcfg["numLevels"] - 1
        self.terrain_levels = torch.randint(0, tcfg["maxInitMapLevel"] + 1, (self.num_envs,), device=self.device)
        self.terrain_types = torch.randint(0, tcfg["numTerrains"], (self.num_envs,), device=self.device)
        if self.custom_origins:
            self.terrain_origins = torch.from_numpy(self.terrain.env_origins).to(self.device).to(torch.float)
            spacing = 0.0

        lower = gymapi.Vec3(-spacing, -spacing, 0.0)
        upper = gymapi.Vec3(spacing, spacing, spacing)
        self.anymal_handles = []
        self.envs = []
        # one device->host copy instead of one blocking read per shape per env (same values)
        friction_host = friction_buckets.cpu().numpy()[:, 0]
        for i in range(self.num_envs):
            env_handle = self.gym.create_env(self.sim, lower, upper, num_per_row)
            if self.custom_origins:
                # spawn on the env's terrain tile, +-1 m (anymal_terrain.py:271-275)
                self.env_origins[i] = self.terrain_origins[self.terrain_levels[i], self.terrain_types[i]]
                pos = self.env_origins[i].clone()
                pos[:2] += torch_rand_float(-1.0, 1.0, (2, 1), device=self.device).squeeze(1)
                start_pose.p = gymapi.Vec3(*pos.tolist())
            for sp in shape_props:
                sp.friction = friction_host[i % num_buckets]
            self.gym.set_asset_rigid_shape_properties(asset, shape_props)
            handle = self.gym.create_actor(env_handle, asset, start_pose, "anymal", i, 0, 0)
            self.gym.set_actor_dof_properties(env_handle, handle, dof_props)
            self.envs.append(env_handle)
            self.anymal_handles.append(handle)
        for i, n in enumerate(feet_names):
            self.feet_indices[i] = self.gym.find_actor_rigid_body_handle(self.envs[0], self.anymal_handles[0], n)
        for i, n in enumerate(knee_names):
            self.knee_indices[i] = self.gym.find_actor_rigid_body_handle(self.envs[0], self.anymal_handles[0], n)
        self.base_index = self.gym.find_actor_rigid_body_handle(self.envs[0], self.anymal_handles[0], "base")

    # ------------------------------------------------------------------ terms
    def check_termination(self):
        self.reset_buf = torch.norm(self.contact_forces[:, self.base_index, :], dim=1) > 1.0
        if not self.allow_knee_contacts:
            knee_contact = torch.norm(self.contact_forces[:, self.knee_indices, :], dim=2) > 1.0
            self.reset_buf |= torch.any(knee_contact, dim=1)
        self.reset_buf = torch.where(self.progress_buf >= self.max_episode_length - 1,
                                     torch.ones_like(self.reset_buf), self.reset_buf)

    def compute_observations(self):
        self.measured_heights = self.get_heights()
        heights = torch.clip(self.root_states[:, 2].unsqueeze(1) - 0.5 - self.measured_heights, -1, 1.0) \
            * self.height_meas_scale
        self.obs_buf = torch.cat((self.base_lin_vel * self.lin_vel_scale,
                                  self.base_ang_vel * self.ang_vel_scale,
                                  self.projected_gravity,
                                  self.commands[:, :3] * self.commands_scale,
                                  self.dof_pos * self.dof_pos_scale,
                                  self.dof_vel * self.dof_vel_scale,
                                  heights,
                                  self.actions), dim=-1)

    def compute_reward(self):
        rs = self.rew_scales
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
        r["joint_acc"] = torch.sum(torch.square(self.last_dof_vel - self.dof_vel), dim=1) * rs["joint_acc"]
        knee_contact = torch.norm(self.contact_forces[:, self.knee_indices, :], dim=2) > 1.0
        r["collision"] = torch.sum(knee_contact, dim=1) * rs["collision"]
        stumble = (torch.norm(self.contact_forces[:, self.feet_indices, :2], dim=2) > 5.0) * \
                  (torch.abs(self.contact_forces[:, self.feet_indices, 2]) < 1.0)
        r["stumble"] = torch.sum(stumble, dim=1) * rs["stumble"]
        r["action_rate"] = torch.sum(torch.square(self.last_actions - self.actions), dim=1) * rs["action_rate"]
        contact = self.contact_forces[:, self.feet_indices, 2] > 1.0
        first_contact = (self.feet_air_time > 0.0) * contact
        self.feet_air_time += self.dt
        air = torch.sum((self.feet_air_time - 0.5) * first_contact, dim=1) * rs["air_time"]
        air *= torch.norm(self.commands[:, :2], dim=1) > 0.1
        r["air_time"] = air
        self.feet_air_time *= ~contact
        r["hip"] = torch.sum(torch.abs(self.dof_pos[:, [0, 3, 6, 9]] - self.default_dof_pos[:, [0, 3, 6, 9]]),
                             dim=1) * rs["hip"]
        # same summation order as the reference (anymal_terrain.py:362-363)
        self.rew_buf = r["lin_vel_xy"] + r["ang_vel_z"] + r["lin_vel_z"] + r["ang_vel_xy"] + r["orient"] + \
            r["base_height"] + r["torques"] + r["joint_acc"] + r["collision"] + r["action_rate"] + \
            r["air_time"] + r["hip"] + r["stumble"]
        self.rew_buf = torch.clip(self.rew_buf, min=0.0, max=None)
        self.rew_buf += rs["termination"] * self.reset_buf * ~self.timeout_buf
        for k in REWARD_TERMS:
            self.episode_sums[k] += r[k]

    def reset_idx(self, env_ids):
        k = len(env_ids)
        positions_offset = torch_rand_float(0.5, 1.5, (k, self.num_dof), device=self.device)
        velocities = torch_rand_float(-0.1, 0.1, (k, self.num_dof), device=self.device)
        root_xy = None
        if self.custom_origins:
            self.update_terrain_level(env_ids)
            root_xy = torch_rand_float(-0.5, 0.5, (k, 2), device=self.device)
        cmd_x = torch_rand_float(self.command_x_range[0], self.command_x_range[1], (k, 1), device=self.device).squeeze()
        cmd_y = torch_rand_float(self.command_y_range[0], self.command_y_range[1], (k, 1), device=self.device).squeeze()
        cmd_h = torch_rand_float(self.command_yaw_range[0], self.command_yaw_range[1], (k, 1),
                                 device=self.device).squeeze()
        env_ids_int32 = env_ids.to(dtype=torch.int32)
        if self._kernels is not None and not self.custom_origins:
            # one kernel applies the draws; it also fills extras["episode"] (episode sums over env_ids)
            self._kernels.reset(env_ids_int32, positions_offset, velocities, cmd_x, cmd_y, cmd_h)
            self._set_reset_state(env_ids_int32)
            return
        self.dof_pos[env_ids] = self.default_dof_pos[env_ids] * positions_offset
        self.dof_vel[env_ids] = velocities
        self.root_states[env_ids] = self.base_init_state
        if self.custom_origins:
            self.root_states[env_ids, :3] += self.env_origins[env_ids]
            self.root_states[env_ids, :2] += root_xy
        self._set_reset_state(env_ids_int32)
        self.commands[env_ids, 0] = cmd_x
        self.commands[env_ids, 1] = cmd_y
        self.commands[env_ids, 3] = cmd_h
        self.commands[env_ids] *= (torch.norm(self.commands[env_ids, :2], dim=1) > 0.25).unsqueeze(1)
        self.last_actions[env_ids] = 0.0
        self.last_dof_vel[env_ids] = 0.0
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
        # set_actor_root_state_tensor_indexed + set_dof_state_tensor_indexed (anymal_terrain.py:401-408), one call
        self.gym.amd_set_root_and_dof_state_indexed(self.sim, gymtorch.unwrap_tensor(self.root_states),
                                                    gymtorch.unwrap_tensor(self.dof_state),
                                                    gymtorch.unwrap_tensor(env_ids_int32), len(env_ids_int32))

    def update_terrain_level(self, env_ids):
        """anymal_terrain.py:427-435: an env that walked less than a quarter of its commanded
        distance moves a level down, one that left its tile moves up (levels wrap modulo numLevels)."""
        if not self.init_done or not self.curriculum:
            return
        distance = torch.norm(self.root_states[env_ids, :2] - self.env_origins[env_ids, :2], dim=1)
        self.terrain_levels[env_ids] -= 1 * (distance < torch.norm(self.commands[env_ids, :2]) *
                                             self.max_episode_length_s * 0.25)
        self.terrain_levels[env_ids] += 1 * (distance > self.terrain.env_length / 2)
        self.terrain_levels[env_ids] = torch.clip(self.terrain_levels[env_ids], 0) % self.terrain.env_rows
        self.env_origins[env_ids] = self.terrain_origins[self.terrain_levels[env_ids], self.terrain_types[env_ids]]

    def push_robots(self):
        self.root_states[:, 7:9] = torch_rand_float(-1.0, 1.0, (self.num_envs, 2), device=self.device)
        self.gym.set_actor_root_state_tensor(self.sim, gymtorch.unwrap_tensor(self.root_states))

    # ------------------------------------------------------------------ step
    def pre_physics_step(self, actions):
        self.actions = actions.clone().to(self.device)
        for _ in range(self.decimation):
            torques = torch.clip(self.Kp * (self.action_scale * self.actions + self.default_dof_pos - self.dof_pos)
                                 - self.Kd * self.dof_vel, -80.0, 80.0)
            self.gym.set_dof_actuation_force_tensor(self.sim, gymtorch.unwrap_tensor(torques))
            self.torques = torques.view(self.torques.shape)
            self.gym.simulate(self.sim)
            if self.device == "cpu":
                self.gym.fetch_results(self.sim, True)
            self.gym.refresh_dof_state_tensor(self.sim)

    def fused_physics_step(self, actions):
        """pre_physics_step + VecTask's simulate loop + post_physics_step's refreshes, one kernel."""
        # (get_device(): an int compare, cheaper per step than comparing torch.device objects)
        if (actions.get_device() == self.torques.get_device() and actions.dtype == torch.float32
                and actions.is_contiguous()):
            # self.actions = actions.clone() (anymal_terrain.py:442), written by the physics kernel into a fresh
            # tensor; the next step's is allocated right after this launch, off the host path before it
            nxt = self._next_actions
            if nxt is None or nxt.shape != actions.shape:
                nxt = torch.empty_like(actions)
            self.actions = nxt
            # post_physics_step's part A (gymtask post_a) in the same launch, except on a push step (the push
            # changes root_states before post_a reads them, anymal_terrain.py:458-460)
            tail = None
            kern = self._kernels
            if kern is not None and (self.common_step_counter + 1) % self.push_interval != 0:
                tail = kern.tail_for_launch()
            self.gym.amd_pd_decimation_step(self.sim, actions, self._default_pos_row(), float(self.Kp),
                                            float(self.Kd), float(self.action_scale), 80.0, self.decimation,
                                            self.control_freq_inv, self.torques, actions_copy_out=nxt, tail=tail)
            self._tail_fused = tail is not None
            self.fused_tail_steps += int(tail is not None)
            self._next_actions = torch.empty_like(actions)
        else:
            self.actions = actions.clone().to(self.device)
            self.gym.amd_pd_decimation_step(self.sim, self.actions, self._default_pos_row(), float(self.Kp),
                                            float(self.Kd), float(self.action_scale), 80.0, self.decimation,
                                            self.control_freq_inv, self.torques)
            self._tail_fused = False
        self._fused_refreshed = True

    _next_actions = None
    _tail_fused = False
    _obs_mirrored = None  # the observation tensor whose values the registered mirror holds (amd_set_obs_mirror)

    def amd_set_obs_mirror(self, buf) -> bool:
        """Register a static buffer that the fused tail also writes every step's observations into (a learner's
        captured act-forward input, so it skips its per-step copy); False where the tail kernels do not run."""
        if self._kernels is None:
            return False
        self._kernels.set_obs_mirror(buf)
        return True
    fused_tail_steps = 0  # steps whose post_a ran inside the physics launch (a counter for tests / probes)

    def _default_pos_row(self):
        if getattr(self, "_default_row", None) is None:
            self._default_row = self.default_dof_pos[0].contiguous()
        return self._default_row

    def post_physics_step(self):
        if not self._fused_refreshed:
            self.gym.refresh_actor_root_state_tensor(self.sim)
            self.gym.refresh_net_contact_force_tensor(self.sim)
        self._fused_refreshed = False
        self.common_step_counter += 1
        push = self.common_step_counter % self.push_interval == 0
        if self._kernels is not None:
            if push:
                self.push_robots()
            kern = self._kernels
            # Optimistic: most steps reset nobody, so draw the noise and build the observations before
            # the host knows the count.  On a reset step, roll the RNG back and redo both after
            # reset_idx: the draws, their order and the results are the reference's either way.
            if self._tail_fused:  # post_a ran in the physics launch (fused_physics_step)
                kern.after_fused_tail()
                snap = kern.rng_snapshot() if self.add_noise else None
                kern.observe()
            elif kern.post_ab_applies():  # post_a + the observations in one launch (gymtask ABI 5)
                snap = kern.rng_snapshot() if self.add_noise else None
                kern.post_ab()
            else:
                kern.post_a()  # counters, base quantities, heading command, termination, reward
                snap = kern.rng_snapshot() if self.add_noise else None
                kern.observe()
            self._tail_fused = False
            if kern.reset_observe_applies():
                # the count, and on a reset step the whole reset + observation sequence, in one C call
                if kern.wait_reset_observe(snap) > 0:
                    kern.finish_reset()
                return
            if kern.wait_reset_count() > 0:
                k = kern.last_reset_count
                if snap is not None:
                    kern.rng_restore(snap)
                kern.reset_flagged(k, torch_rand_unit, defer_extras=True)  # reset_idx without nonzero / host sync
                kern.observe()
                kern.finish_reset()  # extras["episode"], built while the GPU runs the observation kernel
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
        self.last_dof_vel[:] = self.dof_vel[:]

    # ------------------------------------------------------------------ heights
    def init_height_points(self):
        y = 0.1 * torch.tensor([-5, -4, -3, -2, -1, 1, 2, 3, 4, 5], device=self.device, requires_grad=False)
        x = 0.1 * torch.tensor([-8, -7, -6, -5, -4, -3, -2, 2, 3, 4, 5, 6, 7, 8], device=self.device,
                               requires_grad=False)
        grid_x, grid_y = torch.meshgrid(x, y, indexing="ij")
        self.num_height_points = grid_x.numel()
        points = torch.zeros(self.num_envs, self.num_height_points, 3, device=self.device, requires_grad=False)
        points[:, :, 0] = grid_x.flatten()
        points[:, :, 1] = grid_y.flatten()
        return points

    def get_heights(self, env_ids=None):
        ttype = self.cfg["env"]["terrain"]["terrainType"]
        if ttype == "plane":
            return torch.zeros(self.num_envs, self.num_height_points, device=self.device, requires_grad=False)
        if ttype == "none":
            raise NameError("Can't measure height with terrain type 'none'")
        return sample_heights(self.height_samples, self.base_quat, self.root_states, self.height_points,
                              self.terrain.border_size, self.terrain.horizontal_scale,
                              self.terrain.vertical_scale, env_ids)


def sample_heights(height_samples, base_quat, root_states, height_points, border: float, hs: float, vs: float,
                   env_ids=None):
    """get_heights (anymal_terrain.py:515-538): the 14x10 probe grid turned by the base yaw and
    placed at the base, truncated to heightfield cells (clipped to the second-last row/column),
    the lower of the samples at (px, py) and (px+1, py+1), in metres."""
    nh = height_points.shape[1]
    if env_ids:
        pts = quat_apply_yaw(base_quat[env_ids].repeat(1, nh), height_points[env_ids]) + \
            root_states[env_ids, :3].unsqueeze(1)
    else:
        pts = quat_apply_yaw(base_quat.repeat(1, nh), height_points) + root_states[:, :3].unsqueeze(1)
    pts += border
    pts = (pts / hs).long()
    px = torch.clip(pts[:, :, 0].view(-1), 0, height_samples.shape[0] - 2)
    py = torch.clip(pts[:, :, 1].view(-1), 0, height_samples.shape[1] - 2)
    h = torch.min(height_samples[px, py], height_samples[px + 1, py + 1])
    return h.view(pts.shape[0], -1) * vs


class Terrain:
    """The terrain map of anymal_terrain.py:543-673: numLevels x numTerrains tiles of
    mapLength x mapWidth metres inside a 20 m border, int16 heights (0.005 m units, 0.1 m cells),
    converted to a triangle mesh with vertical walls above slopeTreshold.  Curriculum maps vary
    difficulty along the level axis and terrain kind along the type axis (terrainProportions);
    env origins sit at each tile's centre on top of its highest point within +-1 m."""

    horizontal_scale = 0.1
    vertical_scale = 0.005
    border_size = 20

    def __init__(self, cfg, num_robots):
        self.type = cfg["terrainType"]
        if self.type in ("none", "plane"):
            return
        self.env_length = cfg["mapLength"]
        self.env_width = cfg["mapWidth"]
        props = cfg["terrainProportions"]
        self.proportions = [np.sum(props[:i + 1]) for i in range(len(props))]
        self.env_rows = cfg["numLevels"]
        self.env_cols = cfg["numTerrains"]
        self.num_maps = self.env_rows * self.env_cols
        self.num_per_env = int(num_robots / self.num_maps)
        self.env_origins = np.zeros((self.env_rows, self.env_cols, 3))
        self.width_per_env_pixels = int(self.env_width / self.horizontal_scale)
        self.length_per_env_pixels = int(self.env_length / self.horizontal_scale)
        self.border = int(self.border_size / self.horizontal_scale)
        self.tot_cols = int(self.env_cols * self.width_per_env_pixels) + 2 * self.border
        self.tot_rows = int(self.env_rows * self.length_per_env_pixels) + 2 * self.border
        self.height_field_raw = np.zeros((self.tot_rows, self.tot_cols), dtype=np.int16)
        if cfg["curriculum"]:
            self.curiculum(num_robots, num_terrains=self.env_cols, num_levels=self.env_rows)
        else:
            self.randomized_terrain()
        self.heightsamples = self.height_field_raw
        self.vertices, self.triangles = terrain_utils.convert_heightfield_to_trimesh(
            self.height_field_raw, self.horizontal_scale, self.vertical_scale, cfg["slopeTreshold"])

    def _tile(self):
        return terrain_utils.SubTerrain("terrain", width=self.width_per_env_pixels, length=self.width_per_env_pixels,
                                        vertical_scale=self.vertical_scale, horizontal_scale=self.horizontal_scale)

    def _place(self, i, j, tile):
        x0 = self.border + i * self.length_per_env_pixels
        y0 = self.border + j * self.width_per_env_pixels
        self.height_field_raw[x0:x0 + self.length_per_env_pixels, y0:y0 + self.width_per_env_pixels] = \
            tile.height_field_raw
        x1 = int((self.env_length / 2.0 - 1) / self.horizontal_scale)
        x2 = int((self.env_length / 2.0 + 1) / self.horizontal_scale)
        y1 = int((self.env_width / 2.0 - 1) / self.horizontal_scale)
        y2 = int((self.env_width / 2.0 + 1) / self.horizontal_scale)
        top = np.max(tile.height_field_raw[x1:x2, y1:y2]) * self.vertical_scale
        self.env_origins[i, j] = [(i + 0.5) * self.env_length, (j + 0.5) * self.env_width, top]

    def randomized_terrain(self):
        tu = terrain_utils
        for k in range(self.num_maps):
            i, j = np.unravel_index(k, (self.env_rows, self.env_cols))
            tile = self._tile()
            choice = np.random.uniform(0, 1)
            if choice < 0.1:
                if np.random.choice([0, 1]):
                    tu.pyramid_sloped_terrain(tile, np.random.choice([-0.3, -0.2, 0, 0.2, 0.3]))
                    tu.random_uniform_terrain(tile, min_height=-0.1, max_height=0.1, step=0.05,
                                              downsampled_scale=0.2)
                else:
                    tu.pyramid_sloped_terrain(tile, np.random.choice([-0.3, -0.2, 0, 0.2, 0.3]))
            elif choice < 0.6:
                tu.pyramid_stairs_terrain(tile, step_width=0.31, step_height=np.random.choice([-0.15, 0.15]),
                                          platform_size=3.0)
            else:
                tu.discrete_obstacles_terrain(tile, 0.15, 1.0, 2.0, 40, platform_size=3.0)
            self._place(i, j, tile)

    def curiculum(self, num_robots, num_terrains, num_levels):
        tu = terrain_utils
        p = self.proportions
        for j in range(num_terrains):
            for i in range(num_levels):
                tile = self._tile()
                difficulty = i / num_levels
                choice = j / num_terrains
                slope = difficulty * 0.4
                step_height = 0.05 + 0.175 * difficulty
                obstacle_height = 0.025 + difficulty * 0.15
                stone_size = 2 - 1.8 * difficulty
                if choice < p[0]:
                    if choice < 0.05:
                        slope *= -1
                    tu.pyramid_sloped_terrain(tile, slope=slope, platform_size=3.0)
                elif choice < p[1]:
                    if choice < 0.15:
                        slope *= -1
                    tu.pyramid_sloped_terrain(tile, slope=slope, platform_size=3.0)
                    tu.random_uniform_terrain(tile, min_height=-0.1, max_height=0.1, step=0.025,
                                              downsampled_scale=0.2)
                elif choice < p[3]:
                    if choice < p[2]:
                        step_height *= -1
                    tu.pyramid_stairs_terrain(tile, step_width=0.31, step_height=step_height, platform_size=3.0)
                elif choice < p[4]:
                    tu.discrete_obstacles_terrain(tile, obstacle_height, 1.0, 2.0, 40, platform_size=3.0)
                else:
                    tu.stepping_stones_terrain(tile, stone_size=stone_size, stone_distance=0.1, max_height=0.0,
                                               platform_size=3.0)
                self._place(i, j, tile)


def quat_apply_yaw(quat, vec):
    q = quat.clone().view(-1, 4)
    q[:, :2] = 0.0
    q = normalize(q)
    return quat_apply(q, vec)


def wrap_to_pi(angles):
    """anymal_terrain.py:684-687.  The reference function is TorchScript, where ``angles %= 2*pi``
    lowers to C fmod (result has the sign of the dividend), so negative angles are left in
    (-2pi, 0] and only angles > pi are shifted.  Reproduced as is (tests/test_golden_tasks.py)."""
    angles = torch.fmod(angles, 2 * np.pi)
    angles -= 2 * np.pi * (angles > np.pi)
    return angles
