"""Ant locomotion (reference ``tasks/ant.py``), SURVEY.md section 8 row A13.

The behaviour is the reference's, step for step (checked against fixtures recorded from the
reference's own code in tests/golden/ant.npz):

* actions are torques: ``a * gear * powerScale`` with the gears the MJCF motors declare
  (ant.py:158-161, 281-285), written with ``set_dof_actuation_force_tensor``;
* one ``simulate`` per control step (dt 1/60, 2 substeps; Ant.yaml sim block), joint limits
  enforced by the solver, four force sensors on the feet (ant.py:174-178);
* ``post_physics_step`` resets the envs flagged in the previous step, then rebuilds the
  60-wide observation and the reward (ant.py:287-297);
* reset draws: dof offsets U(-0.2, 0.2) then dof velocities U(-0.1, 0.1), in that order,
  positions clamped into the limits (ant.py:252-279); the reset buffer is int64.

On the GPU pipeline the post-reset tail (observations, reward, done mask, true objective) is one HIP
kernel (libgymtask gt_ant_post_physics) that also publishes the done count to pinned host memory, so
the next step looks for envs to reset only when there are some; the torch statements below stay the
CPU-pipeline path and the golden-tested specification.

Observation layout (ant.py:400-404): torso height, local linear velocity (3), local angular
velocity (3), yaw, roll, angle to target, up projection, heading projection, scaled dof
positions (8), dof velocities * dofVelocityScale (8), force-sensor wrenches * contactForceScale
(24), actions (8).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from isaacgym import gymapi, gymtorch

from ..utils.torch_jit_utils import (compute_heading_and_up, compute_rot, get_axis_params, quat_conjugate,
                                     tensor_clamp, to_torch, torch_rand_float, unscale)
from .base.vec_task import VecTask

ANT_OBS, ANT_ACTIONS, ANT_SENSORS = 60, 8, 4

# column ranges inside the observation (ant.py:400-404)
OBS_HEIGHT, OBS_UP, OBS_HEADING = 0, 10, 11
OBS_DOF_POS = slice(12, 20)
OBS_DOF_VEL = slice(20, 28)
OBS_SENSORS = slice(28, 52)
OBS_ACTIONS = slice(52, 60)


class Ant(VecTask):
    def __init__(self, cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture,
                 force_render):
        self.cfg = cfg
        env = self.cfg["env"]
        self.max_episode_length = env["episodeLength"]
        self.randomization_params = self.cfg["task"]["randomization_params"]
        self.randomize = self.cfg["task"]["randomize"]
        if self.randomize:
            raise NotImplementedError("Ant domain randomisation (task.randomize) is outside the hot-path scope")
        self.dof_vel_scale = env["dofVelocityScale"]
        self.contact_force_scale = env["contactForceScale"]
        self.power_scale = env["powerScale"]
        self.heading_weight = env["headingWeight"]
        self.up_weight = env["upWeight"]
        self.actions_cost_scale = env["actionsCost"]
        self.energy_cost_scale = env["energyCost"]
        self.joints_at_limit_cost_scale = env["jointsAtLimitCost"]
        self.death_cost = env["deathCost"]
        self.termination_height = env["terminationHeight"]
        self.debug_viz = env["enableDebugVis"]
        self.plane_static_friction = env["plane"]["staticFriction"]
        self.plane_dynamic_friction = env["plane"]["dynamicFriction"]
        self.plane_restitution = env["plane"]["restitution"]
        env["numObservations"] = ANT_OBS
        env["numActions"] = ANT_ACTIONS
        super().__init__(config=self.cfg, rl_device=rl_device, sim_device=sim_device,
                         graphics_device_id=graphics_device_id, headless=headless,
                         virtual_screen_capture=virtual_screen_capture, force_render=force_render)
        dev, n = self.device, self.num_envs

        root_t = self.gym.acquire_actor_root_state_tensor(self.sim)
        dof_t = self.gym.acquire_dof_state_tensor(self.sim)
        sensor_t = self.gym.acquire_force_sensor_tensor(self.sim)
        self.vec_sensor_tensor = gymtorch.wrap_tensor(sensor_t).view(n, ANT_SENSORS * 6)
        self.gym.refresh_dof_state_tensor(self.sim)
        self.gym.refresh_actor_root_state_tensor(self.sim)

        self.root_states = gymtorch.wrap_tensor(root_t)
        self.initial_root_states = self.root_states.clone()
        self.initial_root_states[:, 7:13] = 0.0
        self.dof_state = gymtorch.wrap_tensor(dof_t)
        per_dof = self.dof_state.view(n, self.num_dof, 2)
        self.dof_pos, self.dof_vel = per_dof[..., 0], per_dof[..., 1]
        # the start pose is 0 unless 0 lies outside a joint's range (ant.py:96-99)
        lo, hi = self.dof_limits_lower, self.dof_limits_upper
        start = torch.where(lo > 0.0, lo, torch.where(hi < 0.0, hi, torch.zeros_like(lo)))
        self.initial_dof_pos = start.expand(n, -1).clone()
        self.initial_dof_vel = torch.zeros_like(self.dof_vel)

        self.up_vec = to_torch(get_axis_params(1.0, self.up_axis_idx), device=dev).repeat((n, 1))
        self.heading_vec = to_torch([1, 0, 0], device=dev).repeat((n, 1))
        self.inv_start_rot = quat_conjugate(self.start_rotation).repeat((n, 1))
        self.basis_vec0 = self.heading_vec.clone()
        self.basis_vec1 = self.up_vec.clone()
        self.targets = to_torch([1000, 0, 0], device=dev).repeat((n, 1))
        self.target_dirs = to_torch([1, 0, 0], device=dev).repeat((n, 1))
        self.dt = self.cfg["sim"]["dt"]
        self.potentials = to_torch([-1000.0 / self.dt], device=dev).repeat(n)
        self.prev_potentials = self.potentials.clone()
        self._tail = None
        if self.device != "cpu":
            # GPU pipeline: observations + reward + done mask are one kernel (gt_ant_post_physics)
            from ...gymtask import AntTailKernel  # fails loudly when libgymtask.so is missing
            self._tail = AntTailKernel(self)

    # ------------------------------------------------------------------ scene
    def create_sim(self):
        self.up_axis_idx = 2
        self.sim = super().create_sim(self.device_id, self.graphics_device_id, self.physics_engine, self.sim_params)
        plane = gymapi.PlaneParams()
        plane.normal = gymapi.Vec3(0.0, 0.0, 1.0)
        plane.static_friction = self.plane_static_friction
        plane.dynamic_friction = self.plane_dynamic_friction
        self.gym.add_ground(self.sim, plane)
        spacing = self.cfg["env"]["envSpacing"]
        self._create_envs(self.num_envs, spacing, int(np.sqrt(self.num_envs)))

    def _create_envs(self, num_envs, spacing, num_per_row):
        here = os.path.dirname(os.path.abspath(__file__))
        asset_root = os.environ.get("ISAACGYMENVS_ASSET_ROOT", os.path.join(here, "../../assets"))
        asset_file = self.cfg["env"].get("asset", {}).get("assetFileName", "mjcf/nv_ant.xml")
        path = os.path.join(asset_root, asset_file)
        opts = gymapi.AssetOptions()
        opts.default_dof_drive_mode = gymapi.DOF_MODE_NONE  # drives come from the MJCF (ant.py:150-152)
        opts.angular_damping = 0.0
        asset = self.gym.load_asset(self.sim, os.path.dirname(path), os.path.basename(path), opts)
        self.num_dof = self.gym.get_asset_dof_count(asset)
        self.num_bodies = self.gym.get_asset_rigid_body_count(asset)
        gears = [p.motor_effort for p in self.gym.get_asset_actuator_properties(asset)]
        self.joint_gears = to_torch(gears, device=self.device)

        start_pose = gymapi.Transform()
        start_pose.p = gymapi.Vec3(*get_axis_params(0.44, self.up_axis_idx))
        r = start_pose.r
        self.start_rotation = torch.tensor([r.x, r.y, r.z, r.w], device=self.device)
        self.torso_index = 0

        body_names = [self.gym.get_asset_rigid_body_name(asset, i) for i in range(self.num_bodies)]
        feet = [name for name in body_names if "foot" in name]
        for name in feet:
            self.gym.create_asset_force_sensor(asset, self.gym.find_asset_rigid_body_index(asset, name),
                                               gymapi.Transform())

        lower, upper = gymapi.Vec3(-spacing, -spacing, 0.0), gymapi.Vec3(spacing, spacing, spacing)
        self.envs, self.ant_handles = [], []
        for i in range(num_envs):
            env_ptr = self.gym.create_env(self.sim, lower, upper, num_per_row)
            handle = self.gym.create_actor(env_ptr, asset, start_pose, "ant", i, 1, 0)
            self.envs.append(env_ptr)
            self.ant_handles.append(handle)

        # limits of the last actor, each pair ordered (ant.py:199-209)
        props = self.gym.get_actor_dof_properties(self.envs[-1], self.ant_handles[-1])
        a, b = np.asarray(props["lower"], np.float64), np.asarray(props["upper"], np.float64)
        self.dof_limits_lower = to_torch(np.minimum(a, b).tolist(), device=self.device)
        self.dof_limits_upper = to_torch(np.maximum(a, b).tolist(), device=self.device)
        self.extremities_index = torch.tensor(
            [self.gym.find_actor_rigid_body_handle(self.envs[0], self.ant_handles[0], name) for name in feet],
            dtype=torch.long, device=self.device)

    # ------------------------------------------------------------------ step
    def pre_physics_step(self, actions):
        self.actions = actions.clone().to(self.device)
        forces = self.actions * self.joint_gears * self.power_scale
        self.gym.set_dof_actuation_force_tensor(self.sim, gymtorch.unwrap_tensor(forces))

    def post_physics_step(self):
        self.progress_buf += 1
        self.randomize_buf += 1
        if self._tail is not None:
            # the previous step's kernel published how many envs it flagged: look for them only then
            k = self._tail.done_count()
            if k is None:  # before the first launch: no ballots yet
                env_ids = self.reset_buf.nonzero(as_tuple=False).flatten()
                if len(env_ids) > 0:
                    self.reset_idx(env_ids)
            elif k > 0:  # reset_idx fused (gt_ant_reset_flagged): no nonzero() host sync
                self._tail.reset_flagged(k)
            self.gym.refresh_dof_state_tensor(self.sim)
            self.gym.refresh_actor_root_state_tensor(self.sim)
            self.gym.refresh_force_sensor_tensor(self.sim)
            self._tail()  # compute_observations + compute_reward + compute_true_objective
            self.extras["true_objective"] = self._tail.true_objective
            return
        env_ids = self.reset_buf.nonzero(as_tuple=False).flatten()
        if len(env_ids) > 0:
            self.reset_idx(env_ids)
        self.compute_observations()
        self.compute_reward(self.actions)
        self.compute_true_objective()

    def reset_idx(self, env_ids):
        k = len(env_ids)
        offsets = torch_rand_float(-0.2, 0.2, (k, self.num_dof), device=self.device)
        velocities = torch_rand_float(-0.1, 0.1, (k, self.num_dof), device=self.device)
        self.dof_pos[env_ids] = tensor_clamp(self.initial_dof_pos[env_ids] + offsets, self.dof_limits_lower,
                                             self.dof_limits_upper)
        self.dof_vel[env_ids] = velocities
        ids32 = env_ids.to(dtype=torch.int32)
        self.gym.set_actor_root_state_tensor_indexed(self.sim, gymtorch.unwrap_tensor(self.initial_root_states),
                                                     gymtorch.unwrap_tensor(ids32), k)
        self.gym.set_dof_state_tensor_indexed(self.sim, gymtorch.unwrap_tensor(self.dof_state),
                                              gymtorch.unwrap_tensor(ids32), k)
        planar = self.targets[env_ids] - self.initial_root_states[env_ids, 0:3]
        planar[:, 2] = 0.0
        self.prev_potentials[env_ids] = -torch.norm(planar, p=2, dim=-1) / self.dt
        self.potentials[env_ids] = self.prev_potentials[env_ids].clone()
        self.progress_buf[env_ids] = 0
        self.reset_buf[env_ids] = 0

    def compute_observations(self):
        self.gym.refresh_dof_state_tensor(self.sim)
        self.gym.refresh_actor_root_state_tensor(self.sim)
        self.gym.refresh_force_sensor_tensor(self.sim)
        obs, pot, prev, up, heading = compute_ant_observations(
            self.root_states, self.targets, self.potentials, self.inv_start_rot, self.dof_pos, self.dof_vel,
            self.dof_limits_lower, self.dof_limits_upper, self.dof_vel_scale, self.vec_sensor_tensor,
            self.actions, self.dt, self.contact_force_scale, self.basis_vec0, self.basis_vec1, self.up_axis_idx)
        self.obs_buf[:] = obs
        self.potentials[:] = pot
        self.prev_potentials[:] = prev
        self.up_vec[:] = up
        self.heading_vec[:] = heading

    def compute_reward(self, actions):
        self.rew_buf[:], self.reset_buf[:] = compute_ant_reward(
            self.obs_buf, self.reset_buf, self.progress_buf, self.actions, self.up_weight, self.heading_weight,
            self.potentials, self.prev_potentials, self.actions_cost_scale, self.energy_cost_scale,
            self.joints_at_limit_cost_scale, self.termination_height, self.death_cost, self.max_episode_length)

    def compute_true_objective(self):
        """Forward (x) root velocity, the PBT objective (ant.py:245-250)."""
        self.extras["true_objective"] = self.root_states[:, 7].squeeze()


def compute_ant_observations(root_states, targets, potentials, inv_start_rot, dof_pos, dof_vel, lower, upper,
                             dof_vel_scale: float, sensors, actions, dt: float, contact_force_scale: float,
                             basis_vec0, basis_vec1, up_axis_idx: int):
    """ant.py:374-406; returns (obs, potentials, previous potentials, up vector, heading vector)."""
    pos, rot = root_states[:, 0:3], root_states[:, 3:7]
    to_target = targets - pos
    to_target[:, 2] = 0.0
    prev = potentials.clone()
    pot = -torch.norm(to_target, p=2, dim=-1) / dt
    torso_quat, up_proj, heading_proj, up_vec, heading_vec = compute_heading_and_up(
        rot, inv_start_rot, to_target, basis_vec0, basis_vec1, 2)
    vel_loc, angvel_loc, roll, _pitch, yaw, angle_to_target = compute_rot(
        torso_quat, root_states[:, 7:10], root_states[:, 10:13], targets, pos)
    n = root_states.shape[0]
    obs = torch.empty((n, ANT_OBS), dtype=root_states.dtype, device=root_states.device)
    obs[:, OBS_HEIGHT] = pos[:, up_axis_idx]
    obs[:, 1:4] = vel_loc
    obs[:, 4:7] = angvel_loc
    obs[:, 7] = yaw
    obs[:, 8] = roll
    obs[:, 9] = angle_to_target
    obs[:, OBS_UP] = up_proj
    obs[:, OBS_HEADING] = heading_proj
    obs[:, OBS_DOF_POS] = unscale(dof_pos, lower, upper)
    obs[:, OBS_DOF_VEL] = dof_vel * dof_vel_scale
    obs[:, OBS_SENSORS] = sensors.view(-1, ANT_SENSORS * 6) * contact_force_scale
    obs[:, OBS_ACTIONS] = actions
    return obs, pot, prev, up_vec, heading_vec


def compute_ant_reward(obs, reset_buf, progress_buf, actions, up_weight: float, heading_weight: float, potentials,
                       prev_potentials, actions_cost_scale: float, energy_cost_scale: float,
                       joints_at_limit_cost_scale: float, termination_height: float, death_cost: float,
                       max_episode_length: float):
    """ant.py:325-371: progress + alive + upright + heading - action, energy and joint-limit costs;
    a fallen torso (height below terminationHeight) pays deathCost and resets, as does the episode end."""
    heading = obs[:, OBS_HEADING]
    heading_reward = torch.where(heading > 0.8, torch.ones_like(heading) * heading_weight,
                                 heading_weight * heading / 0.8)
    up_reward = torch.where(obs[:, OBS_UP] > 0.93, torch.zeros_like(heading_reward) + up_weight,
                            torch.zeros_like(heading_reward))
    actions_cost = torch.sum(actions ** 2, dim=-1)
    electricity_cost = torch.sum(torch.abs(actions * obs[:, OBS_DOF_VEL]), dim=-1)
    dof_at_limit_cost = torch.sum(obs[:, OBS_DOF_POS] > 0.99, dim=-1)
    alive_reward = torch.ones_like(potentials) * 0.5
    progress_reward = potentials - prev_potentials
    total = (progress_reward + alive_reward + up_reward + heading_reward - actions_cost_scale * actions_cost
             - energy_cost_scale * electricity_cost - dof_at_limit_cost * joints_at_limit_cost_scale)
    fallen = obs[:, OBS_HEIGHT] < termination_height
    total = torch.where(fallen, torch.ones_like(total) * death_cost, total)
    reset = torch.where(fallen, torch.ones_like(reset_buf), reset_buf)
    reset = torch.where(progress_buf >= max_episode_length - 1, torch.ones_like(reset_buf), reset)
    return total, reset
