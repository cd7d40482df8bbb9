"""Cartpole (reference ``tasks/cartpole.py``): BASELINE.json config 0, the plumbing case.

Same observation / reward / reset semantics and RNG draw order as the
reference (cartpole.py:131-196): efforts on DOF 0 only (a * maxEffort), one
simulate per step (dt 1/60, 2 substeps), reset of the envs flagged in the
PREVIOUS step at the start of post_physics_step, int64 reset buffer.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from isaacgym import gymapi, gymtorch

from .base.vec_task import VecTask


class Cartpole(VecTask):
    def __init__(self, cfg, rl_device, sim_device, graphics_device_id, headless, virtual_screen_capture,
                 force_render):
        self.cfg = cfg
        self.reset_dist = self.cfg["env"]["resetDist"]
        self.max_push_effort = self.cfg["env"]["maxEffort"]
        self.max_episode_length = 500
        self.cfg["env"]["numObservations"] = 4
        self.cfg["env"]["numActions"] = 1
        super().__init__(config=self.cfg, rl_device=rl_device, sim_device=sim_device,
                         graphics_device_id=graphics_device_id, headless=headless,
                         virtual_screen_capture=virtual_screen_capture, force_render=force_render)
        dof_state_tensor = self.gym.acquire_dof_state_tensor(self.sim)
        self.dof_state = gymtorch.wrap_tensor(dof_state_tensor)
        self.dof_pos = self.dof_state.view(self.num_envs, self.num_dof, 2)[..., 0]
        self.dof_vel = self.dof_state.view(self.num_envs, self.num_dof, 2)[..., 1]

    def create_sim(self):
        self.up_axis = self.cfg["sim"]["up_axis"]
        self.sim = super().create_sim(self.device_id, self.graphics_device_id, self.physics_engine, self.sim_params)
        self._create_ground_plane()
        self._create_envs(self.num_envs, self.cfg["env"]["envSpacing"], int(np.sqrt(self.num_envs)))

    def _create_ground_plane(self):
        plane = gymapi.PlaneParams()
        plane.normal = gymapi.Vec3(0.0, 0.0, 1.0) if self.up_axis == "z" else gymapi.Vec3(0.0, 1.0, 0.0)
        self.gym.add_ground(self.sim, plane)

    def _create_envs(self, num_envs, spacing, num_per_row):
        if self.up_axis == "z":
            lower, upper = gymapi.Vec3(0.5 * -spacing, -spacing, 0.0), gymapi.Vec3(0.5 * spacing, spacing, spacing)
        else:
            lower, upper = gymapi.Vec3(0.5 * -spacing, 0.0, -spacing), gymapi.Vec3(0.5 * spacing, spacing, spacing)
        here = os.path.dirname(os.path.abspath(__file__))
        asset_root = os.environ.get("ISAACGYMENVS_ASSET_ROOT", os.path.join(here, "../../assets"))
        asset_file = "urdf/cartpole.urdf"
        if "asset" in self.cfg["env"]:
            asset_root = os.path.join(here, self.cfg["env"]["asset"].get("assetRoot", asset_root))
            asset_file = self.cfg["env"]["asset"].get("assetFileName", asset_file)
        path = os.path.join(asset_root, asset_file)
        asset_root, asset_file = os.path.dirname(path), os.path.basename(path)
        opts = gymapi.AssetOptions()
        opts.fix_base_link = True
        asset = self.gym.load_asset(self.sim, asset_root, asset_file, opts)
        self.num_dof = self.gym.get_asset_dof_count(asset)
        pose = gymapi.Transform()
        if self.up_axis == "z":
            pose.p.z = 2.0
            pose.r = gymapi.Quat(0.0, 0.0, 0.0, 1.0)
        else:
            pose.p.y = 2.0
            pose.r = gymapi.Quat(-np.sqrt(2) / 2, 0.0, 0.0, np.sqrt(2) / 2)
        self.cartpole_handles = []
        self.envs = []
        for i in range(self.num_envs):
            env_ptr = self.gym.create_env(self.sim, lower, upper, num_per_row)
            handle = self.gym.create_actor(env_ptr, asset, pose, "cartpole", i, 1, 0)
            props = self.gym.get_actor_dof_properties(env_ptr, handle)
            props["driveMode"][0] = gymapi.DOF_MODE_EFFORT
            props["driveMode"][1] = gymapi.DOF_MODE_NONE
            props["stiffness"][:] = 0.0
            props["damping"][:] = 0.0
            self.gym.set_actor_dof_properties(env_ptr, handle, props)
            self.envs.append(env_ptr)
            self.cartpole_handles.append(handle)

    def compute_reward(self):
        pole_angle, pole_vel = self.obs_buf[:, 2], self.obs_buf[:, 3]
        cart_vel, cart_pos = self.obs_buf[:, 1], self.obs_buf[:, 0]
        self.rew_buf[:], self.reset_buf[:] = compute_cartpole_reward(
            pole_angle, pole_vel, cart_vel, cart_pos, self.reset_dist, self.reset_buf, self.progress_buf,
            self.max_episode_length)

    def compute_observations(self, env_ids=None):
        if env_ids is None:
            env_ids = np.arange(self.num_envs)
        self.gym.refresh_dof_state_tensor(self.sim)
        self.obs_buf[env_ids, 0] = self.dof_pos[env_ids, 0].squeeze()
        self.obs_buf[env_ids, 1] = self.dof_vel[env_ids, 0].squeeze()
        self.obs_buf[env_ids, 2] = self.dof_pos[env_ids, 1].squeeze()
        self.obs_buf[env_ids, 3] = self.dof_vel[env_ids, 1].squeeze()
        return self.obs_buf

    def reset_idx(self, env_ids):
        positions = 0.2 * (torch.rand((len(env_ids), self.num_dof), device=self.device) - 0.5)
        velocities = 0.5 * (torch.rand((len(env_ids), self.num_dof), device=self.device) - 0.5)
        self.dof_pos[env_ids, :] = positions[:]
        self.dof_vel[env_ids, :] = velocities[:]
        env_ids_int32 = env_ids.to(dtype=torch.int32)
        self.gym.set_dof_state_tensor_indexed(self.sim, gymtorch.unwrap_tensor(self.dof_state),
                                              gymtorch.unwrap_tensor(env_ids_int32), len(env_ids_int32))
        self.reset_buf[env_ids] = 0
        self.progress_buf[env_ids] = 0

    def pre_physics_step(self, actions):
        forces = torch.zeros(self.num_envs * self.num_dof, device=self.device, dtype=torch.float)
        forces[::self.num_dof] = actions.to(self.device).squeeze() * self.max_push_effort
        self.gym.set_dof_actuation_force_tensor(self.sim, gymtorch.unwrap_tensor(forces))

    def post_physics_step(self):
        self.progress_buf += 1
        env_ids = self.reset_buf.nonzero(as_tuple=False).squeeze(-1)
        if len(env_ids) > 0:
            self.reset_idx(env_ids)
        self.compute_observations()
        self.compute_reward()


def compute_cartpole_reward(pole_angle, pole_vel, cart_vel, cart_pos, reset_dist: float, reset_buf, progress_buf,
                            max_episode_length: float):
    """cartpole.py:180-196."""
    reward = 1.0 - pole_angle * pole_angle - 0.01 * torch.abs(cart_vel) - 0.005 * torch.abs(pole_vel)
    reward = torch.where(torch.abs(cart_pos) > reset_dist, torch.ones_like(reward) * -2.0, reward)
    reward = torch.where(torch.abs(pole_angle) > np.pi / 2, torch.ones_like(reward) * -2.0, reward)
    reset = torch.where(torch.abs(cart_pos) > reset_dist, torch.ones_like(reset_buf), reset_buf)
    reset = torch.where(torch.abs(pole_angle) > np.pi / 2, torch.ones_like(reset_buf), reset)
    reset = torch.where(progress_buf >= max_episode_length - 1, torch.ones_like(reset_buf), reset)
    return reward, reset
