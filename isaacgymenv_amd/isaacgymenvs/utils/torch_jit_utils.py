"""Quaternion / sampling helpers used on the hot path (xyzw quaternions).

Restates the subset of the reference's ``utils/torch_jit_utils.py`` the
in-scope tasks call, with the same formulas so results agree to float rounding:
``to_torch`` (:37), ``normalize`` (:66), ``quat_apply`` (:71), ``quat_rotate`` (:81),
``quat_rotate_inverse`` (:94), ``quat_conjugate`` (:107), ``quat_mul`` (:42),
``get_axis_params`` (:157), ``get_euler_xyz`` (:176), ``torch_rand_float`` (:216),
``tensor_clamp`` (:229), ``scale``/``unscale`` (:234-240),
``compute_heading_and_up`` (:248), ``compute_rot`` (:266).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch


def to_torch(x, dtype=torch.float, device="cuda:0", requires_grad=False):
    return torch.tensor(x, dtype=dtype, device=device, requires_grad=requires_grad)


def normalize(x: torch.Tensor, eps: float = 1e-9) -> torch.Tensor:
    return x / x.norm(p=2, dim=-1).clamp(min=eps, max=None).unsqueeze(-1)


def quat_mul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    shape = a.shape
    a = a.reshape(-1, 4)
    b = b.reshape(-1, 4)
    x1, y1, z1, w1 = a.unbind(-1)
    x2, y2, z2, w2 = b.unbind(-1)
    ww = (z1 + x1) * (x2 + y2)
    yy = (w1 - y1) * (w2 + z2)
    zz = (w1 + y1) * (w2 - z2)
    xx = ww + yy + zz
    qq = 0.5 * (xx + (z1 - x1) * (x2 - y2))
    w = qq - ww + (z1 - y1) * (y2 - z2)
    x = qq - xx + (x1 + w1) * (x2 + w2)
    y = qq - yy + (w1 - x1) * (y2 + z2)
    z = qq - zz + (z1 + y1) * (w2 - x2)
    return torch.stack([x, y, z, w], dim=-1).view(shape)


def quat_apply(q: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    shape = v.shape
    q = q.reshape(-1, 4)
    v = v.reshape(-1, 3)
    u = q[:, :3]
    t = torch.cross(u, v, dim=-1) * 2
    return (v + q[:, 3:] * t + torch.cross(u, t, dim=-1)).view(shape)


def _rotate(q: torch.Tensor, v: torch.Tensor, sign: float) -> torch.Tensor:
    n = q.shape[0]
    w = q[:, -1]
    u = q[:, :3]
    a = v * (2.0 * w ** 2 - 1.0).unsqueeze(-1)
    b = torch.cross(u, v, dim=-1) * w.unsqueeze(-1) * 2.0
    c = u * torch.bmm(u.view(n, 1, 3), v.view(n, 3, 1)).squeeze(-1) * 2.0
    return a + b + c if sign > 0 else a - b + c


def quat_rotate(q: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    return _rotate(q, v, 1.0)


def quat_rotate_inverse(q: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    return _rotate(q, v, -1.0)


def quat_conjugate(a: torch.Tensor) -> torch.Tensor:
    shape = a.shape
    a = a.reshape(-1, 4)
    return torch.cat((-a[:, :3], a[:, -1:]), dim=-1).view(shape)


def get_axis_params(value, axis_idx, x_value=0.0, dtype=float, n_dims=3):
    params = np.zeros((n_dims,))
    assert axis_idx < n_dims
    params[axis_idx] = value
    params[0] = x_value  # the reference overwrites component 0 unconditionally (torch_jit_utils.py:164)
    return list(params.astype(dtype))


def copysign(a: float, b: torch.Tensor) -> torch.Tensor:
    return torch.full_like(b, abs(a)) * torch.sign(b)


def get_euler_xyz(q: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    roll = torch.atan2(2.0 * (w * x + y * z), w * w - x * x - y * y + z * z)
    sinp = 2.0 * (w * y - z * x)
    pitch = torch.where(torch.abs(sinp) >= 1, copysign(np.pi / 2.0, sinp), torch.asin(sinp))
    yaw = torch.atan2(2.0 * (w * z + x * y), w * w + x * x - y * y - z * z)
    return roll % (2 * np.pi), pitch % (2 * np.pi), yaw % (2 * np.pi)


def torch_rand_float(lower: float, upper: float, shape: Tuple[int, int], device) -> torch.Tensor:
    return (upper - lower) * torch.rand(*shape, device=device) + lower


def tensor_clamp(t, min_t, max_t):
    return torch.max(torch.min(t, max_t), min_t)


def scale(x, lower, upper):
    return 0.5 * (x + 1.0) * (upper - lower) + lower


def unscale(x, lower, upper):
    return (2.0 * x - upper - lower) / (upper - lower)


def compute_heading_and_up(torso_rotation, inv_start_rot, to_target, vec0, vec1, up_idx: int):
    num_envs = torso_rotation.shape[0]
    target_dirs = normalize(to_target)
    torso_quat = quat_mul(torso_rotation, inv_start_rot)
    up_vec = quat_rotate(torso_quat, vec1).view(num_envs, 3)
    heading_vec = quat_rotate(torso_quat, vec0).view(num_envs, 3)
    up_proj = up_vec[:, up_idx]
    heading_proj = torch.bmm(heading_vec.view(num_envs, 1, 3), target_dirs.view(num_envs, 3, 1)).view(num_envs)
    return torso_quat, up_proj, heading_proj, up_vec, heading_vec


def compute_rot(torso_quat, velocity, ang_velocity, targets, torso_positions):
    vel_loc = quat_rotate_inverse(torso_quat, velocity)
    angvel_loc = quat_rotate_inverse(torso_quat, ang_velocity)
    roll, pitch, yaw = get_euler_xyz(torso_quat)
    walk_target_angle = torch.atan2(targets[:, 2] - torso_positions[:, 2], targets[:, 0] - torso_positions[:, 0])
    return vel_loc, angvel_loc, roll, pitch, yaw, walk_target_angle - yaw
