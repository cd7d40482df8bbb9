"""Probe: how often would ANYmal's non-adjacent shape pairs be within contact_offset under the bench workload
(AnymalTerrain, random actions)?  CPU pipeline (host backend), rigid-body states -> shape pair distances."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import isaacgymenv_amd  # noqa
import isaacgymenvs
from tests import helpers as H

n, steps = int(sys.argv[1]) if len(sys.argv) > 1 else 256, int(sys.argv[2]) if len(sys.argv) > 2 else 300
env = isaacgymenvs.make(seed=42, task="AnymalTerrain", num_envs=n, sim_device="cpu", rl_device="cpu", headless=True)
gym, sim = env.gym, env.sim
rb = __import__("isaacgymenv_amd.isaacgym.gymtorch", fromlist=["x"]).wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
art, flat = H.anymal()
# shapes: (body, kind, p0, p1, r) in body frame
shapes = []
for bi, b in enumerate(art.bodies):
    for s in b.shapes:
        if s.kind == 0:
            shapes.append((bi, s.pose.t, s.pose.t, s.size[0]))
        else:
            r, L = s.size; ax = s.pose.R @ np.array([0, 0, 1.0])
            shapes.append((bi, s.pose.t - 0.5 * L * ax, s.pose.t + 0.5 * L * ax, r))
par = [b.parent for b in art.bodies]
pairs = [(i, j) for i in range(len(shapes)) for j in range(i + 1, len(shapes))
         if shapes[i][0] != shapes[j][0] and par[shapes[i][0]] != shapes[j][0] and par[shapes[j][0]] != shapes[i][0]]
print(len(shapes), "shapes", len(pairs), "non-adjacent pairs")

def segdist(p1, q1, p2, q2):
    d1, d2, r = q1 - p1, q2 - p2, p1 - p2
    a = (d1 * d1).sum(-1); e = (d2 * d2).sum(-1); f = (d2 * r).sum(-1)
    c = (d1 * r).sum(-1); b = (d1 * d2).sum(-1)
    den = a * e - b * b
    s = np.where(den > 1e-12, np.clip((b * f - c * e) / np.maximum(den, 1e-12), 0, 1), 0.0)
    s = np.where(a > 1e-12, s, 0.0)
    t = np.where(e > 1e-12, (b * s + f) / np.maximum(e, 1e-12), 0.0)
    s = np.where(t < 0, np.where(a > 1e-12, np.clip(-c / np.maximum(a, 1e-12), 0, 1), 0), s)
    s = np.where(t > 1, np.where(a > 1e-12, np.clip((b - c) / np.maximum(a, 1e-12), 0, 1), 0), s)
    t = np.clip(t, 0, 1)
    c1 = p1 + d1 * s[..., None]; c2 = p2 + d2 * t[..., None]
    return np.linalg.norm(c1 - c2, axis=-1)

def quat_rot(q, v):
    x, y, z, w = q[..., 0:1], q[..., 1:2], q[..., 2:3], q[..., 3:4]
    u = np.concatenate([x, y, z], -1)
    t = 2 * np.cross(u, v)
    return v + w * t + np.cross(u, t)

cnt = np.zeros(len(pairs), dtype=np.int64); act_env_steps = 0; mind = np.full(len(pairs), 9.0)
torch.manual_seed(1)
for it in range(steps):
    env.step(2 * torch.rand(n, 12) - 1)
    gym.refresh_rigid_body_state_tensor(sim)
    st = rb.view(n, -1, 13).numpy().astype(np.float64)
    anyact = np.zeros(n, bool)
    for k, (i, j) in enumerate(pairs):
        bi, a0, a1, ra = shapes[i]; bj, b0, b1, rb_ = shapes[j]
        P, Q = st[:, bi, 0:3], st[:, bi, 3:7]; P2, Q2 = st[:, bj, 0:3], st[:, bj, 3:7]
        A0 = P + quat_rot(Q, np.broadcast_to(a0, P.shape)); A1 = P + quat_rot(Q, np.broadcast_to(a1, P.shape))
        B0 = P2 + quat_rot(Q2, np.broadcast_to(b0, P.shape)); B1 = P2 + quat_rot(Q2, np.broadcast_to(b1, P.shape))
        d = segdist(A0, A1, B0, B1) - ra - rb_
        a = d < 0.02
        cnt[k] += a.sum(); anyact |= a; mind[k] = min(mind[k], d.min())
    act_env_steps += anyact.sum()
names = [art.bodies[s[0]].name for s in shapes]
for k in np.argsort(-cnt)[:15]:
    i, j = pairs[k]
    print(f"{names[i]:>10s} - {names[j]:<10s} active env-steps {cnt[k]:8d}  min sep {mind[k]:+.3f}")
print("env-steps with any active pair:", act_env_steps, "of", n * steps, f"({act_env_steps / (n * steps):.4%})")
