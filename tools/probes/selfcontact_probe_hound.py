"""Probe: UsefulHound non-adjacent shape pairs under random actions (CPU pipeline): approximate shapes by point
sets (box: surface grid, hull: its vertices, capsule: segment samples + radius, sphere: centre + radius) and
report pairs whose separation falls below contact_offset."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import isaacgymenv_amd  # noqa
import isaacgymenvs
from isaacgymenv_amd.isaacgym import gymtorch
from tests import helpers as H

n, steps = int(sys.argv[1]), int(sys.argv[2])
env = isaacgymenvs.make(seed=42, task="UsefulHound", num_envs=n, sim_device="cpu", rl_device="cpu", headless=True)
gym, sim = env.gym, env.sim
rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
art = env.sim.art if hasattr(env.sim, "art") else None
art, flat = H.hound()
links = art.link_table()
# shapes per LINK (reported rigid bodies: rigid_body_state rows are links)
shapes = []  # (link, pts [k,3] in link frame, radius)
s_index = 0
for bi, b in enumerate(art.bodies):
    for s in b.shapes:
        li = art.shape_links[s_index] if art.shape_links is not None else bi
        # shape pose is in the BODY frame; convert to the link frame
        lp = links[li].pose
        Rinv = lp.R.T
        def to_link(p):
            return (Rinv @ (np.asarray(p) - lp.t).T).T
        if s.kind == 0:
            pts, r = to_link(s.pose.t[None]), s.size[0]
        elif s.kind in (1, 3):
            r, L = s.size; ax = s.pose.R @ np.array([0, 0, 1.0])
            pts = to_link(np.array([s.pose.t + (u - 0.5) * L * ax for u in np.linspace(0, 1, 9)])); r = r
        elif s.kind == 2:
            h = 0.5 * np.array(s.size)
            g = np.linspace(-1, 1, 6)
            P = np.array([[x, y, z] for x in g for y in g for z in g])
            P = P[(np.abs(P) == 1).any(1)] * h
            pts, r = to_link(np.array([s.pose.apply(p) for p in P])), 0.0
        else:
            pts, r = to_link(np.array([s.pose.apply(p) for p in np.asarray(s.size).reshape(-1, 3)])), 0.0
        shapes.append((li, pts, r))
        s_index += 1
lpar = [l.parent for l in links]
lbody = [l.body for l in links]
def adjacent(a, b):
    # PhysX: links joined by a joint (parent-child) do not collide; links welded into the same body are one body
    return lpar[a] == b or lpar[b] == a or lbody[a] == lbody[b]
pairs = [(i, j) for i in range(len(shapes)) for j in range(i + 1, len(shapes))
         if shapes[i][0] != shapes[j][0] and not adjacent(shapes[i][0], shapes[j][0])]
names = [links[s[0]].name for s in shapes]
print(len(shapes), "shapes", len(pairs), "non-adjacent pairs")

def quat_rot(q, v):
    u, w = q[..., :3], q[..., 3:4]
    t = 2 * np.cross(u, v)
    return v + w * t + np.cross(u, t)

cnt = np.zeros(len(pairs), np.int64); mind = np.full(len(pairs), 9.0)
torch.manual_seed(1)
for it in range(steps + 1):
    if it:
        env.step(2 * torch.rand(n, 18) - 1)
    gym.refresh_rigid_body_state_tensor(sim)
    st = rb.view(n, -1, 13).numpy().astype(np.float64)
    W = []
    for li, pts, r in shapes:
        P, Q = st[:, li, None, 0:3], st[:, li, None, 3:7]
        W.append(P + quat_rot(np.broadcast_to(Q, (n, len(pts), 4)), np.broadcast_to(pts, (n, len(pts), 3))))
    for k, (i, j) in enumerate(pairs):
        d = np.linalg.norm(W[i][:, :, None] - W[j][:, None], axis=-1).min((1, 2)) - shapes[i][2] - shapes[j][2]
        cnt[k] += (d < 0.02).sum(); mind[k] = min(mind[k], d.min())
    if it == 0:
        print("rest pose: pairs below 0.02:", [(names[pairs[k][0]], names[pairs[k][1]], round(mind[k], 3)) for k in range(len(pairs)) if mind[k] < 0.02])
for k in np.argsort(mind)[:20]:
    i, j = pairs[k]
    print(f"{names[i]:>12s} - {names[j]:<12s} active env-steps {cnt[k]:7d}  min sep {mind[k]:+.3f}")
