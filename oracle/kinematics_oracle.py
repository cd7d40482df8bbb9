"""fp64 numpy restatement of the link kinematics the tensor API exports -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module; it never backs a product code path.

What it restates (the reference reads these through Isaac Gym, useful_hound.py:440-455 acquire,
:725-732 refresh, :660-691 OSC use):
* rigid body state per reported link: origin position, orientation (xyzw, w >= 0), COM linear
  velocity, angular velocity (world);
* Jacobian per link, rows = COM linear velocity (3) + angular velocity (3), columns = the
  generalized velocity nu = [root link COM linear velocity, root angular velocity, dof velocities];
* mass matrix M = sum_b J_b^T diag(m_b 1, I_b) J_b over the dynamic bodies.

Parity with PhysX's own jacobian / mass-matrix tensors is UNPINNED (Isaac Gym is a closed binary,
SURVEY.md section 8c); this oracle is pinned instead by known answers (cartpole's analytic mass
matrix, FK at q = 0 from the URDF joint origins) and by finite differences of its own FK
(tests/test_kinematics_oracle.py), and the HIP kernel (gs_kinematics.hip) is checked against it.

Inputs use the internal state layout of the simulator: root [13] = pos, quat xyzw, root ORIGIN
linear velocity, angular velocity; dof [nd][2] = (q, qd).
"""
from __future__ import annotations

import numpy as np


def quat_to_mat(q):
    x, y, z, w = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def mat_to_quat(m):
    """Shepperd's method, w >= 0 (the kernel's canonical sign)."""
    t = np.trace(m)
    if t > 0:
        s = np.sqrt(t + 1.0) * 2
        w, x, y, z = 0.25 * s, (m[2, 1] - m[1, 2]) / s, (m[0, 2] - m[2, 0]) / s, (m[1, 0] - m[0, 1]) / s
    elif m[0, 0] > m[1, 1] and m[0, 0] > m[2, 2]:
        s = np.sqrt(1.0 + m[0, 0] - m[1, 1] - m[2, 2]) * 2
        w, x, y, z = (m[2, 1] - m[1, 2]) / s, 0.25 * s, (m[0, 1] + m[1, 0]) / s, (m[0, 2] + m[2, 0]) / s
    elif m[1, 1] > m[2, 2]:
        s = np.sqrt(1.0 + m[1, 1] - m[0, 0] - m[2, 2]) * 2
        w, x, y, z = (m[0, 2] - m[2, 0]) / s, (m[0, 1] + m[1, 0]) / s, 0.25 * s, (m[1, 2] + m[2, 1]) / s
    else:
        s = np.sqrt(1.0 + m[2, 2] - m[0, 0] - m[1, 1]) * 2
        w, x, y, z = (m[1, 0] - m[0, 1]) / s, (m[0, 2] + m[2, 0]) / s, (m[1, 2] + m[2, 1]) / s, 0.25 * s
    q = np.array([x, y, z, w])
    q /= np.linalg.norm(q)
    return -q if q[3] < 0 else q


def rodrigues(axis, th):
    a = np.asarray(axis, dtype=np.float64)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * (K @ K)


def fk(flat, root, q):
    """Body frames (R [nb,3,3], p [nb,3]), joint axes and points (world) for one env."""
    nb = flat["nb"]
    R = np.zeros((nb, 3, 3))
    p = np.zeros((nb, 3))
    a = np.zeros((nb, 3))
    o = np.zeros((nb, 3))
    R[0] = quat_to_mat(root[3:7] / np.linalg.norm(root[3:7]))
    p[0] = root[0:3]
    for b in range(1, nb):
        pb = flat["parent"][b]
        jR = flat["jorigin"][b, :9].reshape(3, 3)
        jt = flat["jorigin"][b, 9:]
        Rj = R[pb] @ jR
        o[b] = p[pb] + R[pb] @ jt
        a[b] = Rj @ flat["jaxis"][b]
        j = flat["bdof"][b]
        qj = q[j] if j >= 0 else 0.0
        kind = flat["jkind"][b]
        if kind == 1:
            R[b] = Rj @ rodrigues(flat["jaxis"][b], qj)
            p[b] = o[b]
        else:
            R[b] = Rj
            p[b] = o[b] + (a[b] * qj if kind == 2 else 0.0)
    return R, p, a, o


def _ancestors(flat, b):
    out = set()
    while b >= 0:
        out.add(b)
        b = flat["parent"][b]
    return out


def point_jacobian(flat, R, p, a, o, b, x):
    """[6, nv] Jacobian of point x rigidly attached to body b: rows (linear, angular)."""
    nbase = 0 if flat["fixed_base"] else 6
    nd = flat["nd"]
    J = np.zeros((6, nbase + nd))
    croot = p[0] + R[0] @ flat["lcom"][0]  # root LINK COM (the root link's frame is body 0's)
    if nbase:
        J[0:3, 0:3] = np.eye(3)
        for k in range(3):
            e = np.zeros(3)
            e[k] = 1.0
            J[3:6, 3 + k] = e
            J[0:3, 3 + k] = np.cross(e, x - croot)
    anc = _ancestors(flat, b)
    for bj in range(1, flat["nb"]):
        j = flat["bdof"][bj]
        if j < 0 or bj not in anc:
            continue
        if flat["jkind"][bj] == 2:
            J[0:3, nbase + j] = a[bj]
        else:
            J[3:6, nbase + j] = a[bj]
            J[0:3, nbase + j] = np.cross(a[bj], x - o[bj])
    return J


def generalized_velocity(flat, root, dof, R, p):
    nbase = 0 if flat["fixed_base"] else 6
    nu = np.zeros(nbase + flat["nd"])
    if nbase:
        c = p[0] + R[0] @ flat["lcom"][0]
        w = root[10:13]
        nu[0:3] = root[7:10] + np.cross(w, c - p[0])
        nu[3:6] = w
    nu[nbase:] = dof[:, 1]
    return nu


def link_frames(flat, R, p):
    """World rotation, origin and COM of every reported link."""
    out = []
    for l in range(flat["nr"]):
        b = flat["lbody"][l]
        lR = flat["lpose"][l, :9].reshape(3, 3)
        lt = flat["lpose"][l, 9:]
        Rl = R[b] @ lR
        pl = p[b] + R[b] @ lt
        out.append((b, Rl, pl, pl + Rl @ flat["lcom"][l]))
    return out


def env_kinematics(flat, root, dof):
    """(rigid body state [nr,13], jacobian [nr,6,nv], mass matrix [nv,nv]) for one env."""
    root = np.asarray(root, dtype=np.float64)
    dof = np.asarray(dof, dtype=np.float64)
    R, p, a, o = fk(flat, root, dof[:, 0])
    nu = generalized_velocity(flat, root, dof, R, p)
    nr = flat["nr"]
    nv = nu.size
    rb = np.zeros((nr, 13))
    jac = np.zeros((nr, 6, nv))
    for l, (b, Rl, pl, xc) in enumerate(link_frames(flat, R, p)):
        J = point_jacobian(flat, R, p, a, o, b, xc)
        jac[l] = J
        v = J @ nu
        rb[l, 0:3] = pl
        rb[l, 3:7] = root[3:7] / np.linalg.norm(root[3:7]) if l == 0 else mat_to_quat(Rl)
        rb[l, 7:10] = v[0:3]
        rb[l, 10:13] = v[3:6]
    M = np.zeros((nv, nv))
    for b in range(flat["nb"]):
        c = p[b] + R[b] @ flat["com"][b]
        J = point_jacobian(flat, R, p, a, o, b, c)
        Iw = R[b] @ flat["inertia"][b].reshape(3, 3) @ R[b].T
        M += flat["mass"][b] * J[0:3].T @ J[0:3] + J[3:6].T @ Iw @ J[3:6]
    return rb, jac, M


def batch(flat, root, dof):
    """env_kinematics over [N] envs -> ([N*nr,13], [N,nr,6,nv], [N,nv,nv])."""
    outs = [env_kinematics(flat, root[e], dof[e]) for e in range(root.shape[0])]
    rb = np.concatenate([o[0] for o in outs], axis=0)
    return rb, np.stack([o[1] for o in outs]), np.stack([o[2] for o in outs])
