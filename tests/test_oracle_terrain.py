"""CPU oracle: contacts against the heightfield triangle mesh (parity vs PhysX unpinned).

Known answers that pin the mesh contact generation and its contact frames:
* a flat mesh at z = 0 reproduces the ground plane exactly (same rows, frames and iterates);
* on an inclined planar mesh the dynamics equal the flat-plane dynamics in the rotated frame with
  gravity rotated the other way (rotational invariance of contact normal and box-friction axes).
"""
import numpy as np

from oracle.oracle import OracleSim
from tests import helpers as H


def _flat_mesh(z_fn, lo=-6.0, n=121, hs=0.1):
    xs = lo + hs * np.arange(n)
    gx, gy = np.meshgrid(xs, xs, indexing="ij")
    v = np.stack([gx, gy, z_fn(gx, gy)], axis=-1).reshape(-1, 3).astype(np.float32)
    from isaacgymenv_amd.isaacgym.terrain_utils import convert_heightfield_to_trimesh
    _, t = convert_heightfield_to_trimesh(np.zeros((n, n), np.int16), hs, 0.005, None)
    return H.mesh_terrain(v, t, n, n, hs)["oracle"]


def test_flat_mesh_equals_ground_plane():
    art, flat = H.anymal()
    root, dof, tau, mu = H.anymal_states(64, seed=4)
    root[:, 2] += 0.1  # penetrations within the mesh's back window (r + 0.1), unlike the plane's unbounded one
    plane = OracleSim(flat, H.ANYMAL_PARAMS)
    mesh = OracleSim(flat, dict(H.ANYMAL_PARAMS, has_ground=0), terrain=_flat_mesh(lambda x, y: 0 * x))
    r1, d1, r2, d2 = root.copy(), dof.copy(), root.copy(), dof.copy()
    c1, c2 = np.zeros((64, flat["nb"], 3)), np.zeros((64, flat["nb"], 3))
    for _ in range(5):
        plane.simulate(r1, d1, np.ascontiguousarray(tau), mu, c1)
        mesh.simulate(r2, d2, np.ascontiguousarray(tau), mu, c2)
    assert np.abs(c1).sum() > 100  # contacts happened
    np.testing.assert_allclose(r2, r1, atol=1e-9)
    np.testing.assert_allclose(d2, d1, atol=1e-8)
    np.testing.assert_allclose(c2, c1, atol=1e-6)


def _rot_y(th):
    c, s = np.cos(th), np.sin(th)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def _quat_mul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])


def test_inclined_mesh_equals_rotated_flat_world():
    th = 0.2  # rad: the plane z = x tan(th) is the flat plane rotated by -th about y
    art, flat = H.anymal()
    n = 32
    root, dof, tau, mu = H.anymal_states(n, seed=5, spread=0.5)
    root[:, 0:2] = np.random.RandomState(1).uniform(-1, 1, (n, 2))
    Rw = _rot_y(-th)  # flat frame -> world
    qw = np.array([0.0, np.sin(-th / 2), 0.0, np.cos(-th / 2)])
    g = np.array([0.0, 0.0, -9.81])
    flat_sim = OracleSim(flat, dict(H.ANYMAL_PARAMS, gravity=list(Rw.T @ g)))
    mesh_sim = OracleSim(flat, dict(H.ANYMAL_PARAMS, has_ground=0),
                         terrain=_flat_mesh(lambda x, y: x * np.tan(th)))
    rw = root.copy()
    for i in range(n):
        rw[i, 0:3] = Rw @ root[i, 0:3]
        rw[i, 3:7] = _quat_mul(qw, root[i, 3:7])
        rw[i, 7:10] = Rw @ root[i, 7:10]
        rw[i, 10:13] = Rw @ root[i, 10:13]
    d1, d2 = dof.copy(), dof.copy()
    for _ in range(5):
        flat_sim.simulate(root, d1, np.ascontiguousarray(tau), mu)
        mesh_sim.simulate(rw, d2, np.ascontiguousarray(tau), mu)
    back = rw.copy()
    for i in range(n):
        back[i, 0:3] = Rw.T @ rw[i, 0:3]
        back[i, 3:7] = _quat_mul(np.array([-qw[0], -qw[1], -qw[2], qw[3]]), rw[i, 3:7])
        back[i, 7:10] = Rw.T @ rw[i, 7:10]
        back[i, 10:13] = Rw.T @ rw[i, 10:13]
    # float32 mesh vertices: the plane is exact to ~1e-7 m
    np.testing.assert_allclose(back[:, 0:3], root[:, 0:3], atol=2e-5)
    np.testing.assert_allclose(np.abs(np.sum(back[:, 3:7] * root[:, 3:7], axis=1)), 1.0, atol=1e-8)
    np.testing.assert_allclose(back[:, 7:13], root[:, 7:13], atol=5e-3)
    np.testing.assert_allclose(d2, d1, atol=5e-3)


def test_rough_terrain_supports_a_standing_robot():
    """On stairs / blocks the feet find the surface: a PD-held robot dropped above the terrain comes
    to rest on it (no fall-through) with its weight on the contacts."""
    art, flat = H.anymal()
    ter = H.rough_terrain(seed=3)
    sim = OracleSim(flat, dict(H.ANYMAL_PARAMS, has_ground=0), terrain=ter["oracle"])
    q0 = np.array([H.ANYMAL_DEFAULT[d] for d in art.dof_names()])
    n = 6
    root = np.zeros((n, 13)); root[:, 6] = 1.0
    root[:, 0] = np.linspace(-2.5, 2.5, n)
    root[:, 1] = np.linspace(-1.5, 1.5, n)
    # start 0.7 m above the highest mesh point under the body
    v = ter["oracle"]["vertices"].reshape(-1, 3)
    lo, hi = np.zeros(n), np.zeros(n)
    for i in range(n):
        near = (np.abs(v[:, 0] - root[i, 0]) < 0.6) & (np.abs(v[:, 1] - root[i, 1]) < 0.4)
        lo[i], hi[i] = v[near, 2].min(), v[near, 2].max()
        root[i, 2] = hi[i] + 0.7
    dof = np.zeros((n, 12, 2)); dof[:, :, 0] = q0
    mu = np.ones((n, flat["ns"]))
    cf = np.zeros((n, flat["nb"], 3))
    z0 = root[:, 2].copy()
    for _ in range(600):
        tau = np.clip(80 * (q0 - dof[:, :, 0]) - 2 * dof[:, :, 1], -80, 80)
        sim.simulate(root, dof, np.ascontiguousarray(tau), mu, cf)
    weight = sum(b.mass for b in art.bodies) * 9.81
    assert np.all(np.isfinite(root))
    assert np.all(root[:, 2] < z0 - 0.1), root[:, 2] - z0
    # standing on the surface under it (base 0.3-0.65 m above the local terrain), not through it
    assert np.all(root[:, 2] > lo + 0.3) and np.all(root[:, 2] < hi + 0.65), (root[:, 2] - lo, root[:, 2] - hi)
    np.testing.assert_allclose(np.linalg.norm(cf.sum(1), axis=1), weight, rtol=0.1)
