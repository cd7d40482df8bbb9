"""Self-collision of filter-0 actors and exact convex-hull ground contacts.

Reference: AnymalTerrain and UsefulHound create their actors with collision filter 0
(anymal_terrain.py:282, useful_hound.py:421), which makes Isaac Gym collide the actor's own shapes except on
links joined by a joint; UsefulHound's arm collides through STL meshes (Hound.urdf:508-733,
useful_hound.py:329) that Isaac Gym treats as their convex hulls.  Parity vs PhysX is unpinned (closed,
absent); the oracle (oracle/physics_oracle.c) restates the rules and is pinned here by known answers:

* the pair table: every shape pair on links that are not jointed and not the same dynamic body;
* internal impulses: in zero gravity without ground, self-contacts change no total linear momentum, and
  legs pressed into each other are pushed apart;
* a convex hull's ground contact is its true lowest vertex at any orientation (the old 14-direction
  sampling missed it), and a hull face resting on the ground contacts at the face's corners.

The host backend (the same solver source as the HIP kernels) and, with -m gpu, the one-env-per-lane and
lane-team kernels are checked against the oracle on ANYmal states with crossed legs.
"""
import numpy as np
import pytest
import torch

from oracle import kinematics_oracle as KO
from oracle.oracle import OracleSim
from tests import helpers as H


def crossed_leg_states(n, seed=3, min_contacts=1, spread=1.2, pool=40):
    """ANYmal states with wide joint perturbations, first `n` of them that have at least `min_contacts`
    self-contacts (oracle)."""
    art, flat = H.anymal()
    m = pool * n
    rng = np.random.RandomState(seed)
    root, dof, tau, mu = H.anymal_states(m, seed=seed)
    dof[:, :, 0] += rng.uniform(-spread, spread, (m, 12))
    o = OracleSim(flat, H.ANYMAL_PARAMS)
    c, cnt = o.self_contacts(root, dof, mu)
    idx = np.nonzero(cnt >= min_contacts)[0][:n]
    assert len(idx) == n
    return root[idx].copy(), dof[idx].copy(), tau[idx].copy(), mu[idx].copy()


def test_pair_tables():
    from isaacgymenv_amd.isaacgym._assets import PAIR_CC, PAIR_SC, PAIR_SS
    art, flat = H.anymal()
    lt = art.link_table()
    par = [l.parent for l in lt]
    pairs = art.self_collision_pairs()
    # 9 shapes (base capsule, 4 knee capsules, 4 foot spheres); THIGH-SHANK of a leg are jointed
    assert len(pairs) == flat["npair"] == 32 and flat["npool"] == 4
    tab = art.shape_table()
    for a, b, kind, _ in pairs:
        la, lb = tab[a]["link"], tab[b]["link"]
        assert la != lb and par[la] != lb and par[lb] != la
        assert kind in (PAIR_SS, PAIR_SC, PAIR_CC)
    # UsefulHound: links welded into one dynamic body never pair; its flat-ended cylinders pair through GJK
    art, flat = H.hound()
    tab = art.shape_table()
    assert all(tab[a]["body"] != tab[b]["body"] for a, b, _, _ in art.self_collision_pairs())
    assert {t["kind"] for t in tab} == {0, 2, 3, 4}


def test_self_contacts_conserve_momentum_and_push_legs_apart():
    """Zero gravity, no ground, no torque: self-contact impulses are internal (total linear momentum
    unchanged to fp64 rounding) and legs pressed into each other separate within a few substeps."""
    n = 24
    art, flat = H.anymal()
    root, dof, tau, mu = crossed_leg_states(n)
    params = dict(H.ANYMAL_PARAMS, gravity=[0.0, 0.0, 0.0], has_ground=0)
    o = OracleSim(flat, params)
    c0, k0 = o.self_contacts(root, dof, mu)
    assert (k0 > 0).all() and c0[:, 0, 6].min() < -0.005

    def momentum(r, d):
        """Total linear momentum of the new velocities at the step's starting configuration (the semi-implicit
        step solves M(q0) (v1 - v_free) = J^T lambda there)."""
        r0, d0 = root.copy(), dof.copy()
        r0[:, 7:13] = r[:, 7:13]
        d0[:, :, 1] = d[:, :, 1]
        rb, _, _ = KO.batch(flat, r0, d0)
        v = rb[:, 7:10].reshape(n, flat["nr"], 3)
        return (flat["mass"][None, :, None] * v).sum(1)

    r, d = root.copy(), dof.copy()
    zero = np.zeros((n, 12))
    o.simulate(r, d, zero, mu)
    # the same step without self-collision: same total momentum (the contact impulses are internal; the
    # integrator's own momentum change -- velocity limits, the mixed-frame term -- is common to both), and
    # the legs stay interpenetrating
    r_off, d_off = root.copy(), dof.copy()
    OracleSim(flat, params, self_collide=False).simulate(r_off, d_off, zero, mu)
    p_on, p_off = momentum(r, d), momentum(r_off, d_off)
    # (envs where a joint hit its 20 rad/s velocity limit are excluded: the clamp is not momentum-conserving)
    free = (np.abs(d[:, :, 1]) < 0.999 * flat["vmax"]).all(1) & (np.abs(d_off[:, :, 1]) < 0.999 * flat["vmax"]).all(1)
    assert free.sum() >= n // 2
    assert np.abs(p_on - p_off)[free].max() <= 1e-9 * max(1.0, np.abs(p_off).max())
    assert np.abs(d_off - d).max() > 1e-3
    for _ in range(200):
        o.simulate(r, d, zero, mu)
    c1, k1 = o.self_contacts(r, d, mu)
    deepest0 = c0[:, 0, 6]
    deepest1 = np.where(k1 > 0, np.where(np.arange(4)[None] < k1[:, None], c1[:, :, 6], 1.0).min(1), 1.0)
    pressed = deepest0 < -0.005
    assert pressed.sum() >= n // 4
    assert (deepest1[pressed] > deepest0[pressed]).all() and deepest1.min() > -0.01


def _hull_model(tmp_path, points):
    """A free body whose only collision shape is the STL mesh of `points` (triangles of their hull)."""
    from scipy.spatial import ConvexHull
    from isaacgymenv_amd.isaacgym import _assets as A
    from isaacgymenv_amd.isaacgym._model import flatten
    hull = ConvexHull(points)
    rec = np.zeros(len(hull.simplices), dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
    rec["v"] = points[hull.simplices].astype(np.float32)
    (tmp_path / "blob.stl").write_bytes(b"\0" * 80 + len(rec).to_bytes(4, "little") + rec.tobytes())
    (tmp_path / "blob.urdf").write_text(
        '<robot name="blob"><link name="body"><inertial><mass value="1.0"/>'
        '<inertia ixx="0.01" iyy="0.01" izz="0.01" ixy="0" ixz="0" iyz="0"/></inertial>'
        '<collision><geometry><mesh filename="blob.stl"/></geometry></collision></link></robot>')
    art = A.build_articulation(A.parse_urdf(str(tmp_path / "blob.urdf")), {})
    flat = flatten(art)
    return art, flat


def test_hull_ground_contact_is_the_lowest_vertex(tmp_path):
    """At random orientations the hull's deepest ground contact is its lowest vertex (argmin of the world
    height over every hull vertex); the former 14-direction support sampling misses it for most of them."""
    rng = np.random.RandomState(0)
    pts = rng.normal(size=(300, 3))
    pts = 0.05 * pts / np.linalg.norm(pts, axis=1, keepdims=True) * rng.uniform(0.9, 1.0, (300, 1))
    art, flat = _hull_model(tmp_path, pts)
    hv = flat["hverts"][:, :3]
    assert len(hv) > 100
    o = OracleSim(flat, H.ANYMAL_PARAMS)
    dirs = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]] +
                    [[a, b, c] for a in (-1, 1) for b in (-1, 1) for c in (-1, 1)], dtype=np.float64)
    support14 = {int(np.argmax(hv @ d)) for d in dirs}
    missed = 0
    for _ in range(50):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        R = KO.quat_to_mat(q)
        z = (hv @ R.T)[:, 2]
        lo = int(np.argmin(z))
        sel = o.hull_select(0, R, np.zeros(3), rootz=0.003 - z[lo])   # lowest vertex 3 mm above the ground
        assert sel[0] == lo
        # every selected vertex is within contact_offset of the ground
        assert ((z[sel] + 0.003 - z[lo]) < 0.02).all()
        missed += lo not in support14
    assert missed > 25


def test_hull_face_on_ground_contacts_at_its_corners(tmp_path):
    """A box-shaped hull resting on a face: the 4 contacts are the face's corners."""
    corners = np.array([[x, y, z] for x in (-0.1, 0.1) for y in (-0.05, 0.05) for z in (-0.02, 0.02)])
    extra = np.array([[0.0, 0.0, 0.02], [0.05, 0.0, -0.02], [0.0, 0.03, 0.02]])   # face-interior points
    art, flat = _hull_model(tmp_path, np.concatenate([corners, extra]))
    hv = flat["hverts"][:, :3]
    o = OracleSim(flat, H.ANYMAL_PARAMS)
    sel = o.hull_select(0, np.eye(3), np.zeros(3), rootz=0.02 - 0.001)
    bottom = {tuple(np.round(c, 6)) for c in corners if c[2] < 0}
    assert len(sel) == 4 and {tuple(np.round(hv[i], 6)) for i in sel} == bottom


def _sim_vs_oracle(host, variant=0, n=48, steps=1, states=None):
    art, flat = H.anymal()
    root, dof, tau, mu = states if states is not None else crossed_leg_states(n)
    gym, sim = H.make_gpu_sim("anymal", n, H.ANYMAL_PARAMS, host=host)
    if variant:
        assert sim.kernel_variant == variant, sim.kernel_variant
    H.load_state_into(sim, root, dof, mu)
    dev = sim.state.device
    sim.dof_force.copy_(torch.from_numpy(tau.astype(np.float32).reshape(-1)).to(dev))
    for _ in range(steps):
        gym.simulate(sim)
    if not host:
        torch.cuda.synchronize()
    g_root, g_dof = H.read_state(sim, 12)
    g_cf = sim.cf_soa.cpu().numpy().T.reshape(n, 13, 3).astype(np.float64)
    o = OracleSim(flat, H.ANYMAL_PARAMS)
    r, d, cf = root.copy(), dof.copy(), np.zeros((n, 13, 3))
    for _ in range(steps):
        o.simulate(r, d, np.ascontiguousarray(tau), mu, cf)
    # without self-collision the oracle ends elsewhere: the pairs are in effect
    r2, d2 = root.copy(), dof.copy()
    for _ in range(steps):
        OracleSim(flat, H.ANYMAL_PARAMS, self_collide=False).simulate(r2, d2, np.ascontiguousarray(tau), mu)
    assert np.abs(d2[:, :, 1] - d[:, :, 1]).max() > 0.1
    assert np.all(np.isfinite(g_root)) and np.all(np.isfinite(g_dof))
    # worst env reported (no element fraction): one substep from identical states
    err_q = np.abs(g_dof[:, :, 0] - d[:, :, 0]).max()
    err_p = np.abs(g_root[:, 0:7] - r[:, 0:7]).max()
    err_v = (np.abs(g_dof[:, :, 1] - d[:, :, 1]) / (5e-3 + 5e-3 * np.abs(d[:, :, 1]))).max()
    err_f = (np.abs(g_cf - cf) / (1.0 + 2e-2 * np.abs(cf))).max()
    assert err_q <= 2e-5 and err_p <= 2e-5, (err_q, err_p)
    assert err_v <= 1.0 and err_f <= 1.0, (err_v, err_f)
    return sim


def test_host_self_contacts_match_oracle():
    _sim_vs_oracle(host=True)


@pytest.mark.gpu
def test_lane_kernel_self_contacts_match_oracle():
    art, flat = H.anymal()
    from isaacgymenv_amd.isaacgym import gymapi  # noqa: F401
    sim = _sim_vs_oracle(host=False)
    assert sim.kernel_variant in (1, 2)


@pytest.mark.gpu
def test_team_kernel_self_contacts_match_oracle():
    _sim_vs_oracle(host=False, variant=2)


@pytest.mark.gpu
def test_team_kernel_full_self_contact_pools_match_oracle():
    """States whose pool is full (the oracle keeps NPK = 4 contacts in pair order and drops later ones): the
    team narrowphase keeps each lane's NPK contacts of smallest pair order (round 6, gs_team.hip team_lc), so a
    lane that finds more than two contacts -- which took the replicated narrowphase before -- still yields the
    oracle's pool."""
    states = crossed_leg_states(32, seed=5, min_contacts=4, spread=1.8, pool=200)
    _sim_vs_oracle(host=False, variant=2, n=32, states=states)


def _pool_vs_oracle(pools, flat, root, dof, mu, what):
    """Self-contact pools (gs_debug_self_contacts) against the oracle's from the same states: same contact count
    in >= 98 % of the envs; where the counts agree, every contact's point, normal and separation within 1e-2
    (the fp32 GJK's contact normal on near-parallel hull faces)."""
    o_pool, o_cnt = OracleSim(flat, H.HOUND_PARAMS).self_contacts(root, dof, mu)
    g_pool, g_cnt = pools
    n = len(o_cnt)
    same = g_cnt == o_cnt
    assert same.mean() >= 0.98, (what, np.nonzero(~same)[0][:10])
    assert o_cnt.sum() > n, "the states must have self-contacts"
    worst = 0.0
    for e in np.nonzero(same)[0]:
        k = o_cnt[e]
        if k:
            assert np.array_equal(g_pool[e, :k, 8:10], o_pool[e, :k, 8:10]), (what, e)  # same pairs, same order
            worst = max(worst, float(np.abs(g_pool[e, :k, :7] - o_pool[e, :k, :7]).max()))
    assert worst <= 1e-2, (what, worst)
    H.parity_report(f"{what}: self-contact pools vs oracle, {int(same.sum())} of {n} envs with equal counts, "
                    f"worst point / normal / separation difference {worst:.3g}")


def test_host_hound_self_contact_pools_match_oracle():
    n = 96
    art, flat = H.hound()
    root, dof, tau, mu = H.hound_states(n, seed=9)
    gym, sim = H.make_host_sim("hound", n, H.HOUND_PARAMS)
    H.load_state_into(sim, root, dof, mu)
    _pool_vs_oracle(H.sim_self_contacts(sim, 0), flat, root, dof, mu, "hound host")


@pytest.mark.gpu
def test_gpu_hound_self_contact_pools_match_oracle():
    """Device pools in both forms -- inline narrowphase, and the split form's near-pair records kernel plus the
    records' gather (what UsefulHound's simulate runs) -- against the oracle, and against each other."""
    n = 256
    art, flat = H.hound()
    root, dof, tau, mu = H.hound_states(n, seed=9)
    gym, sim = H.make_gpu_sim("hound", n, H.HOUND_PARAMS)
    H.load_state_into(sim, root, dof, mu)
    inline = H.sim_self_contacts(sim, 0)
    records = H.sim_self_contacts(sim, 1)
    _pool_vs_oracle(inline, flat, root, dof, mu, "hound gpu inline")
    _pool_vs_oracle(records, flat, root, dof, mu, "hound gpu records")
    np.testing.assert_array_equal(inline[1], records[1])
    np.testing.assert_allclose(inline[0], records[0], rtol=0, atol=1e-6)
