"""Known-answer checks of the CPU oracle -- pins the solver spec
the HIP kernel is compared against, since PhysX itself is unavailable (parity vs PhysX: unpinned)."""
import numpy as np

from oracle.oracle import OracleSim
from tests import helpers as H


def _stand(n=2, pos_iters=4):
    art, flat = H.anymal()
    q0 = np.array([H.ANYMAL_DEFAULT[d] for d in art.dof_names()])
    root = np.zeros((n, 13)); root[:, 2] = 0.62; root[:, 6] = 1.0
    dof = np.zeros((n, 12, 2)); dof[:, :, 0] = q0
    return art, flat, q0, root, dof


def test_free_fall_semi_implicit_euler():
    art, flat, q0, root, dof = _stand(1)
    root[:, 2] = 10.0
    sim = OracleSim(flat, dict(H.ANYMAL_PARAMS, has_ground=0))
    h, n = 0.005, 100
    for _ in range(n):
        sim.simulate(root, dof, np.zeros((1, 12)), np.ones((1, flat["ns"])))
    # semi-implicit Euler: z_n = z0 - g h^2 n(n+1)/2, v_n = -g h n; joints stay put (no gravity torque
    # difference in free fall)
    np.testing.assert_allclose(root[0, 2], 10.0 - 9.81 * h * h * n * (n + 1) / 2, atol=1e-9)
    np.testing.assert_allclose(root[0, 9], -9.81 * h * n, atol=1e-9)
    np.testing.assert_allclose(dof[0, :, 0], q0, atol=1e-9)


def test_standing_contact_forces_carry_the_weight():
    art, flat, q0, root, dof = _stand(1)
    sim = OracleSim(flat, H.ANYMAL_PARAMS)
    mu = np.ones((1, flat["ns"]))
    cf = np.zeros((1, flat["nb"], 3))
    for _ in range(1000):
        tau = np.clip(80 * (q0 - dof[:, :, 0]) - 2 * dof[:, :, 1], -80, 80)
        sim.simulate(root, dof, np.ascontiguousarray(tau), mu, cf)
    weight = sum(b.mass for b in art.bodies) * 9.81
    # after 5 s the base still creeps down slowly (friction not converged in 4+1 iterations), so the
    # support force equals the weight to within the residual vertical deceleration
    np.testing.assert_allclose(cf[0, :, 2].sum(), weight, rtol=1e-2)
    assert np.all(cf[0, [3, 6, 9, 12], 2] > 50)      # the four feet carry it
    assert np.all(cf[0, [0, 2, 5, 8, 11], :] == 0)   # no base / knee contact
    assert 0.45 < root[0, 2] < 0.55


def test_pendulum_small_angle_period():
    """Cartpole pole as a pendulum (cart force 0, cart mass 1, pole mass 1 at 0.47 m): for a
    prismatic-cart pendulum, omega^2 = g (m_c + m_p) / (m_c l) with l the COM distance."""
    art, flat = H.cartpole()
    p = dict(H.CARTPOLE_PARAMS, dt=0.001, substeps=1, has_ground=0)
    sim = OracleSim(flat, p)
    root = np.zeros((1, 13)); root[:, 2] = 2.0; root[:, 6] = 1.0
    dof = np.zeros((1, 2, 2)); dof[0, 1, 0] = np.pi - 0.02  # hanging down (pole along +z at q=0)
    qs = []
    for _ in range(6000):
        sim.simulate(root, dof, np.zeros((1, 2)), np.ones((1, flat["ns"])))
        qs.append(dof[0, 1, 0] - np.pi)
    qs = np.array(qs)
    crossings = np.where(np.diff(np.sign(qs)) != 0)[0]
    period = 2 * np.mean(np.diff(crossings)) * 1e-3
    pole = art.bodies[2]
    l = abs(pole.com[2])
    I = pole.inertia[0, 0]
    mc, mp = art.bodies[1].mass, pole.mass
    # exact linearised cart-pendulum: omega^2 = mp g l (mc+mp) / ((mc+mp)(I + mp l^2) - mp^2 l^2)
    w2 = mp * 9.81 * l * (mc + mp) / ((mc + mp) * (I + mp * l * l) - (mp * l) ** 2)
    np.testing.assert_allclose(period, 2 * np.pi / np.sqrt(w2), rtol=5e-3)


def test_unactuated_spinning_chain_stays_bounded():
    """No ground, no torque, zero gravity: a spinning ANYmal stays finite and bounded."""
    art, flat, q0, root, dof = _stand(1)
    root[0, 10:13] = [0.5, -0.3, 0.8]
    dof[0, :, 1] = np.linspace(-1, 1, 12)
    p = dict(H.ANYMAL_PARAMS, gravity=[0.0, 0.0, 0.0], has_ground=0, dt=0.001)
    sim = OracleSim(flat, p)

    for i in range(500):
        sim.simulate(root, dof, np.zeros((1, 12)), np.ones((1, flat["ns"])))
    assert np.all(np.isfinite(root)) and np.all(np.isfinite(dof))
    assert np.abs(dof[0, :, 1]).max() < 20.0


def test_fp32_build_agrees_with_fp64():
    art, flat = H.anymal()
    root, dof, tau, mu = H.anymal_states(32, seed=9)
    a = OracleSim(flat, H.ANYMAL_PARAMS, 64)
    b = OracleSim(flat, H.ANYMAL_PARAMS, 32)
    r64, d64 = root.copy(), dof.copy()
    r32, d32 = root.astype(np.float32), dof.astype(np.float32)
    a.simulate(r64, d64, np.ascontiguousarray(tau), mu)
    b.simulate(r32, d32, np.ascontiguousarray(tau, dtype=np.float32), mu.astype(np.float32))
    np.testing.assert_allclose(r32[:, :7], r64[:, :7], atol=2e-5)
    np.testing.assert_allclose(d32[:, :, 1], d64[:, :, 1], atol=5e-3, rtol=5e-3)


def _heavy_rest(run_sim, steps=200):
    """ANYmal on its back with a 27.8 t base (J M^-1 J^T of the base's ground rows ~2e-4, below the 1e-3
    self-contact response cutoff): 1 s of zero torque -- the base capsule rests on the plane, it does not fall
    through it.  Returns the final base heights."""
    n = 8
    root, dof = H.upside_down_anymal(n)
    root[:, 0] = np.arange(n) * 2.0
    z = run_sim(root, dof, steps)
    assert np.all(np.isfinite(z))
    return z


def test_heavy_body_rests_on_the_plane():
    """Known answer: ground and terrain contact rows take no response cutoff, in the oracle and in
    the host backend (the same solver source as the HIP kernels)."""
    art, flat = H.anymal()
    H.heavy_base(flat)
    mu = np.ones((8, flat["ns"]))

    def oracle(root, dof, steps):
        sim = OracleSim(flat, H.ANYMAL_PARAMS)
        for _ in range(steps):
            sim.simulate(root, dof, np.zeros((root.shape[0], 12)), mu)
        return root[:, 2]

    def host(root, dof, steps):
        import torch
        gym, sim = H.make_host_sim("anymal", root.shape[0], H.ANYMAL_PARAMS, asset_hook=lambda a: H.heavy_base(a.flat))
        H.load_state_into(sim, root, dof, mu)
        sim.dof_force.zero_()
        for _ in range(steps):
            gym.simulate(sim)
        return H.read_state(sim, 12)[0][:, 2]

    for run in (oracle, host):
        z = _heavy_rest(run)
        # resting on the capsule (radius 0.1): penetration bounded by the solver's push-out, a few mm
        assert np.all(z > 0.09) and np.all(z < 0.11), (run.__name__, z)
