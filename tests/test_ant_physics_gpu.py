"""Ant physics on the GPU (one-env-per-lane kernel, Topo_nv_ant) vs the fp64 oracle.

Covers what the Ant row adds to the solver: the MJCF model (capsule/sphere candidates, geom
masses), joint-limit rows (states start up to 0.05 rad beyond the limits) and force sensors on
the four feet.  Tolerances as for ANYmal; the sensor tolerance is 1 % of
the robot's weight (0.09 N) + 2 %.
"""
import numpy as np
import pytest
import torch

from oracle.oracle import OracleSim
from tests import helpers as H

pytestmark = pytest.mark.gpu


def _gpu(n, root, dof, tau, mu, steps=1):
    gym, sim = H.make_gpu_sim("ant", n, H.ANT_PARAMS)
    assert sim.kernel_variant == 1 and sim.num_sensors == 4
    H.load_state_into(sim, root, dof, mu)
    for _ in range(steps):
        sim.dof_force.copy_(torch.from_numpy(tau.astype(np.float32).reshape(-1)))
        gym.simulate(sim)
    torch.cuda.synchronize()
    g_root, g_dof = H.read_state(sim, 8)
    g_sens = sim.sens_soa.cpu().numpy().astype(np.float64).T.reshape(n, 4, 6)
    gym.refresh_force_sensor_tensor(sim)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(sim.sensor_tensor.cpu().numpy().reshape(n, 4, 6), g_sens.astype(np.float32))
    return g_root, g_dof, g_sens


def _oracle(flat, root, dof, tau, mu, steps=1):
    sim = OracleSim(flat, H.ANT_PARAMS, sensor_bodies=H.ANT_FEET)
    r, d = root.copy(), dof.copy()
    sens = np.zeros((root.shape[0], 4, 6))
    for _ in range(steps):
        sim.simulate(r, d, np.ascontiguousarray(tau), mu, sens=sens)
    return r, d, sens


def test_ant_one_simulate_matches_oracle():
    n = 512
    art, flat = H.ant()
    root, dof, tau, mu = H.ant_states(n, seed=3)
    g_root, g_dof, g_sens = _gpu(n, root, dof, tau, mu)
    o_root, o_dof, o_sens = _oracle(flat, root, dof, tau, mu)
    assert np.all(np.isfinite(g_root)) and np.all(np.isfinite(g_dof)) and np.all(np.isfinite(g_sens))

    def rerun(idx, rng, bits):
        r, d = H.perturbed(root, dof, idx, rng)
        o_r, o_d, _, o_s = H.oracle_run(flat, H.ANT_PARAMS, r, d, tau[idx], mu[idx], bits, nsens=4,
                                        sensor_bodies=H.ANT_FEET)
        return H.state_fields(o_r, o_d, sens=o_s)
    H.assert_close_or_explained(H.state_fields(g_root, g_dof, sens=g_sens), H.state_fields(o_root, o_dof, sens=o_sens),
                                rerun, what="ant gpu")


def test_ant_limits_hold_on_gpu():
    """Full torque into the limits for 1 s: every joint stays within 0.02 of its range."""
    n = 256
    art, flat = H.ant()
    root = np.zeros((n, 13)); root[:, 2] = 0.44; root[:, 6] = 1.0
    dof = np.zeros((n, 8, 2)); dof[:, :, 0] = np.clip(0.0, flat["lower"], flat["upper"])
    rng = np.random.RandomState(0)
    tau = 15.0 * np.sign(rng.uniform(-1, 1, (n, 8)))
    mu = np.full((n, flat["ns"]), 1.5)
    g_root, g_dof, g_sens = _gpu(n, root, dof, tau, mu, steps=60)
    q = g_dof[:, :, 0]
    assert np.all(q >= flat["lower"] - 0.02) and np.all(q <= flat["upper"] + 0.02), (q.min(0), q.max(0))
    assert np.all(np.isfinite(g_sens))


def test_ant_rest_rollout_tracks_oracle():
    """Zero torque for 1 s from the reference's start pose: the GPU trajectory and the foot
    sensors follow the oracle's."""
    n = 32
    art, flat = H.ant()
    root = np.zeros((n, 13)); root[:, 2] = 0.44; root[:, 6] = 1.0
    dof = np.zeros((n, 8, 2)); dof[:, :, 0] = np.clip(0.0, flat["lower"], flat["upper"])
    tau = np.zeros((n, 8))
    mu = np.full((n, flat["ns"]), 1.5)
    g_root, g_dof, g_sens = _gpu(n, root, dof, tau, mu, steps=60)
    o_root, o_dof, o_sens = _oracle(flat, root, dof, tau, mu, steps=60)
    np.testing.assert_allclose(g_root[:, 0:3], o_root[:, 0:3], atol=2e-3)
    np.testing.assert_allclose(g_dof[:, :, 0], o_dof[:, :, 0], atol=2e-3)
    np.testing.assert_allclose(g_sens, o_sens, atol=0.05, rtol=2e-2)
