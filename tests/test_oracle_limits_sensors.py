"""Oracle known answers for joint limits and force sensors -- CPU only.

* a joint driven hard into its limit stays there (within the speculative margin's reach);
* far from its limits a joint moves exactly as without limits;
* at rest on the ground, every foot sensor reads the joint reaction m_foot*g*z - F_contact
  (Newton-Euler of the foot), expressed in the foot frame.
"""
import numpy as np
import pytest

from tests import helpers as H

pytest.importorskip("numpy")


def _oracle(flat, params, sensors=()):
    from oracle.oracle import OracleSim
    return OracleSim(flat, params, sensor_bodies=sensors)


def _ant_standing(n=1):
    art, flat = H.ant()
    root = np.zeros((n, 13)); root[:, 2] = 0.44; root[:, 6] = 1.0
    lo, hi = flat["lower"], flat["upper"]
    dof = np.zeros((n, 8, 2)); dof[:, :, 0] = np.clip(0.0, lo, hi)  # ant.py:100-102
    return art, flat, root, dof


def test_joint_limit_holds_under_full_torque():
    art, flat, root, dof = _ant_standing()
    p = dict(H.ANT_PARAMS, has_ground=0, gravity=[0.0, 0.0, 0.0])
    sim = _oracle(flat, p)
    tau = np.zeros((1, 8)); tau[0, 0] = 15.0; tau[0, 1] = -15.0  # hip_1 up, ankle_1 down
    mu = np.full((1, flat["ns"]), 1.5)
    for _ in range(120):
        sim.simulate(root, dof, tau, mu)
    assert dof[0, 0, 0] <= flat["upper"][0] + 0.02, dof[0, 0, 0]
    assert dof[0, 1, 0] >= flat["lower"][1] - 0.02, dof[0, 1, 0]
    assert abs(dof[0, 0, 0] - flat["upper"][0]) < 0.05 and abs(dof[0, 1, 0] - flat["lower"][1]) < 0.05


def test_limits_do_not_act_away_from_the_limits():
    art, flat, root, dof = _ant_standing()
    dof[0, :, 0] = 0.5 * (flat["lower"] + flat["upper"])
    p = dict(H.ANT_PARAMS, has_ground=0, gravity=[0.0, 0.0, 0.0])
    tau = np.full((1, 8), 0.01)
    mu = np.full((1, flat["ns"]), 1.5)
    a = _oracle(flat, p)
    flat_nolim = dict(flat, has_limits=np.zeros_like(flat["has_limits"]))
    b = _oracle(flat_nolim, p)
    ra, da, rb, db = root.copy(), dof.copy(), root.copy(), dof.copy()
    for _ in range(5):
        a.simulate(ra, da, tau, mu)
        b.simulate(rb, db, tau, mu)
    np.testing.assert_array_equal(da, db)
    np.testing.assert_array_equal(ra, rb)


def test_foot_sensors_read_the_joint_reaction_at_rest():
    art, flat, root, dof = _ant_standing()
    p = dict(H.ANT_PARAMS, collect_contacts=1)
    sim = _oracle(flat, p, sensors=H.ANT_FEET)
    tau = np.zeros((1, 8))
    mu = np.full((1, flat["ns"]), 1.5)
    cf = np.zeros((1, flat["nb"], 3))
    sens = np.zeros((1, 4, 6))
    for _ in range(240):  # 4 s: settle
        sim.simulate(root, dof, tau, mu, cf=cf, sens=sens)
    # at rest up to the solver's slow frictional yaw creep (4 position iterations, no velocity pass)
    assert np.abs(root[0, 7:12]).max() < 1e-2 and abs(root[0, 12]) < 0.1, root[0, 7:13]
    g = 9.81
    total = sum(flat["mass"])
    assert abs(cf[0, :, 2].sum() - total * g) < 0.02 * total * g  # the ground carries the Ant
    from isaacgymenv_amd.isaacgym._assets import quat_xyzw_to_mat
    for si, b in enumerate(H.ANT_FEET):
        # foot orientation in the world: root rotation x joint chain (oracle kinematics, float64)
        Rw = _body_rotation(flat, root[0], dof[0], b)
        f_world = Rw @ sens[0, si, :3]
        expect = np.array([0.0, 0.0, flat["mass"][b] * g]) - cf[0, b]
        np.testing.assert_allclose(f_world, expect, atol=0.02 * total * g)


def _body_rotation(flat, root, dof, b):
    from isaacgymenv_amd.isaacgym._assets import quat_xyzw_to_mat
    import math
    chain = []
    x = b
    while x > 0:
        chain.append(x)
        x = int(flat["parent"][x])
    R = quat_xyzw_to_mat(root[3:7])
    for i in reversed(chain):
        Ro = np.array(flat["jorigin"][i][:9]).reshape(3, 3)
        a = np.array(flat["jaxis"][i])
        q = dof[int(flat["bdof"][i]), 0]
        c, s = math.cos(q), math.sin(q)
        K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
        Rq = np.eye(3) + s * K + (1 - c) * K @ K
        R = R @ Ro @ Rq
    return R
