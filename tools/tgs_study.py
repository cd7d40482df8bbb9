"""PGS vs TGS on the fp64 oracle.

The reference configs ask PhysX for TGS (`solver_type: 1`, cfg/config.yaml:31); the MI355X kernels run PGS
with split impulse.  The oracle (oracle/physics_oracle.c) has both: solver_type 0 is the kernels' PGS, 1 (and 2: the
joint velocity limit applied in every position sub-step, round 5) is
TGS restated -- num_position_iterations sub-steps of h / n, each row's separation advanced by the displacement
integrated so far (linearised, J dq), positions integrated with the sub-steps' velocities, no bias in the
velocity iterations.  This script runs AnymalTerrain's physics (plane, the task's PD at 4 x decimation + 1
simulate per env step, dt 0.005, 4 position / 1 velocity iterations) in both and reports:

  * standing: zero actions from the task's start pose -- settled base height, foot penetration, drift;
  * locomotion: uniform random actions -- base height / speed statistics, penetration, and how far the
    PGS and TGS trajectories separate compared with PGS against itself from a 1e-7 perturbed start
    (the chaos floor: a contact-rich rollout separates from any perturbation).

    python tools/tgs_study.py [--envs 64] [--steps 80] [--out profiles/r03_tgs_study.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.oracle import OracleSim  # noqa: E402
from oracle.kinematics_oracle import fk  # noqa: E402
from tests import helpers as H  # noqa: E402

DEFAULT = {"LF_HAA": 0.03, "LF_HFE": 0.4, "LF_KFE": -0.8, "LH_HAA": 0.03, "LH_HFE": -0.4, "LH_KFE": 0.8,
           "RF_HAA": -0.03, "RF_HFE": 0.4, "RF_KFE": -0.8, "RH_HAA": -0.03, "RH_HFE": -0.4, "RH_KFE": 0.8}
KP, KD, SCALE, TLIM, DECIMATION = 80.0, 2.0, 0.5, 80.0, 4  # AnymalTerrain.yaml control block


def start_states(art, flat, n, seed):
    rng = np.random.RandomState(seed)
    names = art.dof_names()
    default = np.array([DEFAULT[nm] for nm in names])
    root = np.zeros((n, 13))
    root[:, 2] = 0.62  # AnymalTerrain.yaml baseInitState pos
    root[:, 6] = 1.0
    dof = np.zeros((n, 12, 2))
    dof[:, :, 0] = default + rng.uniform(-0.05, 0.05, (n, 12))
    mu = np.ones((n, flat["ns"]))
    return root, dof, mu, default


def penetration(flat, root, dof):
    """Deepest ground overlap of any collision sphere / capsule end (m, positive = inside the ground)."""
    worst = 0.0
    for e in range(root.shape[0]):
        R, p, _, _ = fk(flat, root[e], dof[e, :, 0])
        for c in range(flat["nc"]):
            b = flat["cbody"][c]
            x = R[b] @ flat["cpoint"][c] + p[b]
            worst = max(worst, -(x[2] - flat["cradius"][c]))
    return worst


def rollout(flat, params, root, dof, mu, default, actions, threads):
    sim = OracleSim(flat, params)
    r, d = root.copy(), dof.copy()
    n = r.shape[0]
    cf = np.zeros((n, flat["nb"], 3))
    traj, pen, fz = [], [], []
    q, qd = d[:, :, 0].copy(), d[:, :, 1].copy()
    for t in range(actions.shape[0]):
        for i in range(DECIMATION + 1):
            if i < DECIMATION:
                tau = np.clip(KP * (SCALE * actions[t] + default - q) - KD * qd, -TLIM, TLIM)
            sim.simulate(r, d, np.ascontiguousarray(tau), mu, cf, num_threads=threads)
            if i == DECIMATION - 1:
                q, qd = d[:, :, 0].copy(), d[:, :, 1].copy()
        traj.append(r[:, :7].copy())
        fz.append(float(np.abs(cf[:, :, 2]).sum(axis=1).mean()))
        if t % 10 == 9 or t == actions.shape[0] - 1:
            pen.append(penetration(flat, r[:8], d[:8]))
    return np.stack(traj), dict(final_root=r, pen_max=float(max(pen)), contact_fz_mean=float(np.mean(fz)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=80)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=None)
    ap.add_argument("--self-collide", type=int, default=1, help="0: ANYmal's self-collision pairs off")
    ap.add_argument("--no-velocity-limit", action="store_true",
                    help="drop the URDF joint velocity limit (20 rad/s): the round-4 diagnosis of the TGS divergence")
    a = ap.parse_args()
    art, flat = H.anymal()
    flat["self_collide"] = a.self_collide
    if a.no_velocity_limit:
        flat["vmax"] = np.zeros_like(np.asarray(flat["vmax"], dtype=np.float64))  # <= 0: unlimited
    base = dict(H.ANYMAL_PARAMS)
    out = {"config": dict(envs=a.envs, env_steps=a.steps, dt=base["dt"], pos_iters=base["pos_iters"],
                          vel_iters=base["vel_iters"], decimation=DECIMATION, self_collide=int(flat["self_collide"]),
                          joint_velocity_limit=not a.no_velocity_limit)}
    t0 = time.time()
    for scen in ("standing", "locomotion"):
        root, dof, mu, default = start_states(art, flat, a.envs, seed=3)
        rng = np.random.RandomState(7)
        acts = np.zeros((a.steps, a.envs, 12)) if scen == "standing" else rng.uniform(-1, 1, (a.steps, a.envs, 12))
        res = {}
        trajs = {}
        for name, st in (("pgs", 0), ("tgs", 1), ("tgs_substep_vlimit", 2), ("tgs_step_pushout", 3)):
            p = dict(base, solver_type=st)
            traj, info = rollout(flat, p, root, dof, mu, default, acts, a.threads)
            trajs[name] = traj
            z = traj[:, :, 2]
            finite = np.isfinite(traj).all(axis=(0, 2))
            res[name] = dict(envs_finite=int(finite.sum()), base_z_final_mean=float(z[-1].mean()), base_z_final_std=float(z[-1].std()),
                             base_z_min=float(z.min()), pen_max_m=info["pen_max"],
                             contact_fz_mean_N=info["contact_fz_mean"],
                             base_xy_travel_mean_m=float(np.linalg.norm(traj[-1, :, :2] - traj[0, :, :2], axis=1).mean()))
        # chaos floor: PGS from a start perturbed at 1e-7
        pr = root.copy()
        pr[:, :3] += np.random.RandomState(1).normal(0, 1e-7, (a.envs, 3))
        traj_p, _ = rollout(flat, dict(base, solver_type=0), pr, dof, mu, default, acts, a.threads)
        sep = lambda x, y: np.linalg.norm(x[:, :, :3] - y[:, :, :3], axis=2).mean(axis=1)  # noqa: E731
        d_solver = sep(trajs["pgs"], trajs["tgs"])
        d_solver2 = sep(trajs["pgs"], trajs["tgs_substep_vlimit"])
        d_solver3 = sep(trajs["pgs"], trajs["tgs_step_pushout"])
        d_chaos = sep(trajs["pgs"], traj_p)
        marks = sorted(k for k in {0, 4, 19, a.steps // 2, a.steps - 1} if k < a.steps)
        res["pgs_vs_tgs_base_pos_sep_m"] = {str(k + 1): float(d_solver[k]) for k in marks}
        res["pgs_vs_tgs_substep_vlimit_base_pos_sep_m"] = {str(k + 1): float(d_solver2[k]) for k in marks}
        res["pgs_vs_tgs_step_pushout_base_pos_sep_m"] = {str(k + 1): float(d_solver3[k]) for k in marks}
        res["pgs_vs_perturbed_pgs_sep_m"] = {str(k + 1): float(d_chaos[k]) for k in marks}
        out[scen] = res
        print(scen, json.dumps(res, indent=1))
    out["wall_s"] = time.time() - t0
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
