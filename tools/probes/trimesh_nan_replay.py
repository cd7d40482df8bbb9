"""Replay a captured trimesh blow-up step (tools/probes/trimesh_nan_capture.py) on the CPU: the host
backend (libgymsim's solver source on host threads) and the fp64 oracle, substep by substep.

    python tools/probes/trimesh_nan_replay.py gpurun_out/r02r/nan_case.npz
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import helpers as H
    from oracle.oracle import OracleSim
    d = np.load(sys.argv[1])
    np.set_printoptions(precision=4, suppress=True, linewidth=200)
    ox, oy = (float(v) for v in d["patch_origin"])
    ter = H.terrain_from_heights(d["hpatch"], hs=float(d["hs"]), vs=float(d["vs"]),
                                 slope_threshold=float(d["slope_threshold"]), shift=(ox, oy, 0.0),
                                 friction=float(d["terrain_mu"]))
    params = dict(dt=float(d["dt"]), substeps=int(d["substeps"]), gravity=[0.0, 0.0, -9.81],
                  pos_iters=int(d["pos_iters"]), vel_iters=int(d["vel_iters"]),
                  contact_offset=float(d["contact_offset"]), rest_offset=float(d["rest_offset"]),
                  max_depen_vel=float(d["max_depen"]), collect_contacts=1, has_ground=0)
    gym, sim = H.make_host_sim("anymal", 1, params, terrain=ter, threads=1)
    from isaacgymenv_amd.isaacgym import gymtorch
    root_t = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    dof_t = gymtorch.wrap_tensor(gym.acquire_dof_state_tensor(sim))
    root_t.copy_(torch.from_numpy(d["root"]).view(1, 13))
    gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root_t))
    dof_t.copy_(torch.from_numpy(d["dof_true"]).view(-1, 2))
    gym.set_dof_state_tensor(sim, gymtorch.unwrap_tensor(dof_t))
    sim.shape_mu.copy_(torch.from_numpy(d["shape_mu"]).view(-1, 1))
    internal0 = sim.state.clone()
    a = torch.from_numpy(d["actions"])
    dflt = torch.from_numpy(d["default_dof_pos"])
    kp, kd, sc = float(d["kp"]), float(d["kd"]), float(d["action_scale"])
    dof_for_pd = torch.from_numpy(d["dof_stale"]).clone()
    taus = []
    print("pre  root", d["root"])
    for it in range(int(d["decimation"]) + 1):
        if it < int(d["decimation"]):
            q, qd = dof_for_pd[:, 0], dof_for_pd[:, 1]
            tau = torch.clamp(kp * (sc * a + dflt - q) - kd * qd, -80.0, 80.0)
        taus.append(tau.clone())
        sim.dof_force.copy_(tau.reshape(-1))
        gym.simulate(sim)
        gym.refresh_dof_state_tensor(sim)
        gym.refresh_actor_root_state_tensor(sim)
        dof_for_pd = dof_t.view(12, 2).clone()
        print(f"host substep {it}: root", root_t[0].numpy())
    print("GPU  after", d["root_after"])
    # the fp64 oracle from the same internal state, same torques
    art, flat = H.anymal()
    osim = OracleSim(flat, params, terrain=ter["oracle"])
    st = internal0.cpu().numpy().astype(np.float64)
    r = st[0:13].T.copy()
    q = np.stack([st[13:25].T, st[25:37].T], axis=-1)
    mu = np.asarray(d["shape_mu"], dtype=np.float64).reshape(1, -1)
    cf = np.zeros((1, flat["nb"], 3))
    from oracle import kinematics_oracle as ko
    for it, tau in enumerate(taus):
        # candidates touching the mesh before this substep: separation, normal
        R, pb, _, _ = ko.fk(flat, r[0], q[0, :, 0])
        cen = np.array([pb[b] + R[b] @ flat["cpoint"][c] for c, b in enumerate(flat["cbody"])])
        rad = np.asarray(flat["cradius"], dtype=np.float64)
        tq = osim.terrain_query(cen, rad)
        act = np.nonzero((tq[:, 0] > 0) & (tq[:, 1] < params["contact_offset"]))[0]
        print(f"  before substep {it}: active", [(int(c), round(float(tq[c, 1]), 4), np.round(tq[c, 2:], 3).tolist())
                                             for c in act])
        osim.simulate(r, q, np.ascontiguousarray(tau.numpy().astype(np.float64).reshape(1, -1)), mu, cf)
        print("  contact force per body", np.round(cf[0][np.abs(cf[0]).sum(1) > 0], 1).tolist())
        print(f"oracle substep {it}: root(internal) p {r[0, :3]} w {r[0, 10:13]} vo {r[0, 7:10]}")


if __name__ == "__main__":
    main()
