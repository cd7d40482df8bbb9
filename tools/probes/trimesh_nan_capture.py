"""Probe: capture the pre-step state of the first env whose root state turns non-finite on the trimesh
AnymalTerrain config (random actions), with the heightfield patch under it, for a CPU replay
(tools/probes/trimesh_nan_replay.py: host backend = the same solver source, and the fp64 oracle).

    python tools/probes/trimesh_nan_capture.py [out.npz]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


LIN_MAX = float(os.environ.get("LIN_MAX", "12"))
ANG_MAX = float(os.environ.get("ANG_MAX", "40"))


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/trimesh_nan_case.npz"
    for seed in range(1, 9):
        if capture(out, seed, 1000):
            return
    print("no non-finite state", flush=True)


def capture(out, seed, steps):
    import isaacgymenvs
    from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
    from isaacgymenv_amd.isaacgymenvs.utils.utils import set_seed
    vec_task.EXISTING_SIM = None
    set_seed(seed)
    dev = "cuda:0"
    env = isaacgymenvs.make(seed=seed, task="AnymalTerrain", num_envs=4096, sim_device=dev, rl_device=dev,
                            graphics_device_id=-1, headless=True, force_render=False,
                            overrides=["task.env.terrain.terrainType=trimesh"])
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    gym, sim = env.gym, env.sim
    print("seed", seed, flush=True)
    H = 40
    hist_root, hist_dof, hist_act = [], [], []
    for t in range(steps):
        a = torch.empty((env.num_envs, env.num_actions), device=dev).uniform_(-1, 1, generator=g)
        root0 = env.root_states.clone()
        stale = env.dof_state.clone()
        gym.refresh_dof_state_tensor(sim)  # the sim's true dof state (read only)
        true_dof = env.dof_state.clone()
        env.dof_state.copy_(stale)          # keep the task's stale tensor (first PD evaluation reads it)
        hist_root.append(root0)
        hist_dof.append(true_dof)
        hist_act.append(a)
        if len(hist_root) > H:
            hist_root.pop(0), hist_dof.pop(0), hist_act.pop(0)
        env.step(a)
        rs = env.root_states
        # the first sign of a blow-up: non-finite, or base speeds no gait reaches
        bad = ~torch.isfinite(rs).all(dim=1) | (rs[:, 7:10].norm(dim=1) > LIN_MAX) | (rs[:, 10:13].norm(dim=1) > ANG_MAX)
        if bad.any():
            e = int(torch.nonzero(bad)[0])
            nd = env.num_dof
            ter = env.terrain
            hs, vs = float(ter.horizontal_scale), float(ter.vertical_scale)
            border = float(ter.border_size)
            px, py = float(root0[e, 0]), float(root0[e, 1])
            # heightfield patch of +-3 m around the base (sample (i, j) sits at (i*hs - border, j*hs - border))
            hsamp = env.height_samples.cpu().numpy()
            ci, cj = int((px + border) / hs), int((py + border) / hs)
            w = int(3.0 / hs)
            i0, j0 = max(ci - w, 0), max(cj - w, 0)
            i1, j1 = min(ci + w, hsamp.shape[0]), min(cj + w, hsamp.shape[1])
            sp = env.sim_params
            np.savez(out, step=t, env=e, root=root0[e].cpu().numpy(), dof_true=true_dof.view(env.num_envs, nd, 2)[e]
                     .cpu().numpy(), dof_stale=stale.view(env.num_envs, nd, 2)[e].cpu().numpy(),
                     actions=a[e].cpu().numpy(), default_dof_pos=env.default_dof_pos[e].cpu().numpy(),
                     kp=env.Kp, kd=env.Kd, action_scale=env.action_scale, decimation=env.decimation,
                     hpatch=hsamp[i0:i1, j0:j1], patch_origin=np.array([i0 * hs - border, j0 * hs - border]),
                     hs=hs, vs=vs, slope_threshold=float(env.cfg["env"]["terrain"]["slopeTreshold"]),
                     dt=sp.dt, substeps=sp.substeps, pos_iters=sp.physx.num_position_iterations,
                     vel_iters=sp.physx.num_velocity_iterations, contact_offset=sp.physx.contact_offset,
                     rest_offset=sp.physx.rest_offset, max_depen=sp.physx.max_depenetration_velocity,
                     terrain_mu=float(env.cfg["env"]["terrain"]["staticFriction"]),
                     root_after=env.root_states[e].cpu().numpy(), shape_mu=sim.shape_mu[:, e].cpu().numpy(),
                     seed=seed, hist_root=torch.stack([x[e] for x in hist_root]).cpu().numpy(),
                     hist_dof=torch.stack([x.view(env.num_envs, nd, 2)[e] for x in hist_dof]).cpu().numpy(),
                     hist_act=torch.stack([x[e] for x in hist_act]).cpu().numpy())
            print(f"non-finite root: seed {seed} env {e} at step {t}; saved {out}", flush=True)
            return True
    del env
    torch.cuda.empty_cache()
    return False


if __name__ == "__main__":
    main()
