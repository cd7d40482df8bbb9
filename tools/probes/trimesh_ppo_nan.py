"""Probe: where do non-finite values first appear on the trimesh AnymalTerrain config (env state,
observations, PPO statistics)?  python tools/probes/trimesh_ppo_nan.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import isaacgymenvs
    from isaacgymenv_amd.isaacgymenvs.config import compose
    from isaacgymenv_amd.rl import A2CAgent, PpoConfig
    dev = "cuda:0"
    env = isaacgymenvs.make(seed=42, task="AnymalTerrain", num_envs=4096, sim_device=dev, rl_device=dev,
                            graphics_device_id=-1, headless=True, force_render=False,
                            overrides=["task.env.terrain.terrainType=trimesh"])
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    for t in range(300):
        a = torch.empty((env.num_envs, env.num_actions), device=dev).uniform_(-1, 1, generator=g)
        obs, rew, done, _ = env.step(a)
        o = obs["obs"]
        bad_o = ~torch.isfinite(o).all(dim=1)
        bad_r = ~torch.isfinite(env.root_states).all(dim=1)
        bad_d = ~torch.isfinite(env.dof_state.view(env.num_envs, -1)).all(dim=1)
        big = o.abs().max().item()
        if bad_o.any() or bad_r.any() or bad_d.any() or t % 50 == 0:
            print(f"step {t}: nonfinite obs {int(bad_o.sum())} root {int(bad_r.sum())} dof {int(bad_d.sum())} "
                  f"max|obs| {big:.3g} max|rew| {rew.abs().max().item():.3g}", flush=True)
            if bad_o.any() or bad_r.any() or bad_d.any():
                e = int(torch.nonzero(bad_o | bad_r | bad_d)[0])
                print("env", e, "root", env.root_states[e].tolist(), flush=True)
                print("obs cols nonfinite", torch.nonzero(~torch.isfinite(o[e])).flatten().tolist()[:20], flush=True)
                break
    train = compose("config", ["task=AnymalTerrain"])["train"]
    agent = A2CAgent(env, PpoConfig.from_train_cfg(train), device=dev, seed=42)
    agent.env_reset()
    for ep in range(4):
        agent.train_epoch()
        print("epoch", ep, agent.epoch_stats(), flush=True)


if __name__ == "__main__":
    main()
