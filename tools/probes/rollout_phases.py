"""Rollout phase probe (PPO on AnymalTerrain 4096): time each phase of a horizon step in isolation,
back-to-back replays without host syncs in between (GPU-bound timing), after one warm-up epoch.
    python tools/probes/rollout_phases.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import isaacgymenvs  # noqa: E402
from isaacgymenv_amd.isaacgymenvs.config import compose  # noqa: E402
from isaacgymenv_amd.rl import A2CAgent, PpoConfig  # noqa: E402

env = isaacgymenvs.make(seed=42, task="AnymalTerrain", num_envs=4096, sim_device="cuda:0", rl_device="cuda:0",
                        headless=True, force_render=False)
pcfg = PpoConfig.from_train_cfg(compose("config", ["task=AnymalTerrain"])["train"])
agent = A2CAgent(env, pcfg, device="cuda:0", seed=42)
agent.env_reset()
agent.train_epoch()
agent.train_epoch()
R = 200


def t(fn, reps=R):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / reps


obs = agent.obs
res = agent.get_action_values(obs)
act = res["actions"].clone()
out = {
    "act_graph_ms": t(lambda: agent.get_action_values(obs)),
    "pre_graph_ms": t(lambda: agent._step_graphs[0][0].replay()),
    "post_ms": t(lambda: agent._store_post_fused(0, res, env.rew_buf, env.reset_buf, env.timeout_buf)),
    "env_step_ms": t(lambda: env.step(act)),
    "play_steps_ms_per_step": t(agent.play_steps, 10) / agent.horizon,
}
# host-side cost of env.step: time with the GPU idle beforehand
torch.cuda.synchronize()
t0 = time.perf_counter()
env.step(act)
out["env_step_host_return_ms"] = 1e3 * (time.perf_counter() - t0)
torch.cuda.synchronize()
print(out, flush=True)
