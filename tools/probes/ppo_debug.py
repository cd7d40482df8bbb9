"""GPU learning-curve probe with diagnostics: python tools/ppo_debug.py <Task> <envs> <epochs> <variant>

variant: graphs | eager | plain (eager, non-fused Adam with a host float lr)
Prints per epoch: lr, kl, losses, mean episode length, sigma, |obs| max, nan flags, grad norm."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from isaacgymenv_amd.isaacgymenvs.config import compose  # noqa: E402
from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task  # noqa: E402
from isaacgymenv_amd.rl import A2CAgent, PpoConfig  # noqa: E402
import isaacgymenvs  # noqa: E402

task, N, epochs, variant = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
vec_task.EXISTING_SIM = None
cfg = compose("config", [f"task={task}"])
env = isaacgymenvs.make(seed=42, task=task, num_envs=N, sim_device="cuda:0", rl_device="cuda:0",
                        headless=True, force_render=False)
agent = A2CAgent(env, PpoConfig.from_train_cfg(cfg["train"]), device="cuda:0", seed=42,
                 use_graphs=(variant == "graphs"))
if os.environ.get("PATCH_CLIP"):
    import isaacgymenv_amd.rl.a2c_continuous as M

    def _clip(params, max_norm):
        g = agent.flat_grad
        coef = torch.clamp(max_norm / (torch.linalg.vector_norm(g) + 1e-6), max=1.0)
        g.mul_(coef)
    M.nn.utils.clip_grad_norm_ = _clip
if variant == "plain":
    agent._opt_lr = None
    agent.optimizer = torch.optim.Adam(agent.params, lr=agent.cfg.learning_rate, eps=1e-8)
for ep in range(epochs):
    agent.train_epoch()
    s = agent.epoch_stats()
    o = agent.b_obs
    sig = agent.model.a2c_network.sigma.detach()
    print(f"{variant} ep {ep + 1} lr {s['lr']:.2e} kl {s['kl']:.4f} a {s['a_loss']:.4f} c {s['c_loss']:.4f} "
          f"len {s['mean_length']:.1f} rew {s['mean_reward']:.2f} sigma {sig.mean().item():.3f} "
          f"obsmax {o.abs().max().item():.3g} obsnan {bool(torch.isnan(o).any())} "
          f"gnorm {agent.flat_grad.norm().item():.3g} pnan {any(bool(torch.isnan(p).any()) for p in agent.params)} "
          f"rms_mean {agent.model.running_mean_std.running_mean.abs().max().item():.3g} "
          f"rms_var {agent.model.running_mean_std.running_var.max().item():.3g}", flush=True)

if len(sys.argv) > 5:  # deep graph probe: grads per replay
    fg0, fg1 = agent.flat_grad.data_ptr(), agent.flat_grad.data_ptr() + agent.flat_grad.numel() * 4
    orig = agent._run_minibatch

    def run(i):
        orig(i)
        alias = all(p.grad is not None and fg0 <= p.grad.data_ptr() < fg1 for p in agent.params)
        print(f"  mb {i} epoch {agent.epoch_num} gnorm {agent.flat_grad.norm().item():.4g} alias {alias} "
              f"w0 {agent.params[0].detach().norm().item():.6g} c {agent._stats_acc[1].item():.4g}", flush=True)
    agent._run_minibatch = run
    for ep in range(3):
        agent.train_epoch()
