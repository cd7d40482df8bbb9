"""Training entry point (reference ``isaacgymenvs/train.py``): compose the task + train
configs with Hydra-style overrides, create the env through ``isaacgymenvs.make``, train with
the rl_games-compatible PPO learner (isaacgymenv_amd/rl).

    python -m isaacgymenvs.train task=AnymalTerrain headless=True [num_envs=4096] [max_iterations=N]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m isaacgymenvs.train task=AnymalTerrain multi_gpu=True headless=True

multi_gpu: one process per GPU (LOCAL_RANK -> cuda:k, rlgames_utils.py:53-127), seed + rank
(train.py:120-123 via set_seed), torch.distributed over RCCL ("nccl"); each rank steps its own
envs and the learner all-reduces gradients once per minibatch.
"""
from __future__ import annotations

import os
import sys
from typing import List, Optional

from .config import compose
from .utils.reformat import omegaconf_to_dict
from .utils.utils import set_seed


def preprocess_train_config(cfg: dict, config_dict: dict) -> dict:
    """train.py:52-83: rl_device into the train config; model_size_multiplier."""
    train_cfg = config_dict["params"]["config"]
    train_cfg["device"] = cfg["rl_device"]
    train_cfg["full_experiment_name"] = cfg.get("full_experiment_name")
    mlp = config_dict["params"]["network"].get("mlp", {})
    mult = mlp.get("model_size_multiplier", 1)
    if mult != 1:
        mlp["units"] = [u * mult for u in mlp["units"]]
    return config_dict


def launch(overrides: Optional[List[str]] = None, printer=print):
    """Returns (agent, last epoch stats)."""
    import torch
    import torch.distributed as dist

    import isaacgymenv_amd.isaacgymenvs as igenvs
    from isaacgymenv_amd.rl import A2CAgent, PpoConfig

    cfg = compose("config", overrides or [])
    if cfg.get("task") is None or cfg.get("train") is None:
        raise ValueError("task=<Name> must name a task with a cfg/train/<Name>PPO.yaml")
    multi_gpu = bool(cfg["multi_gpu"])
    rank, local_rank = int(os.getenv("RANK", "0")), int(os.getenv("LOCAL_RANK", "0"))
    if multi_gpu and not dist.is_initialized():
        world = int(os.getenv("WORLD_SIZE", "1"))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if torch.cuda.is_available():
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    seed = set_seed(cfg["seed"], torch_deterministic=cfg["torch_deterministic"], rank=rank)
    rl_device = f"cuda:{local_rank}" if multi_gpu and torch.cuda.is_available() else cfg["rl_device"]
    sim_device = f"cuda:{local_rank}" if multi_gpu and torch.cuda.is_available() else cfg["sim_device"]
    cfg["rl_device"], cfg["sim_device"] = rl_device, sim_device
    task_cfg = omegaconf_to_dict(cfg["task"])
    if cfg.get("num_envs") not in ("", None):
        task_cfg["env"]["numEnvs"] = int(cfg["num_envs"])
    env = igenvs.make(seed, cfg["task_name"], task_cfg["env"]["numEnvs"], sim_device, rl_device,
                      cfg["graphics_device_id"], cfg["headless"], False, False, cfg["force_render"],
                      cfg={"task": task_cfg})
    train_cfg = preprocess_train_config(cfg, omegaconf_to_dict(cfg["train"]))
    over = {"multi_gpu": multi_gpu}
    if cfg.get("max_iterations") not in ("", None):
        over["max_epochs"] = int(cfg["max_iterations"])
    pcfg = PpoConfig.from_train_cfg(train_cfg, **over)
    agent = A2CAgent(env, pcfg, device=rl_device, seed=seed)
    if cfg.get("checkpoint"):
        agent.restore(cfg["checkpoint"])
    stats = agent.train(pcfg.max_epochs, printer=printer)
    if not cfg.get("test") and rank == 0:
        out = os.path.join("runs", pcfg.name, "nn", f"{pcfg.name}.pth")
        agent.save(out)
    return agent, stats


def main(argv: Optional[List[str]] = None):
    launch(list(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    main()
