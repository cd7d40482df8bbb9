"""rl_games adapter (reference ``utils/rlgames_utils.py``): env creator + ``RLGPUEnv``.

rl_games is an external dependency (``setup.py:22`` ``rl-games>=1.6.0``) and is
not installed in this image; the adapter imports it lazily so ``make()`` works
without it, and ``RLGPUEnv`` subclasses ``vecenv.IVecEnv`` when it is present.
"""
import os
from typing import Callable


def multi_gpu_get_rank(multi_gpu):
    if multi_gpu:
        rank = int(os.getenv("LOCAL_RANK", "0"))
        print("GPU rank: ", rank)
        return rank
    return 0


def get_rlgames_env_creator(seed: int, task_config: dict, task_name: str, sim_device: str, rl_device: str,
                            graphics_device_id: int, headless: bool, multi_gpu: bool = False,
                            post_create_hook: Callable = None, virtual_screen_capture: bool = False,
                            force_render: bool = False):
    """Returns a closure creating the task; multi-GPU maps LOCAL_RANK -> cuda:k (rlgames_utils.py:53-127)."""

    def create_rlgpu_env():
        from ..tasks import isaacgym_task_map
        if multi_gpu:
            local_rank = int(os.getenv("LOCAL_RANK", "0"))
            global_rank = int(os.getenv("RANK", "0"))
            world_size = int(os.getenv("WORLD_SIZE", "1"))
            print(f"global_rank = {global_rank} local_rank = {local_rank} world_size = {world_size}")
            _sim_device = f"cuda:{local_rank}"
            _rl_device = f"cuda:{local_rank}"
            task_config["rank"] = local_rank
            task_config["rl_device"] = _rl_device
        else:
            _sim_device, _rl_device = sim_device, rl_device
        env = isaacgym_task_map[task_name](cfg=task_config, rl_device=_rl_device, sim_device=_sim_device,
                                           graphics_device_id=graphics_device_id, headless=headless,
                                           virtual_screen_capture=virtual_screen_capture, force_render=force_render)
        if post_create_hook is not None:
            post_create_hook()
        return env

    return create_rlgpu_env


try:  # pragma: no cover - rl_games is absent here
    from rl_games.common import env_configurations, vecenv  # type: ignore
    _IVecEnv = vecenv.IVecEnv
except Exception:
    env_configurations = None
    _IVecEnv = object


class RLGPUEnv(_IVecEnv):
    """rl_games ``IVecEnv`` over a VecTask (rlgames_utils.py:242-295)."""

    def __init__(self, config_name, num_actors, **kwargs):
        if env_configurations is None:
            raise ImportError("rl_games is not installed")
        self.env = env_configurations.configurations[config_name]["env_creator"](**kwargs)

    @classmethod
    def from_env(cls, env):
        obj = cls.__new__(cls)
        obj.env = env
        return obj

    def step(self, actions):
        return self.env.step(actions)

    def reset(self):
        return self.env.reset()

    def reset_done(self):
        return self.env.reset_done()

    def get_number_of_agents(self):
        return self.env.get_number_of_agents()

    def get_env_info(self):
        info = {"action_space": self.env.action_space, "observation_space": self.env.observation_space}
        if self.env.num_states > 0:
            info["state_space"] = self.env.state_space
        return info

    def set_train_info(self, env_frames, *args_, **kwargs_):
        if hasattr(self.env, "set_train_info"):
            self.env.set_train_info(env_frames, *args_, **kwargs_)

    def get_env_state(self):
        return self.env.get_env_state() if hasattr(self.env, "get_env_state") else None

    def set_env_state(self, env_state):
        if hasattr(self.env, "set_env_state"):
            self.env.set_env_state(env_state)
