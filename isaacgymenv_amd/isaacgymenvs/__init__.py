"""MI355X-native ``isaacgymenvs``: the ``make()`` env-creation API (reference ``isaacgymenvs/__init__.py:14-55``).

Configs are composed from this package's ``cfg/`` (same keys/values as the
reference) by a Hydra-compatible composer (``config.py``), since hydra and
omegaconf are not part of this image.
"""
from .config import compose
from .utils.reformat import omegaconf_to_dict


def make(seed: int, task: str, num_envs: int, sim_device: str, rl_device: str, graphics_device_id: int = -1,
         headless: bool = False, multi_gpu: bool = False, virtual_screen_capture: bool = False,
         force_render: bool = True, cfg=None, overrides=None):
    from .utils.rlgames_utils import get_rlgames_env_creator
    if cfg is None:
        cfg = compose("config", [f"task={task}", f"sim_device={sim_device}", f"rl_device={rl_device}"]
                      + list(overrides or []))
        cfg_dict = omegaconf_to_dict(cfg["task"])
        cfg_dict["env"]["numEnvs"] = num_envs
    else:
        cfg_dict = omegaconf_to_dict(cfg["task"] if "task" in cfg else cfg.task)
    create_rlgpu_env = get_rlgames_env_creator(
        seed=seed, task_config=cfg_dict, task_name=cfg_dict["name"], sim_device=sim_device, rl_device=rl_device,
        graphics_device_id=graphics_device_id, headless=headless, multi_gpu=multi_gpu,
        virtual_screen_capture=virtual_screen_capture, force_render=force_render)
    return create_rlgpu_env()
