"""``Env`` / ``VecTask``: the hot-loop orchestrator (reference ``tasks/base/vec_task.py``).

Behaviour kept identical to the reference, because rl_games and the task
subclasses depend on it:

* device selection and buffer allocation (vec_task.py:78-88, 301-324);
* ``step`` = clamp -> ``pre_physics_step`` -> ``controlFrequencyInv`` x
  ``gym.simulate`` -> ``post_physics_step`` -> ``timeout_buf`` -> ``extras`` ->
  obs clamp (vec_task.py:360-408), including the quirk that a task whose
  ``pre_physics_step`` already simulates (AnymalTerrain's decimation loop) gets
  one more simulate from this loop;
* ``reset`` returns the (initially all-zero) obs buffer without computing it
  (vec_task.py:426-438); ``reset_done`` resets flagged envs (:440-455);
* ``SimParams`` parsing from the ``sim`` config block (vec_task.py:514-562).

MI355X addition: a task may implement ``fused_physics_step(actions)``; when it
does (and the sim runs the GPU pipeline), ``step`` calls it INSTEAD of
``pre_physics_step`` + the simulate loop.  The fused call must have exactly the
observable effect of the unfused sequence (tests/test_task_gpu.py).  A task's
fused tail may also hand ``step`` its ``(time_outs, clamped obs)`` pair through
``self._fused_outputs`` (computed by the same kernel that writes ``obs_buf``),
which replaces the three torch ops of vec_task.py:393-402.
"""
from __future__ import annotations

import abc
import math
import os
import sys
import time
from typing import Any, Dict, Tuple

import numpy as np
import torch

from isaacgym import gymapi, gymtorch  # the MI355X drop-in (top-level alias package)

try:  # pragma: no cover - gym is not installed in this image
    from gym import spaces  # type: ignore
except Exception:  # minimal stand-in with the attributes rl_games reads
    class _Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low = np.asarray(low, dtype=dtype)
            self.high = np.asarray(high, dtype=dtype)
            self.shape = self.low.shape if shape is None else tuple(shape)
            self.dtype = np.dtype(dtype)

        def __repr__(self):
            return f"Box({self.shape})"

    class spaces:  # noqa: N801
        Box = _Box

EXISTING_SIM = None


def _create_sim_once(gym, *args, **kwargs):
    """One sim per process, reused by later VecTasks (vec_task.py:55-64)."""
    global EXISTING_SIM
    if EXISTING_SIM is None:
        EXISTING_SIM = gym.create_sim(*args, **kwargs)
    return EXISTING_SIM


class Env(abc.ABC):
    def __init__(self, config: Dict[str, Any], rl_device: str, sim_device: str, graphics_device_id: int,
                 headless: bool):
        parts = sim_device.split(":")
        self.device_type = parts[0]
        self.device_id = int(parts[1]) if len(parts) > 1 else 0
        self.device = "cpu"
        if config["sim"]["use_gpu_pipeline"]:
            if self.device_type.lower() in ("cuda", "gpu"):
                self.device = f"cuda:{self.device_id}"
            else:
                print("GPU Pipeline can only be used with GPU simulation. Forcing CPU Pipeline.")
                config["sim"]["use_gpu_pipeline"] = False
        self.rl_device = rl_device
        self.headless = headless
        self.graphics_device_id = graphics_device_id
        if not config.get("enableCameraSensors", False) and self.headless:
            self.graphics_device_id = -1
        env_cfg = config["env"]
        self.num_environments = env_cfg["numEnvs"]
        self.num_agents = env_cfg.get("numAgents", 1)
        self.num_observations = env_cfg.get("numObservations", 0)
        self.num_states = env_cfg.get("numStates", 0)
        self.obs_space = spaces.Box(np.ones(self.num_obs) * -np.inf, np.ones(self.num_obs) * np.inf)
        self.state_space = spaces.Box(np.ones(self.num_states) * -np.inf, np.ones(self.num_states) * np.inf)
        self.num_actions = env_cfg["numActions"]
        self.control_freq_inv = env_cfg.get("controlFrequencyInv", 1)
        self.act_space = spaces.Box(np.ones(self.num_actions) * -1.0, np.ones(self.num_actions) * 1.0)
        self.clip_obs = env_cfg.get("clipObservations", np.inf)
        self.clip_actions = env_cfg.get("clipActions", np.inf)
        self.total_train_env_frames = 0
        self.control_steps = 0
        self.render_fps = env_cfg.get("renderFPS", -1)
        self.last_frame_time = 0.0
        self.record_frames = False

    @abc.abstractmethod
    def allocate_buffers(self):
        ...

    @abc.abstractmethod
    def step(self, actions: torch.Tensor):
        ...

    @abc.abstractmethod
    def reset(self):
        ...

    @abc.abstractmethod
    def reset_idx(self, env_ids: torch.Tensor):
        ...

    @property
    def observation_space(self):
        return self.obs_space

    @property
    def action_space(self):
        return self.act_space

    @property
    def num_envs(self) -> int:
        return self.num_environments

    @property
    def num_acts(self) -> int:
        return self.num_actions

    @property
    def num_obs(self) -> int:
        return self.num_observations

    def set_train_info(self, env_frames, *args, **kwargs):
        self.total_train_env_frames = env_frames

    def get_env_state(self):
        return None

    def set_env_state(self, env_state):
        pass


class VecTask(Env):
    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": 24}

    def __init__(self, config, rl_device, sim_device, graphics_device_id, headless,
                 virtual_screen_capture: bool = False, force_render: bool = False):
        super().__init__(config, rl_device, sim_device, graphics_device_id, headless)
        self.virtual_screen_capture = virtual_screen_capture
        self.virtual_display = None
        self.force_render = force_render
        self.sim_params = self._parse_sim_params(self.cfg["physics_engine"], self.cfg["sim"])
        if self.cfg["physics_engine"] == "physx":
            self.physics_engine = gymapi.SIM_PHYSX
        elif self.cfg["physics_engine"] == "flex":
            self.physics_engine = gymapi.SIM_FLEX
        else:
            raise ValueError(f"Invalid physics engine backend: {self.cfg['physics_engine']}")
        self.dt: float = self.sim_params.dt
        self.gym = gymapi.acquire_gym()
        self.first_randomization = True
        self.original_props = {}
        self.dr_randomizations = {}
        self.actor_params_generator = None
        self.extern_actor_params = {env_id: None for env_id in range(self.num_envs)}
        self.last_step = -1
        self.last_rand_step = -1
        self.sim_initialized = False
        self.create_sim()
        self.gym.prepare_sim(self.sim)
        self.sim_initialized = True
        self.set_viewer()
        self.allocate_buffers()
        self.obs_dict = {}

    def set_viewer(self):
        self.enable_viewer_sync = True
        self.viewer = None
        if not self.headless:
            self.viewer = self.gym.create_viewer(self.sim, gymapi.CameraProperties())

    def allocate_buffers(self):
        dev = self.device
        self.obs_buf = torch.zeros((self.num_envs, self.num_obs), device=dev, dtype=torch.float)
        self.states_buf = torch.zeros((self.num_envs, self.num_states), device=dev, dtype=torch.float)
        self.rew_buf = torch.zeros(self.num_envs, device=dev, dtype=torch.float)
        self.reset_buf = torch.ones(self.num_envs, device=dev, dtype=torch.long)
        self.timeout_buf = torch.zeros(self.num_envs, device=dev, dtype=torch.long)
        self.progress_buf = torch.zeros(self.num_envs, device=dev, dtype=torch.long)
        self.randomize_buf = torch.zeros(self.num_envs, device=dev, dtype=torch.long)
        self.extras = {}

    def create_sim(self, compute_device: int, graphics_device: int, physics_engine, sim_params):
        sim = _create_sim_once(self.gym, compute_device, graphics_device, physics_engine, sim_params)
        if sim is None:
            print("*** Failed to create sim")
            quit()
        return sim

    def get_state(self):
        return torch.clamp(self.states_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)

    @abc.abstractmethod
    def pre_physics_step(self, actions: torch.Tensor):
        ...

    @abc.abstractmethod
    def post_physics_step(self):
        ...

    # the fused path is optional; tasks that provide it set this to True
    supports_fused_physics = False
    _fused_outputs = None

    def _use_fused(self) -> bool:
        return (self.supports_fused_physics and self.device != "cpu" and not self.force_render
                and os.environ.get("GS_DISABLE_FUSED", "0") != "1")

    def step(self, actions: torch.Tensor) -> Tuple[Dict[str, torch.Tensor], torch.Tensor, torch.Tensor,
                                                   Dict[str, Any]]:
        if self.dr_randomizations.get("actions", None):
            actions = self.dr_randomizations["actions"]["noise_lambda"](actions)
        if math.isinf(self.clip_actions):  # (a Python float: math.isinf, ~1 us cheaper per step than np.isinf)
            action_tensor = actions  # clamp(+-inf) is an identity copy; pre_physics_step clones anyway
        else:
            action_tensor = torch.clamp(actions, -self.clip_actions, self.clip_actions)
        if self._use_fused():
            self.fused_physics_step(action_tensor)
        else:
            self.pre_physics_step(action_tensor)
            for _ in range(self.control_freq_inv):
                if self.force_render:
                    self.render()
                self.gym.simulate(self.sim)
        if self.device == "cpu":
            self.gym.fetch_results(self.sim, True)
        self.post_physics_step()
        self.control_steps += 1
        fused_out, self._fused_outputs = self._fused_outputs, None
        if fused_out is not None:
            self.timeout_buf, obs = fused_out
            if self._rl_on_sim_device():  # .to(rl_device) returns the tensor itself: skip the device parse
                self.extras["time_outs"] = self.timeout_buf
                self.obs_dict["obs"] = obs
                if self.num_states > 0:
                    self.obs_dict["states"] = self.get_state()
                return self.obs_dict, self.rew_buf, self.reset_buf, self.extras
            self.extras["time_outs"] = self.timeout_buf.to(self.rl_device)
            self.obs_dict["obs"] = obs.to(self.rl_device)
        else:
            # set to 1 only when the episode length is reached AND the env is being reset (vec_task.py:393-394)
            self.timeout_buf = (self.progress_buf >= self.max_episode_length - 1) & (self.reset_buf != 0)
            if self.dr_randomizations.get("observations", None):
                self.obs_buf = self.dr_randomizations["observations"]["noise_lambda"](self.obs_buf)
            self.extras["time_outs"] = self.timeout_buf.to(self.rl_device)
            self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        if self.num_states > 0:
            self.obs_dict["states"] = self.get_state()
        return self.obs_dict, self.rew_buf.to(self.rl_device), self.reset_buf.to(self.rl_device), self.extras

    _rl_same_device = None

    def _rl_on_sim_device(self) -> bool:
        """rl_device names the tensors' own device (then every .to(rl_device) of step() is the identity)."""
        if self._rl_same_device is None:
            self._rl_same_device = torch.device(self.rl_device) == self.rew_buf.device == self.reset_buf.device
        return self._rl_same_device

    def zero_actions(self) -> torch.Tensor:
        return torch.zeros([self.num_envs, self.num_actions], dtype=torch.float32, device=self.rl_device)

    def reset_idx(self, env_idx):
        pass

    def reset(self):
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        if self.num_states > 0:
            self.obs_dict["states"] = self.get_state()
        return self.obs_dict

    def reset_done(self):
        done_env_ids = self.reset_buf.nonzero(as_tuple=False).flatten()
        if len(done_env_ids) > 0:
            self.reset_idx(done_env_ids)
        self.obs_dict["obs"] = torch.clamp(self.obs_buf, -self.clip_obs, self.clip_obs).to(self.rl_device)
        if self.num_states > 0:
            self.obs_dict["states"] = self.get_state()
        return self.obs_dict, done_env_ids

    def render(self, mode="rgb_array"):
        return None  # headless build (viewer is out of scope)

    def _parse_sim_params(self, physics_engine: str, config_sim: Dict[str, Any]):
        sim_params = gymapi.SimParams()
        if config_sim["up_axis"] not in ("z", "y"):
            msg = f"Invalid physics up-axis: {config_sim['up_axis']}"
            print(msg)
            raise ValueError(msg)
        sim_params.dt = config_sim["dt"]
        sim_params.num_client_threads = config_sim.get("num_client_threads", 0)
        sim_params.use_gpu_pipeline = config_sim["use_gpu_pipeline"]
        sim_params.substeps = config_sim.get("substeps", 2)
        sim_params.up_axis = gymapi.UP_AXIS_Z if config_sim["up_axis"] == "z" else gymapi.UP_AXIS_Y
        sim_params.gravity = gymapi.Vec3(*config_sim["gravity"])
        if physics_engine == "physx":
            for opt, val in config_sim.get("physx", {}).items():
                if opt == "contact_collection":
                    setattr(sim_params.physx, opt, gymapi.ContactCollection(val))
                else:
                    setattr(sim_params.physx, opt, val)
        else:
            for opt, val in config_sim.get("flex", {}).items():
                setattr(sim_params.flex, opt, val)
        return sim_params
