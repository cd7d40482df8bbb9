"""PPO learner for VecTask envs: an rl_games-compatible ``a2c_continuous`` (the reference's
trainer, isaacgymenvs/train.py:188-218; rl-games>=1.6.0 per setup.py:22 is not installed in
this image) with GAE on the device (libgymrl.so) and one flat RCCL all-reduce of the
gradients per minibatch for multi-GPU data parallelism."""
from .a2c_continuous import A2CAgent, PpoConfig  # noqa: F401
