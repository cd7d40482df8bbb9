"""Drop-in ``isaacgym.gymtorch``: zero-copy views between sim tensors and torch.

The sim's global tensors are torch tensors allocated on the sim device at
``prepare_sim``; ``wrap_tensor`` returns that tensor (sharing memory, as the
reference relies on at anymal_terrain.py:126-130) and ``unwrap_tensor`` hands a
borrowed descriptor to the ``set_*`` calls (anymal_terrain.py:401-407).
"""
from .gymapi import GymTensor


def wrap_tensor(gym_tensor, offsets=None, counts=None):
    if not isinstance(gym_tensor, GymTensor):
        raise TypeError("wrap_tensor expects a tensor descriptor returned by acquire_*_tensor")
    return gym_tensor.tensor


def unwrap_tensor(torch_tensor):
    return GymTensor(torch_tensor)
