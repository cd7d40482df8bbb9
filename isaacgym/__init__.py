"""Top-level alias so reference code doing ``from isaacgym import gymapi, gymtorch``
(vec_task.py:37) gets the MI355X-native implementation in isaacgymenv_amd/isaacgym."""
import sys as _sys

from isaacgymenv_amd.isaacgym import gymapi, gymtorch, gymutil, terrain_utils  # noqa: F401

_sys.modules[__name__ + ".gymapi"] = gymapi
_sys.modules[__name__ + ".gymtorch"] = gymtorch
_sys.modules[__name__ + ".gymutil"] = gymutil
_sys.modules[__name__ + ".terrain_utils"] = terrain_utils
