"""Top-level alias: ``import isaacgymenvs`` / ``isaacgymenvs.make(...)`` resolve to the
MI355X-native implementation in isaacgymenv_amd/isaacgymenvs."""
import sys as _sys

import isaacgymenv_amd.isaacgymenvs as _impl
from isaacgymenv_amd.isaacgymenvs import *  # noqa: F401,F403
from isaacgymenv_amd.isaacgymenvs import make, compose  # noqa: F401

_sys.modules[__name__] = _impl
