"""Task registry (reference ``tasks/__init__.py:90-119``), in-scope tasks only."""
from .anymal_terrain import AnymalTerrain
from .cartpole import Cartpole

isaacgym_task_map = {
    "AnymalTerrain": AnymalTerrain,
    "Cartpole": Cartpole,
}
