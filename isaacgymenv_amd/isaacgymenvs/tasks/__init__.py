"""Task registry (reference ``tasks/__init__.py:90-119``), in-scope tasks only."""
from .ant import Ant
from .anymal_terrain import AnymalTerrain
from .cartpole import Cartpole
from .useful_hound import UsefulHound

isaacgym_task_map = {
    "Ant": Ant,
    "AnymalTerrain": AnymalTerrain,
    "Cartpole": Cartpole,
    "UsefulHound": UsefulHound,
}
