#!/usr/bin/env python3
"""Import the in-scope Hydra configs of the reference as data.

The task/train YAMLs are part of the API surface the build keeps identical
(BASELINE.json north_star: "Hydra task configs ... stay identical"), so their
keys and values are loaded from /root/reference/isaacgymenvs/cfg with
``yaml.safe_load`` and re-emitted (sorted keys, no comments) under
isaacgymenv_amd/isaacgymenvs/cfg/.  Interpolations such as
``${resolve_default:4096,${...num_envs}}`` are kept verbatim; our composer
(isaacgymenvs/config.py) resolves them.
"""
import os
import sys

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = "/root/reference/isaacgymenvs/cfg"
DST = os.path.join(ROOT, "isaacgymenv_amd", "isaacgymenvs", "cfg")
FILES = ["config.yaml"] + [f"task/{t}.yaml" for t in ("AnymalTerrain", "Ant", "Cartpole", "UsefulHound")] + \
        [f"train/{t}PPO.yaml" for t in ("AnymalTerrain", "Ant", "Cartpole", "UsefulHound")]

HEADER = "# Imported from the reference config of the same name by tools/import_configs.py (data, keys/values unchanged)\n"


def main():
    for f in FILES:
        with open(os.path.join(SRC, f)) as fh:
            data = yaml.safe_load(fh)
        out = os.path.join(DST, f)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        with open(out, "w") as fh:
            fh.write(HEADER)
            yaml.safe_dump(data, fh, sort_keys=True, default_flow_style=None, width=120)
        print("imported", f)


if __name__ == "__main__":
    sys.exit(main())
