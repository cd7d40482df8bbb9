#!/usr/bin/env python3
"""Pack the reference's in-scope robot descriptions into our own JSON form.

The reference ships its robots as URDF/MJCF under ``/root/reference/assets``
(``anymal_terrain.py:212``, ``cartpole.py:76``), which is not present on the GPU
box.  This script runs *our* importer (``isaacgymenv_amd/isaacgym/_assets.py``)
over those files and stores the parsed, pre-collapse description
(links, inertials, collision geometry, joints, limits) as
``isaacgymenv_amd/assets/<name>.model.json``.  ``gym.load_asset`` parses the URDF
itself when the file exists and falls back to the packed form otherwise.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from isaacgymenv_amd.isaacgym._assets import parse_urdf, PACKED_DIR  # noqa: E402
from isaacgymenv_amd.isaacgym._mjcf import parse_mjcf  # noqa: E402

REF = "/root/reference/assets"
SOURCES = {
    "anymal_c.model.json": "urdf/anymal_c/urdf/anymal_minimal.urdf",
    "cartpole.model.json": "urdf/cartpole.urdf",
    "hound.model.json": "urdf/UsefulHound/urdf/Hound.urdf",
    "nv_ant.model.json": "mjcf/nv_ant.xml",
    # the fork's own quadruped (hound.py:168-183): no compiled topology, the runtime-sized kernel runs it
    "hound_new.model.json": "urdf/Hound_new/Hound.urdf",
}


def main():
    os.makedirs(PACKED_DIR, exist_ok=True)
    for out, src in SOURCES.items():
        path = os.path.join(REF, src)
        raw = parse_mjcf(path) if src.endswith(".xml") else parse_urdf(path)
        with open(os.path.join(PACKED_DIR, out), "w") as f:
            json.dump(raw.to_json(), f, indent=1)
        print("packed", src, "->", out)


if __name__ == "__main__":
    main()
