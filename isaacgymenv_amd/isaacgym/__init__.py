"""MI355X-native drop-in for the ``isaacgym`` package (gymapi / gymtorch).

Import it as ``isaacgym`` through the top-level alias package in the repo root,
or directly as ``isaacgymenv_amd.isaacgym``.
"""
