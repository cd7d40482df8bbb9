"""Minimal ``isaacgym.gymutil`` (viewer helpers are headless no-ops)."""


class WireframeSphereGeometry:
    def __init__(self, *args, **kwargs):
        pass


def draw_lines(*args, **kwargs):
    return None
