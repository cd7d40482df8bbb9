"""Heightfield terrain generators and the heightfield -> triangle-mesh conversion (``isaacgym.terrain_utils``).

The reference imports these from the closed Isaac Gym package (``anymal_terrain.py:541``), which
is absent here, so this is a restatement of the published algorithms at the
reference's call sites (``anymal_terrain.py:576-653``):

* heights are int16 in units of ``vertical_scale``; cells are ``horizontal_scale`` wide;
* random draws go through numpy's global generator in the order the published code makes
  them (one ``choice`` for the coarse random field; per obstacle: width, length, start row,
  start column, height; per stepping-stone row: start offset then one height per stone);
* ``convert_heightfield_to_trimesh`` turns every grid cell into two triangles and, with a slope
  threshold, moves the low vertex of a too-steep edge under its high neighbour so steps become
  vertical walls.

Parity with Isaac Gym's own binary is unpinned (not importable anywhere in this pipeline); the
task-level fixtures in tests/golden pin the callers given these generators.
"""
from __future__ import annotations

import numpy as np

__all__ = ["SubTerrain", "random_uniform_terrain", "sloped_terrain", "pyramid_sloped_terrain",
           "discrete_obstacles_terrain", "stairs_terrain", "pyramid_stairs_terrain", "stepping_stones_terrain",
           "convert_heightfield_to_trimesh"]


class SubTerrain:
    """One tile of the terrain map: ``height_field_raw`` int16 [width, length]."""

    def __init__(self, terrain_name="terrain", width=256, length=256, vertical_scale=1.0, horizontal_scale=1.0):
        self.terrain_name = terrain_name
        self.vertical_scale = vertical_scale
        self.horizontal_scale = horizontal_scale
        self.width = width
        self.length = length
        self.height_field_raw = np.zeros((self.width, self.length), dtype=np.int16)


def _bilinear_resample(coarse: np.ndarray, extent_x: float, extent_y: float, nx: int, ny: int) -> np.ndarray:
    """Piecewise-linear interpolation of a grid spanning [0, extent] onto nx x ny evenly spaced points
    (the linear 2-D interpolant of the published code)."""
    xs = np.linspace(0, extent_x, coarse.shape[0])
    ys = np.linspace(0, extent_y, coarse.shape[1])
    xf = np.linspace(0, extent_x, nx)
    yf = np.linspace(0, extent_y, ny)
    c = coarse.astype(np.float64)
    # along y for every coarse row, then along x for every fine column
    rows = np.stack([np.interp(yf, ys, c[i]) for i in range(c.shape[0])])
    return np.stack([np.interp(xf, xs, rows[:, j]) for j in range(ny)], axis=1)


def random_uniform_terrain(terrain, min_height, max_height, step=1, downsampled_scale=None):
    """Add a random field drawn on a coarse grid (levels min..max in `step`) and linearly upsampled."""
    if downsampled_scale is None:
        downsampled_scale = terrain.horizontal_scale
    lo = int(min_height / terrain.vertical_scale)
    hi = int(max_height / terrain.vertical_scale)
    st = int(step / terrain.vertical_scale)
    levels = np.arange(lo, hi + st, st)
    ext_x = terrain.width * terrain.horizontal_scale
    ext_y = terrain.length * terrain.horizontal_scale
    coarse = np.random.choice(levels, (int(ext_x / downsampled_scale), int(ext_y / downsampled_scale)))
    fine = _bilinear_resample(coarse, ext_x, ext_y, terrain.width, terrain.length)
    terrain.height_field_raw += np.rint(fine).astype(np.int16)
    return terrain


def sloped_terrain(terrain, slope=1):
    """A plane rising along the first axis with the given slope."""
    rise = int(slope * (terrain.horizontal_scale / terrain.vertical_scale) * terrain.width)
    ramp = np.arange(terrain.width).reshape(terrain.width, 1) / terrain.width
    terrain.height_field_raw += (rise * ramp).astype(terrain.height_field_raw.dtype)
    return terrain


def pyramid_sloped_terrain(terrain, slope=1, platform_size=1.0):
    """Four-sided pyramid (negative slope: a pit), flattened to a square platform at the centre."""
    cx, cy = int(terrain.width / 2), int(terrain.length / 2)
    fx = ((cx - np.abs(cx - np.arange(terrain.width))) / cx).reshape(terrain.width, 1)
    fy = ((cy - np.abs(cy - np.arange(terrain.length))) / cy).reshape(1, terrain.length)
    peak = int(slope * (terrain.horizontal_scale / terrain.vertical_scale) * (terrain.width / 2))
    terrain.height_field_raw += (peak * fx * fy).astype(terrain.height_field_raw.dtype)
    half = int(platform_size / terrain.horizontal_scale / 2)
    edge = terrain.height_field_raw[terrain.width // 2 - half, terrain.length // 2 - half]
    terrain.height_field_raw = np.clip(terrain.height_field_raw, min(edge, 0), max(edge, 0))
    return terrain


def discrete_obstacles_terrain(terrain, max_height, min_size, max_size, num_rects, platform_size=1.0):
    """`num_rects` rectangular blocks of random footprint and height, with a flat centre platform."""
    hmax = int(max_height / terrain.vertical_scale)
    smin = int(min_size / terrain.horizontal_scale)
    smax = int(max_size / terrain.horizontal_scale)
    plat = int(platform_size / terrain.horizontal_scale)
    rows, cols = terrain.height_field_raw.shape
    heights = [-hmax, -hmax // 2, hmax // 2, hmax]
    sizes = range(smin, smax, 4)
    for _ in range(num_rects):
        w = np.random.choice(sizes)
        ln = np.random.choice(sizes)
        i0 = np.random.choice(range(0, rows - w, 4))
        j0 = np.random.choice(range(0, cols - ln, 4))
        terrain.height_field_raw[i0:i0 + w, j0:j0 + ln] = np.random.choice(heights)
    _flatten_centre(terrain, plat)
    return terrain


def stairs_terrain(terrain, step_width, step_height):
    """Straight stairs along the first axis."""
    w = int(step_width / terrain.horizontal_scale)
    dh = int(step_height / terrain.vertical_scale)
    level = 0
    for i in range(terrain.width // w):
        terrain.height_field_raw[i * w:(i + 1) * w, :] += level
        level += dh
    return terrain


def pyramid_stairs_terrain(terrain, step_width, step_height, platform_size=1.0):
    """Concentric square steps (up for a positive height, down for a negative one) to a centre platform."""
    w = int(step_width / terrain.horizontal_scale)
    dh = int(step_height / terrain.vertical_scale)
    plat = int(platform_size / terrain.horizontal_scale)
    x0, x1, y0, y1 = 0, terrain.width, 0, terrain.length
    level = 0
    while (x1 - x0) > plat and (y1 - y0) > plat:
        x0, x1, y0, y1 = x0 + w, x1 - w, y0 + w, y1 - w
        level += dh
        terrain.height_field_raw[x0:x1, y0:y1] = level
    return terrain


def stepping_stones_terrain(terrain, stone_size, stone_distance, max_height, platform_size=1.0, depth=-10):
    """Square stones separated by gaps of depth `depth` (metres), laid row by row along the longer axis."""
    size = int(stone_size / terrain.horizontal_scale)
    gap = int(stone_distance / terrain.horizontal_scale)
    hmax = int(max_height / terrain.vertical_scale)
    plat = int(platform_size / terrain.horizontal_scale)
    heights = np.arange(-hmax - 1, hmax, step=1)
    hf = terrain.height_field_raw
    hf[:, :] = int(depth / terrain.vertical_scale)
    if terrain.length >= terrain.width:
        b0 = 0
        while b0 < terrain.length:
            b1 = min(terrain.length, b0 + size)
            a0 = np.random.randint(0, size)
            hf[0:max(0, a0 - gap), b0:b1] = np.random.choice(heights)
            while a0 < terrain.width:
                hf[a0:min(terrain.width, a0 + size), b0:b1] = np.random.choice(heights)
                a0 += size + gap
            b0 += size + gap
    else:
        a0 = 0
        while a0 < terrain.width:
            a1 = min(terrain.width, a0 + size)
            b0 = np.random.randint(0, size)
            hf[a0:a1, 0:max(0, b0 - gap)] = np.random.choice(heights)
            while b0 < terrain.length:
                hf[a0:a1, b0:min(terrain.length, b0 + size)] = np.random.choice(heights)
                b0 += size + gap
            a0 += size + gap
    _flatten_centre(terrain, plat)
    return terrain


def _flatten_centre(terrain, plat: int):
    x0, x1 = (terrain.width - plat) // 2, (terrain.width + plat) // 2
    y0, y1 = (terrain.length - plat) // 2, (terrain.length + plat) // 2
    terrain.height_field_raw[x0:x1, y0:y1] = 0


def convert_heightfield_to_trimesh(height_field_raw, horizontal_scale, vertical_scale, slope_threshold=None):
    """Grid mesh of a heightfield: vertex (i, j) at (i*hs, j*hs, h*vs), row-major; cell (i, j) -> triangles
    (v[i,j], v[i+1,j+1], v[i,j+1]) and (v[i,j], v[i+1,j], v[i+1,j+1]).  With a slope threshold, a vertex
    whose neighbour along +-x, +-y or the +-(x,y) diagonal is higher by more than threshold*hs moves
    one cell towards that neighbour (vertical walls instead of steep ramps)."""
    hf = np.asarray(height_field_raw)
    rows, cols = hf.shape
    gx = np.repeat(np.linspace(0, (rows - 1) * horizontal_scale, rows)[:, None], cols, axis=1)
    gy = np.repeat(np.linspace(0, (cols - 1) * horizontal_scale, cols)[None, :], rows, axis=0)
    if slope_threshold is not None:
        thr = slope_threshold * horizontal_scale / vertical_scale
        h = hf.astype(np.int64)
        mx = np.zeros((rows, cols))
        my = np.zeros((rows, cols))
        md = np.zeros((rows, cols))
        mx[:-1, :] += (h[1:, :] - h[:-1, :]) > thr
        mx[1:, :] -= (h[:-1, :] - h[1:, :]) > thr
        my[:, :-1] += (h[:, 1:] - h[:, :-1]) > thr
        my[:, 1:] -= (h[:, :-1] - h[:, 1:]) > thr
        md[:-1, :-1] += (h[1:, 1:] - h[:-1, :-1]) > thr
        md[1:, 1:] -= (h[:-1, :-1] - h[1:, 1:]) > thr
        gx = gx + (mx + md * (mx == 0)) * horizontal_scale
        gy = gy + (my + md * (my == 0)) * horizontal_scale
    vertices = np.zeros((rows * cols, 3), dtype=np.float32)
    vertices[:, 0] = gx.reshape(-1)
    vertices[:, 1] = gy.reshape(-1)
    vertices[:, 2] = hf.reshape(-1) * vertical_scale
    base = (np.arange(rows - 1)[:, None] * cols + np.arange(cols - 1)[None, :]).reshape(-1)
    triangles = np.empty((2 * base.size, 3), dtype=np.uint32)
    triangles[0::2, 0] = base
    triangles[0::2, 1] = base + cols + 1
    triangles[0::2, 2] = base + 1
    triangles[1::2, 0] = base
    triangles[1::2, 1] = base + cols
    triangles[1::2, 2] = base + cols + 1
    return vertices, triangles
