"""Asset import (gym.load_asset replacement) -- host logic, CPU only."""
import os

import numpy as np
import pytest

from isaacgymenv_amd.isaacgym._assets import parse_urdf, build_articulation, RawModel
from tests import helpers as H

REF_URDF = "/root/reference/assets/urdf/anymal_c/urdf/anymal_minimal.urdf"


def test_anymal_collapsed_bodies_and_dofs():
    art, flat = H.anymal()
    assert art.body_names() == ["base", "LF_HIP", "LF_THIGH", "LF_SHANK", "LH_HIP", "LH_THIGH", "LH_SHANK",
                                "RF_HIP", "RF_THIGH", "RF_SHANK", "RH_HIP", "RH_THIGH", "RH_SHANK"]
    names = art.dof_names()
    assert names == ["LF_HAA", "LF_HFE", "LF_KFE", "LH_HAA", "LH_HFE", "LH_KFE", "RF_HAA", "RF_HFE", "RF_KFE",
                     "RH_HAA", "RH_HFE", "RH_KFE"]
    assert [names[i] for i in (0, 3, 6, 9)] == ["LF_HAA", "LH_HAA", "RF_HAA", "RH_HAA"]  # anymal_terrain.py:359
    assert art.chains() == [3, 3, 3, 3]
    # 9 collision shapes: base capsule, 4 knee capsules (THIGH), 4 foot spheres (SHANK) -> 14 candidates
    assert art.num_shapes == 9 and flat["nc"] == 14
    assert all(d.effort == 80.0 and d.velocity == 20.0 and not d.has_limits for d in art.dofs)
    total = sum(b.mass for b in art.bodies)
    assert 50.0 < total < 56.0


def test_packed_model_equals_fresh_parse():
    if not os.path.exists(REF_URDF):
        pytest.skip("reference assets not present (GPU box)")
    raw = parse_urdf(REF_URDF)
    a = build_articulation(raw, H.ANYMAL_OPTS)
    b, _ = H.anymal()
    for x, y in zip(a.bodies, b.bodies):
        assert x.name == y.name
        np.testing.assert_allclose(x.mass, y.mass)
        np.testing.assert_allclose(x.com, y.com)
        np.testing.assert_allclose(x.inertia, y.inertia)


def test_inertia_merge_parallel_axis():
    # two point masses welded by a fixed joint -> combined COM and inertia
    raw = RawModel.from_json({"name": "t", "links": [
        {"name": "a", "inertial": {"mass": 1.0, "com": [0, 0, 0], "inertia": np.eye(3).tolist()}, "shapes": []},
        {"name": "b", "inertial": {"mass": 1.0, "com": [0, 0, 0], "inertia": np.eye(3).tolist()}, "shapes": []}],
        "joints": [{"name": "j", "kind": 0, "parent": "a", "child": "b",
                    "origin": {"R": np.eye(3).tolist(), "t": [2.0, 0, 0]}, "axis": [1, 0, 0], "lower": 0,
                    "upper": 0, "has_limits": False, "effort": 0, "velocity": 0, "damping": 0, "friction": 0}]})
    art = build_articulation(raw, dict(collapse_fixed_joints=True))
    b = art.bodies[0]
    assert len(art.bodies) == 1 and b.mass == 2.0
    np.testing.assert_allclose(b.com, [1.0, 0, 0])
    np.testing.assert_allclose(np.diag(b.inertia), [2.0, 4.0, 4.0])


def test_cartpole_model():
    art, flat = H.cartpole()
    assert art.body_names() == ["slider", "cart", "pole"]
    assert art.dof_names() == ["slider_to_cart", "cart_to_pole"]
    assert art.fixed_base and art.dofs[0].has_limits and not art.dofs[1].has_limits
    assert all(b != 0 for b in flat["cbody"])  # no candidates on the welded root


def test_stl_collision_meshes_collide_as_convex_hulls(tmp_path):
    """Hound.urdf:508-661: the arm's STL collision meshes become convex hulls with ALL hull
    vertices kept (a box mesh gives back its 8 corners, interior and duplicate vertices are dropped); each
    hull has HULL_SLOTS dynamic ground candidates."""
    import numpy as np
    from isaacgymenv_amd.isaacgym import _assets as A
    from isaacgymenv_amd.isaacgym._model import flatten
    # a binary STL cube [0, 2] x [0, 4] x [0, 6] mm -> scaled 0.001: corners only
    corners = np.array([[x, y, z] for x in (0, 2) for y in (0, 4) for z in (0, 6)], dtype=np.float32)
    faces = [(0, 1, 3), (0, 3, 2), (4, 6, 7), (4, 7, 5), (0, 4, 5), (0, 5, 1), (2, 3, 7), (2, 7, 6),
             (0, 2, 6), (0, 6, 4), (1, 5, 7), (1, 7, 3)]
    rec = np.zeros(len(faces), dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
    rec["v"] = corners[np.array(faces)]
    (tmp_path / "cube.stl").write_bytes(b"\0" * 80 + len(faces).to_bytes(4, "little") + rec.tobytes())
    pts = A.convex_hull_vertices(A.read_stl(str(tmp_path / "cube.stl")) * 0.001)
    assert pts.shape == (8, 3)
    assert {tuple(np.round(p * 1000).astype(int)) for p in pts} == {tuple(c) for c in corners.astype(int)}
    # an interior point is not a hull vertex
    inner = np.concatenate([A.read_stl(str(tmp_path / "cube.stl")), [[1.0, 2.0, 3.0]]])
    assert len(A.convex_hull_vertices(inner)) == 8
    # the packed Hound model: every arm link collides through its hull, none is dropped
    raw = A.load_raw("/nonexistent", "urdf/UsefulHound/urdf/Hound.urdf")
    arm = ["link1", "link2", "link3", "link4", "link5", "link6", "end_link"]
    for n in arm:
        assert not raw.links[n].dropped_meshes
        assert [s.kind for s in raw.links[n].shapes] == [A.SHAPE_CONVEX]
    art = A.build_articulation(raw, dict(collapse_fixed_joints=False, replace_cylinder_with_capsule=False))
    flat = flatten(art)
    assert flat["nc"] == 84 + 7 * A.HULL_SLOTS and flat["ns"] == 24
    assert len(flat["hverts"]) > 1000 and (flat["cdyn"] >= 0).sum() == 7 * A.HULL_SLOTS
    names = art.link_names()
    cand_links = [names[i] for i in art.candidate_links()]
    assert sum(n in arm for n in cand_links) == 7 * A.HULL_SLOTS
