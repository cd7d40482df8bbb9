"""Shared test helpers (test infrastructure)."""
import json
import os

import numpy as np

from isaacgymenv_amd.isaacgym._assets import PACKED_DIR, RawModel, build_articulation
from isaacgymenv_amd.isaacgym._model import flatten

ANYMAL_OPTS = dict(collapse_fixed_joints=True, replace_cylinder_with_capsule=True)
CARTPOLE_OPTS = dict(fix_base_link=True)
ANYMAL_DEFAULT = {"LF_HAA": 0.03, "LH_HAA": 0.03, "RF_HAA": -0.03, "RH_HAA": -0.03, "LF_HFE": 0.4,
                  "LH_HFE": -0.4, "RF_HFE": 0.4, "RH_HFE": -0.4, "LF_KFE": -0.8, "LH_KFE": 0.8,
                  "RF_KFE": -0.8, "RH_KFE": 0.8}
# AnymalTerrain.yaml:129-146
ANYMAL_PARAMS = dict(dt=0.005, substeps=1, gravity=[0.0, 0.0, -9.81], pos_iters=4, vel_iters=1,
                     contact_offset=0.02, rest_offset=0.0, max_depen_vel=100.0, collect_contacts=1,
                     has_ground=1, ground_friction=1.0)
# Cartpole.yaml:23-42
CARTPOLE_PARAMS = dict(dt=0.0166, substeps=2, gravity=[0.0, 0.0, -9.81], pos_iters=4, vel_iters=0,
                       contact_offset=0.02, rest_offset=0.001, max_depen_vel=100.0, collect_contacts=0,
                       has_ground=1, ground_friction=1.0)


# Ant.yaml:42-61 (dt 1/60, 2 substeps, 4/0 iterations, contact collection never)
ANT_PARAMS = dict(dt=0.0166, substeps=2, gravity=[0.0, 0.0, -9.81], pos_iters=4, vel_iters=0,
                  contact_offset=0.02, rest_offset=0.0, max_depen_vel=10.0, collect_contacts=0,
                  has_ground=1, ground_friction=1.0, limit_margin=0.1)
ANT_FEET = [2, 4, 6, 8]  # bodies whose names contain "foot" (ant.py:166-173)

# UsefulHound.yaml:161-180 (dt 0.005, 1 substep, 4/1 iterations, contact collection last substep);
# asset options useful_hound.py:318-329 (fixed joints kept: 19 dynamic bodies, 24 links)
HOUND_OPTS = dict(collapse_fixed_joints=False, replace_cylinder_with_capsule=False, fix_base_link=False,
                  density=0.001, angular_damping=0.0, linear_damping=0.0, armature=0.0, thickness=0.01)
HOUND_PARAMS = dict(dt=0.005, substeps=1, gravity=[0.0, 0.0, -9.81], pos_iters=4, vel_iters=1,
                    contact_offset=0.02, rest_offset=0.0, max_depen_vel=100.0, collect_contacts=1,
                    has_ground=1, ground_friction=1.0, limit_margin=0.1)


# collision filters of the reference tasks' create_actor calls: 0 (self-collision) for AnymalTerrain
# (anymal_terrain.py:282) and UsefulHound (useful_hound.py:421), 1 for Ant (ant.py:190) and Cartpole
# (cartpole.py:107).  flatten() results of these helpers carry it as flat["self_collide"], which the
# oracle (OracleSim) and make_gpu_sim follow.
SELF_COLLIDE = {"anymal": 1, "hound": 1, "ant": 0, "cartpole": 0, "hound_new": 0}
# hound.py:170-181 (the fork's own quadruped, assets/urdf/Hound_new/Hound.urdf; collision filter 1, :208) and
# cfg/task/Hound.yaml:31-32,53 (position drives 85 / 2, fixed joints kept): no compiled topology -- the
# runtime-sized kernel (gs_generic.hip) runs it
HOUND_NEW_OPTS = dict(HOUND_OPTS, collapse_fixed_joints=False)
HOUND_NEW_DRIVES = (np.full(12, 1, dtype=np.int32), np.full(12, 85.0), np.full(12, 2.0))


def load_art(name, opts):
    with open(os.path.join(PACKED_DIR, name)) as f:
        return build_articulation(RawModel.from_json(json.load(f)), opts)


def anymal():
    art = load_art("anymal_c.model.json", ANYMAL_OPTS)
    flat = flatten(art)
    flat["self_collide"] = SELF_COLLIDE["anymal"]
    return art, flat


def cartpole():
    art = load_art("cartpole.model.json", CARTPOLE_OPTS)
    flat = flatten(art)
    flat["self_collide"] = SELF_COLLIDE["cartpole"]
    return art, flat


def ant():
    art = load_art("nv_ant.model.json", dict(angular_damping=0.0))
    flat = flatten(art)
    flat["self_collide"] = SELF_COLLIDE["ant"]
    return art, flat


def hound():
    art = load_art("hound.model.json", HOUND_OPTS)
    flat = flatten(art)
    flat["self_collide"] = SELF_COLLIDE["hound"]
    return art, flat


def hound_new():
    art = load_art("hound_new.model.json", HOUND_NEW_OPTS)
    flat = flatten(art)
    flat["self_collide"] = SELF_COLLIDE["hound_new"]
    return art, flat


def hound_new_states(n, seed=0, spread=1.0):
    """Random Hound_new states: standing near Hound.yaml's 0.62 m (feet on, above or into the ground), tilted,
    moving, joints within their limits."""
    rng = np.random.RandomState(seed)
    art, flat = hound_new()
    root = np.zeros((n, 13))
    root[:, 0:2] = rng.uniform(-2, 2, (n, 2))
    root[:, 2] = rng.uniform(0.35, 0.65, n)
    axis = rng.normal(size=(n, 3))
    axis /= np.linalg.norm(axis, axis=1, keepdims=True)
    ang = rng.uniform(0, 0.3 * spread, n)
    root[:, 3:6] = axis * np.sin(ang / 2)[:, None]
    root[:, 6] = np.cos(ang / 2)
    root[:, 7:10] = rng.normal(0, 0.3 * spread, (n, 3))
    root[:, 10:13] = rng.normal(0, 0.5 * spread, (n, 3))
    dof = np.zeros((n, 12, 2))
    leg = np.tile([0.0, 0.6, -1.2], 4)
    dof[:, :, 0] = leg + rng.uniform(-0.4, 0.4, (n, 12)) * spread
    dof[:, :, 1] = rng.normal(0, 1.0 * spread, (n, 12))
    tau = rng.uniform(-60, 60, (n, 12))
    mu = np.repeat(rng.uniform(0.5, 1.25, (n, 1)), flat["ns"], axis=1)
    return root, dof, tau, mu


def hound_states(n, seed=0, spread=1.0):
    """Random Hound states: legs near a stand, arm anywhere in its limits, base tilted/moving."""
    rng = np.random.RandomState(seed)
    art, flat = hound()
    root = np.zeros((n, 13))
    root[:, 0:2] = rng.uniform(-2, 2, (n, 2))
    root[:, 2] = rng.uniform(0.45, 0.7, n)
    axis = rng.normal(size=(n, 3))
    axis /= np.linalg.norm(axis, axis=1, keepdims=True)
    ang = rng.uniform(0, 0.3 * spread, n)
    root[:, 3:6] = axis * np.sin(ang / 2)[:, None]
    root[:, 6] = np.cos(ang / 2)
    root[:, 7:10] = rng.normal(0, 0.3 * spread, (n, 3))
    root[:, 10:13] = rng.normal(0, 0.5 * spread, (n, 3))
    dof = np.zeros((n, 18, 2))
    leg = np.tile([0.0, 0.7, -1.4], 4)
    dof[:, :12, 0] = leg + rng.uniform(-0.3, 0.3, (n, 12)) * spread
    dof[:, 12:, 0] = rng.uniform(-1.5, 1.5, (n, 6))
    dof[:, :, 1] = rng.normal(0, 1.0 * spread, (n, 18))
    tau = np.concatenate([rng.uniform(-80, 80, (n, 12)), rng.uniform(-20, 20, (n, 6))], axis=1)
    mu = np.repeat(rng.uniform(0.5, 1.25, (n, 1)), flat["ns"], axis=1)
    return root, dof, tau, mu


def ant_states(n, seed=0, spread=1.0):
    """Random Ant states: near/on/into the ground, dofs anywhere in (and slightly beyond) their limits."""
    rng = np.random.RandomState(seed)
    art, flat = ant()
    lo, hi = flat["lower"], flat["upper"]
    root = np.zeros((n, 13))
    root[:, 0:2] = rng.uniform(-2, 2, (n, 2))
    root[:, 2] = rng.uniform(0.2, 0.6, n)
    axis = rng.normal(size=(n, 3))
    axis /= np.linalg.norm(axis, axis=1, keepdims=True)
    ang = rng.uniform(0, 0.4 * spread, n)
    root[:, 3:6] = axis * np.sin(ang / 2)[:, None]
    root[:, 6] = np.cos(ang / 2)
    root[:, 7:10] = rng.normal(0, 0.5 * spread, (n, 3))
    root[:, 10:13] = rng.normal(0, 1.0 * spread, (n, 3))
    dof = np.zeros((n, 8, 2))
    dof[:, :, 0] = rng.uniform(lo - 0.05, hi + 0.05, (n, 8))
    dof[:, :, 1] = rng.normal(0, 2.0 * spread, (n, 8))
    tau = rng.uniform(-15, 15, (n, 8))
    mu = np.full((n, flat["ns"]), 1.5)
    return root, dof, tau, mu


def anymal_states(n, seed=0, spread=1.0):
    """Random but physically plausible ANYmal states: standing, airborne, penetrating, tilted."""
    rng = np.random.RandomState(seed)
    art, flat = anymal()
    q0 = np.array([ANYMAL_DEFAULT[d] for d in art.dof_names()])
    root = np.zeros((n, 13))
    root[:, 0:2] = rng.uniform(-2, 2, (n, 2))
    root[:, 2] = rng.uniform(0.45, 0.65, n)
    axis = rng.normal(size=(n, 3))
    axis /= np.linalg.norm(axis, axis=1, keepdims=True)
    ang = rng.uniform(0, 0.25 * spread, n)
    root[:, 3:6] = axis * np.sin(ang / 2)[:, None]
    root[:, 6] = np.cos(ang / 2)
    root[:, 7:10] = rng.normal(0, 0.3 * spread, (n, 3))
    root[:, 10:13] = rng.normal(0, 0.5 * spread, (n, 3))
    dof = np.zeros((n, 12, 2))
    dof[:, :, 0] = q0 * rng.uniform(0.5, 1.5, (n, 12))
    dof[:, :, 1] = rng.normal(0, 1.0 * spread, (n, 12))
    tau = rng.uniform(-80, 80, (n, 12))
    mu = np.repeat(rng.uniform(0.5, 1.25, (n, 1)), flat["ns"], axis=1)
    return root, dof, tau, mu


def make_gpu_sim(kind: str, n: int, params: dict, terrain=None, host: bool = False, threads: int = 4, drives=None,
                 self_collide=None, asset_hook=None):
    """A libgymsim sim built through the drop-in gymapi (GPU pipeline); `terrain` (terrain_from_heights)
    adds the heightfield mesh with gym.add_triangle_mesh.  host=True builds the sim_device=cpu pipeline
    instead (physx.use_gpu False: libgymsim's host backend on `threads` threads, host tensors).
    drives = (mode [nd], stiffness [nd], damping [nd]) sets every actor's dof drive properties.
    asset_hook(asset) may edit the loaded asset's model (asset.flat) before the envs are created."""
    from isaacgymenv_amd.isaacgym import gymapi
    gym = gymapi.acquire_gym()
    sp = gymapi.SimParams()
    sp.dt = params["dt"]
    sp.substeps = params["substeps"]
    sp.up_axis = gymapi.UP_AXIS_Z
    sp.gravity = gymapi.Vec3(*params["gravity"])
    sp.use_gpu_pipeline = not host
    sp.physx.use_gpu = not host
    sp.physx.num_threads = threads
    sp.physx.num_position_iterations = params["pos_iters"]
    sp.physx.num_velocity_iterations = params["vel_iters"]
    sp.physx.contact_offset = params["contact_offset"]
    sp.physx.rest_offset = params["rest_offset"]
    sp.physx.max_depenetration_velocity = params["max_depen_vel"]
    sp.physx.contact_collection = gymapi.ContactCollection(params["collect_contacts"])
    # the oracle's parameter dicts mean PGS unless they say otherwise (gymapi's own default is TGS, as Isaac Gym's)
    sp.physx.solver_type = int(params.get("solver_type", 0))
    sim = gym.create_sim(0, -1, gymapi.SIM_PHYSX, sp)
    assert sim is not None
    if params.get("has_ground", 1):
        plane = gymapi.PlaneParams()
        plane.static_friction = params.get("ground_friction", 1.0)
        gym.add_ground(sim, plane)
    if terrain is not None:
        tm = gymapi.TriangleMeshParams()
        tm.nb_vertices = terrain["vertices"].shape[0]
        tm.nb_triangles = terrain["triangles"].shape[0]
        tm.transform.p = gymapi.Vec3(*terrain["shift"])
        tm.static_friction = terrain["friction"]
        gym.add_triangle_mesh(sim, terrain["vertices"].flatten(), terrain["triangles"].flatten(), tm)
    opts = gymapi.AssetOptions()
    sensors = []
    if kind == "anymal":
        opts.collapse_fixed_joints = True
        opts.replace_cylinder_with_capsule = True
        opts.default_dof_drive_mode = gymapi.DOF_MODE_EFFORT
        asset = gym.load_asset(sim, "/nonexistent", "urdf/anymal_c/urdf/anymal_minimal.urdf", opts)
    elif kind == "ant":
        opts.default_dof_drive_mode = gymapi.DOF_MODE_NONE
        opts.angular_damping = 0.0
        asset = gym.load_asset(sim, "/nonexistent", "mjcf/nv_ant.xml", opts)
        for b in ANT_FEET:
            gym.create_asset_force_sensor(asset, b, gymapi.Transform())
    elif kind == "hound":
        for k, v in HOUND_OPTS.items():
            setattr(opts, k, v)
        opts.default_dof_drive_mode = gymapi.DOF_MODE_EFFORT
        asset = gym.load_asset(sim, "/nonexistent", "urdf/UsefulHound/urdf/Hound.urdf", opts)
    elif kind == "hound_new":
        for k, v in HOUND_NEW_OPTS.items():
            setattr(opts, k, v)
        opts.default_dof_drive_mode = gymapi.DOF_MODE_NONE  # hound.py:171
        asset = gym.load_asset(sim, "/nonexistent", "urdf/Hound_new/Hound.urdf", opts)
    else:
        opts.fix_base_link = True
        asset = gym.load_asset(sim, "/nonexistent", "urdf/cartpole.urdf", opts)
    if asset_hook is not None:
        asset_hook(asset)
    for i in range(n):
        env = gym.create_env(sim, gymapi.Vec3(-1, -1, 0), gymapi.Vec3(1, 1, 1), 8)
        pose = gymapi.Transform()
        pose.p = gymapi.Vec3(0, 0, {"anymal": 0.62, "ant": 0.44, "hound": 0.55, "hound_new": 0.62}.get(kind, 2.0))
        a = gym.create_actor(env, asset, pose, kind, i, 0 if (SELF_COLLIDE[kind] if self_collide is None else self_collide)
                             else 1, 0)
        if drives is not None:
            props = gym.get_actor_dof_properties(env, a)
            props["driveMode"], props["stiffness"], props["damping"] = drives
            gym.set_actor_dof_properties(env, a, props)
    gym.prepare_sim(sim)
    return gym, sim


def make_host_sim(kind: str, n: int, params: dict, terrain=None, threads: int = 4, drives=None, self_collide=None,
                  asset_hook=None):
    return make_gpu_sim(kind, n, params, terrain=terrain, host=True, threads=threads, drives=drives,
                        self_collide=self_collide, asset_hook=asset_hook)


def heavy_base(flat, scale=1000.0):
    """ANYmal's base body (27.8 kg) made `scale` times heavier, inertia alike (a body above
    1000 kg must still rest on the plane)."""
    flat["mass"][0] *= scale
    flat["inertia"][0] *= scale
    flat["lmass"][0] *= scale


def upside_down_anymal(n):
    """ANYmal on its back: the base capsule (radius 0.1, axis x) 5 mm above the plane, legs up."""
    root = np.zeros((n, 13))
    root[:, 2] = 0.105
    root[:, 3] = 1.0  # quat xyzw (1, 0, 0, 0): 180 degrees about x
    dof = np.zeros((n, 12, 2))
    dof[:, :, 0] = [ANYMAL_DEFAULT[d] for d in ("LF_HAA", "LF_HFE", "LF_KFE", "LH_HAA", "LH_HFE", "LH_KFE",
                                                 "RF_HAA", "RF_HFE", "RF_KFE", "RH_HAA", "RH_HFE", "RH_KFE")]
    return root, dof


def sim_self_contacts(sim, mode=0):
    """The sim's self-contact pools from its current state (gs_debug_self_contacts): (contacts [n, npk, 10] float64
    = x xyz, n xyz, separation, friction, body a, body b -- the oracle's self_contacts layout; counts [n])."""
    import torch
    from isaacgymenv_amd.isaacgym import _lib
    n, npk = sim.num_envs, max(1, int(sim.asset.flat["npool"]))
    dev = sim.state.device
    out = torch.zeros((n, npk, 10), dtype=torch.float32, device=dev)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    stream = None if dev.type == "cpu" else torch.cuda.current_stream().cuda_stream
    _lib.check(_lib.lib().gs_debug_self_contacts(sim.handle, mode, out.data_ptr(), cnt.data_ptr(), stream),
               "gs_debug_self_contacts")
    return out.cpu().numpy().astype(np.float64), cnt.cpu().numpy()


def load_state_into(sim, root, dof, mu):
    """Write oracle-layout numpy state ([N,13] internal root, [N,nd,2]) into the SoA sim state."""
    import torch
    n, nd = root.shape[0], dof.shape[1]
    st = np.zeros((13 + 2 * nd, n), dtype=np.float32)
    st[0:13] = root.T
    st[13:13 + nd] = dof[:, :, 0].T
    st[13 + nd:] = dof[:, :, 1].T
    sim.state.copy_(torch.from_numpy(st))
    m = np.ones(tuple(sim.shape_mu.shape), dtype=np.float32)
    m[:mu.shape[1]] = mu.T
    sim.shape_mu.copy_(torch.from_numpy(m))


def read_state(sim, nd):
    st = sim.state.cpu().numpy().astype(np.float64)
    n = st.shape[1]
    root = st[0:13].T.copy()
    dof = np.ascontiguousarray(np.stack([st[13:13 + nd].T, st[13 + nd:].T], axis=-1))
    return root, dof


def terrain_from_heights(hf, hs=0.1, vs=0.005, slope_threshold=0.5, shift=(0.0, 0.0, 0.0), friction=1.0):
    """A heightfield as the trimesh gym.add_triangle_mesh receives it (terrain_utils layout, translated by
    `shift`) plus the oracle's terrain dict (world vertices, grid origin, spacing)."""
    from isaacgymenv_amd.isaacgym import terrain_utils
    v, t = terrain_utils.convert_heightfield_to_trimesh(np.asarray(hf, dtype=np.int16), hs, vs, slope_threshold)
    return mesh_terrain(v, t, hf.shape[0], hf.shape[1], hs, shift, friction)


def mesh_terrain(v, t, rows, cols, hs, shift=(0.0, 0.0, 0.0), friction=1.0):
    world = (v.astype(np.float64) + np.asarray(shift)).astype(np.float32)
    grid = v.reshape(rows, cols, 3)
    oracle = dict(vertices=world, rows=rows, cols=cols, x0=float(grid[0, :, 0].min()) + shift[0],
                  y0=float(grid[:, 0, 1].min()) + shift[1], hs=hs, friction=friction)
    return dict(vertices=v, triangles=t, shift=shift, friction=friction, oracle=oracle)


def rough_terrain(seed=0, rows=120, cols=120):
    """Stairs, blocks and a random field around the origin (cells of 0.1 m), centred on (0, 0)."""
    from isaacgymenv_amd.isaacgym import terrain_utils as tu
    np.random.seed(seed)
    hf = np.zeros((rows, cols), dtype=np.int16)
    a = tu.SubTerrain("a", width=rows // 2, length=cols, vertical_scale=0.005, horizontal_scale=0.1)
    tu.pyramid_stairs_terrain(a, step_width=0.31, step_height=0.08, platform_size=1.0)
    b = tu.SubTerrain("b", width=rows - rows // 2, length=cols, vertical_scale=0.005, horizontal_scale=0.1)
    tu.random_uniform_terrain(b, -0.06, 0.06, step=0.01, downsampled_scale=0.2)
    tu.discrete_obstacles_terrain(b, 0.1, 0.5, 1.0, 10, platform_size=0.5)
    hf[: rows // 2] = a.height_field_raw
    hf[rows // 2:] = b.height_field_raw
    return terrain_from_heights(hf, shift=(-rows * 0.05, -cols * 0.05, 0.0))


# per-field tolerances of one simulate (test_physics_gpu.py bounds) for assert_close_or_explained
STATE_TOL = {"pose": (2e-5, 0.0), "q": (2e-5, 0.0), "vel": (5e-3, 5e-3), "qd": (5e-3, 5e-3), "cf": (1.0, 2e-2),
             "sens": (0.09, 2e-2)}


def state_fields(root, dof, cf=None, sens=None):
    """The compared outputs of a simulate as {field: [n, ...]} (STATE_TOL keys)."""
    out = {"pose": root[:, 0:7], "vel": root[:, 7:13], "q": dof[:, :, 0], "qd": dof[:, :, 1]}
    if cf is not None:
        out["cf"] = cf
    if sens is not None:
        out["sens"] = sens
    return out


# an off-tolerance env counts as explained only when, field by field, its error is at most this multiple of the
# largest deviation the reference itself shows from fp32-rounding-sized perturbations of the same start
EXPLAIN_K = 2.0


def parity_report(line):
    """Print a parity report line and append it to $PARITY_REPORT when set (the GPU round scripts set it,
    so the reports of a GPU run are kept under profiles/)."""
    print(line)
    path = os.environ.get("PARITY_REPORT")
    if path:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "a") as f:
            f.write(line + "\n")


def parity_dump(name, **arrays):
    """On a failing parity check, keep its inputs and outputs for a CPU replay: an .npz under $PARITY_DUMP when set
    (the GPU round scripts point it into gpurun_out/, which comes back from the box)."""
    path = os.environ.get("PARITY_DUMP")
    if path:
        os.makedirs(path, exist_ok=True)
        np.savez_compressed(os.path.join(path, name + ".npz"), **arrays)


def _field_ratios(a, d, tol, n):
    """{field: [n]} -- per env, the largest |a - d| / (atol + rtol |d|) over the field's elements."""
    out = {}
    for k in d:
        at, rt = tol[k]
        dd = np.asarray(d[k], np.float64).reshape(n, -1)
        e = np.abs(np.asarray(a[k], np.float64).reshape(n, -1) - dd)
        out[k] = (e / (at + rt * np.abs(dd))).max(axis=1)
    return out


def oracle_run(flat, params, root, dof, tau, mu, bits=64, steps=1, nc=None, nsens=0, **kw):
    """The physics oracle (fp64, or bits=32: the same restatement compiled with float arithmetic) on copies of
    the inputs: returns float64 (root, dof, cf [n, nc, 3] or None, sens [n, nsens, 6] or None).  kw: OracleSim's
    sensor_bodies / terrain / drives and simulate's pos_targets / vel_targets."""
    from oracle.oracle import OracleSim
    dt = np.float64 if bits == 64 else np.float32
    c = lambda a: np.ascontiguousarray(a, dtype=dt)  # noqa: E731
    ctor = {k: kw[k] for k in ("sensor_bodies", "terrain", "drives") if k in kw}
    sim_kw = {k: c(kw[k]) for k in ("pos_targets", "vel_targets") if k in kw}
    o = OracleSim(flat, params, real_bits=bits, **ctor)
    n = root.shape[0]
    r, d = np.array(root, dtype=dt, order="C"), np.array(dof, dtype=dt, order="C")  # copies: stepped in place
    cf = np.zeros((n, nc, 3), dt) if nc else None
    sens = np.zeros((n, nsens, 6), dt) if nsens else None
    for _ in range(steps):
        o.simulate(r, d, c(tau), c(mu), cf, sens=sens, **sim_kw)
    f = lambda a: None if a is None else a.astype(np.float64)  # noqa: E731
    return f(r), f(d), f(cf), f(sens)


def assert_close_or_explained(actual, desired, rerun, tol=None, max_env_frac=0.02, tries=16, k=EXPLAIN_K, what=""):
    """Every env within tolerance, or its divergence explained by the reference's own sensitivity.

    `rerun(idx, rng)` returns the reference's outputs for envs idx started from a state perturbed at
    fp32-rounding size (same {field: [len(idx), ...]} layout as `desired`).  A rerun taking a third argument
    `bits` is also called with bits=32: the oracle restatement itself run in float arithmetic (oracle_run),
    which measures how far fp32 rounding carries through the spec where the dynamics is ill-conditioned
    (light links, joints at their velocity limits), not only where a contact switches.  For an env beyond
    tolerance, spread[field] is the largest deviation (in tolerance units) of those reruns (`tries` of each
    kind) from the unperturbed fp64 reference; the env is explained only when every field beyond tolerance
    has error <= k * spread[field].  At most `max_env_frac` of the envs may be beyond tolerance at all.  The
    report (worst env, off count, unexplained count, the least-explained envs) goes through parity_report."""
    import inspect
    fp32 = len(inspect.signature(rerun).parameters) >= 3
    tol = tol or STATE_TOL
    n = next(iter(desired.values())).shape[0]
    for f in desired:
        assert np.all(np.isfinite(np.asarray(actual[f], np.float64))), f"{what}: non-finite {f}"
    fr = _field_ratios(actual, desired, tol, n)
    r = np.max(np.stack(list(fr.values())), axis=0)
    off = np.nonzero(r > 1.0)[0]
    spread = {f: np.zeros(n) for f in desired}
    if off.size:
        rng = np.random.RandomState(0)
        sub = {f: np.asarray(v)[off] for f, v in desired.items()}
        for bits in ((64, 32) if fp32 else (64,)):
            for _ in range(tries):
                out = rerun(off, rng, bits) if fp32 else rerun(off, rng)
                pr = _field_ratios(out, sub, tol, off.size)
                for f in desired:
                    spread[f][off] = np.maximum(spread[f][off], pr[f])
    explained = np.ones(n, dtype=bool)
    margin = np.zeros(n)  # error / spread of the env's least-explained field
    for f in desired:
        beyond = fr[f] > 1.0
        m = np.where(beyond, fr[f] / np.maximum(spread[f], 1e-30), 0.0)
        margin = np.maximum(margin, m)
        explained &= ~beyond | (fr[f] <= k * spread[f])
    unexplained = off[~explained[off]]
    w = int(np.argmax(r))
    wf = max(fr, key=lambda f: fr[f][w])
    worst = sorted(off.tolist(), key=lambda i: -margin[i])[:5]
    detail = "; ".join(f"env {i}: {r[i]:.3g}x tol, error/spread {margin[i]:.3g}" for i in worst)
    report = (f"{what}: worst env {w} at {r[w]:.3g} x tolerance in {wf} (reference spread {spread[wf][w]:.3g}); "
              f"{off.size} of {n} envs beyond tolerance, {unexplained.size} unexplained "
              f"{unexplained[:8].tolist()} (rule: error <= {k:g} x spread per field, {tries} perturbed reruns"
              f"{' in fp64 and fp32' if fp32 else ''})"
              + (f"; least explained: {detail}" if off.size else ""))
    parity_report(report)
    assert unexplained.size == 0, report
    assert off.size <= max_env_frac * n, report
    return report


def perturbed(root, dof, idx, rng):
    """root[idx], dof[idx] with fp32-rounding-size noise on positions and velocities."""
    import numpy as np
    r, d = root[idx].copy(), dof[idx].copy()
    m = len(idx)
    r[:, :3] += rng.normal(0, 1e-6, (m, 3))
    r[:, 7:] += rng.normal(0, 1e-5, (m, 6))
    d[:, :, 0] += rng.normal(0, 1e-6, d[:, :, 0].shape)
    d[:, :, 1] += rng.normal(0, 1e-5, d[:, :, 1].shape)
    return r, d
