"""Trimesh terrain on the GPU: the TERR physics kernels against the fp64 oracle's
mesh contacts (parity vs PhysX unpinned), and the trimesh AnymalTerrain task end to end."""
import numpy as np
import pytest
import torch

from oracle.oracle import OracleSim
from tests import helpers as H

pytestmark = pytest.mark.gpu


def _terrain_states(n, ter, seed):
    """Random ANYmal states placed just above the mesh under each base."""
    root, dof, tau, mu = H.anymal_states(n, seed=seed)
    rng = np.random.RandomState(seed + 100)
    root[:, 0] = rng.uniform(-5.0, 5.0, n)
    root[:, 1] = rng.uniform(-5.0, 5.0, n)
    v = ter["oracle"]["vertices"].reshape(-1, 3)
    for i in range(n):
        near = (np.abs(v[:, 0] - root[i, 0]) < 0.15) & (np.abs(v[:, 1] - root[i, 1]) < 0.15)
        root[i, 2] += v[near, 2].mean() + 0.05
    return root, dof, tau, mu


KERNELS = {"lane": 1, "team": 2}


def _gpu_vs_oracle(ter, n, seed, steps, kernel="team", solver="pgs"):
    art, flat = H.anymal()
    params = dict(H.ANYMAL_PARAMS, has_ground=0)
    root, dof, tau, mu = _terrain_states(n, ter, seed)
    gym, sim = H.make_gpu_sim("anymal", n, dict(params, solver_type=1 if solver == "tgs" else 0), terrain=ter)
    if solver == "tgs":
        params = dict(params, solver_type=3)  # the oracle's TGS restatement
    # mesh contacts: the lane team's TERR form (default) or the wave-assisted one-env-per-lane kernel
    assert sim.kernel_variant == KERNELS[kernel]
    H.load_state_into(sim, root, dof, mu)
    sim.dof_force.copy_(torch.from_numpy(tau.astype(np.float32).reshape(-1)))
    osim = OracleSim(flat, params, terrain=ter["oracle"])
    r, d = root.copy(), dof.copy()
    cf = np.zeros((n, flat["nb"], 3))
    for _ in range(steps):
        gym.simulate(sim)
        osim.simulate(r, d, np.ascontiguousarray(tau), mu, cf)
    torch.cuda.synchronize()
    g_root, g_dof = H.read_state(sim, 12)
    g_cf = sim.cf_soa.cpu().numpy().T.reshape(n, 13, 3)
    return g_root, g_dof, g_cf, r, d, cf


@pytest.mark.parametrize("kernel,solver", [("lane", "pgs"), ("team", "pgs"), ("lane", "tgs"), ("team", "tgs")])
def test_rough_terrain_one_simulate_matches_oracle(kernel, solver, monkeypatch):
    monkeypatch.setenv("GS_PHYSICS_KERNEL", kernel)
    ter = H.rough_terrain(seed=5)
    n = 512
    g_root, g_dof, g_cf, r, d, cf = _gpu_vs_oracle(ter, n, seed=2, steps=1, kernel=kernel, solver=solver)
    assert np.abs(cf).sum(axis=(1, 2)).astype(bool).mean() > 0.5, "most envs must touch the mesh"
    assert np.all(np.isfinite(g_root)) and np.all(np.isfinite(g_dof))
    # contact activity / closest-triangle choices can switch on a last-bit difference (stair edges): such an
    # env must be one the oracle itself moves under an fp32-sized perturbation
    art, flat = H.anymal()
    params = dict(H.ANYMAL_PARAMS, has_ground=0, solver_type=3 if solver == "tgs" else 0)
    root0, dof0, tau, mu = _terrain_states(n, ter, 2)

    def rerun(idx, rng, bits):
        rr, dd = H.perturbed(root0, dof0, idx, rng)
        rr, dd, c, _ = H.oracle_run(flat, params, rr, dd, tau[idx], mu[idx], bits, nc=flat["nb"], terrain=ter["oracle"])
        return H.state_fields(rr, dd, c)
    H.assert_close_or_explained(H.state_fields(g_root, g_dof, g_cf), H.state_fields(r, d, cf), rerun,
                                what=f"rough terrain gpu ({kernel} kernel, {solver.upper()})")


@pytest.mark.parametrize("kernel", sorted(KERNELS))
def test_flat_mesh_gpu_equals_plane_gpu(kernel, monkeypatch):
    """A flat mesh at z = 0 and the ground plane give the same step on the GPU too (frames, rows), in both kernel
    forms."""
    monkeypatch.setenv("GS_PHYSICS_KERNEL", kernel)
    from isaacgymenv_amd.isaacgym.terrain_utils import convert_heightfield_to_trimesh
    hf = np.zeros((121, 121), np.int16)
    ter = H.terrain_from_heights(hf, shift=(-6.0, -6.0, 0.0))
    n = 256
    root, dof, tau, mu = H.anymal_states(n, seed=6)
    root[:, 2] += 0.1

    def run(kind, r0, d0):
        p = dict(H.ANYMAL_PARAMS, has_ground=int(kind == "plane"))
        gym, sim = H.make_gpu_sim("anymal", n, p, terrain=ter if kind == "mesh" else None)
        H.load_state_into(sim, r0, d0, mu)
        sim.dof_force.copy_(torch.from_numpy(tau.astype(np.float32).reshape(-1)))
        for _ in range(3):
            gym.simulate(sim)
        torch.cuda.synchronize()
        r, d = H.read_state(sim, 12)
        return H.state_fields(r, d, sim.cf_soa.cpu().numpy().T.reshape(n, 13, 3))

    plane = run("plane", root, dof)
    mesh = run("mesh", root, dof)

    def rerun(idx, rng):
        r, d = root.copy(), dof.copy()
        r[idx], d[idx] = H.perturbed(root, dof, idx, rng)
        return {k: v[idx] for k, v in run("plane", r, d).items()}
    tol = {"pose": (1e-4, 1e-4), "vel": (1e-4, 1e-4), "q": (1e-3, 1e-3), "qd": (1e-3, 1e-3), "cf": (1.0, 1e-2)}
    H.assert_close_or_explained(mesh, plane, rerun, tol=tol, max_env_frac=5e-3,
                                what=f"flat mesh vs plane (3 substeps, {kernel} kernel)")


def test_anymal_trimesh_task_runs(monkeypatch):
    """AnymalTerrain with terrainType=trimesh (curriculum map, custom origins, height probes) on the GPU."""
    from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
    monkeypatch.setattr(vec_task, "EXISTING_SIM", None)
    import isaacgymenvs
    n = 512
    env = isaacgymenvs.make(seed=42, task="AnymalTerrain", num_envs=n, sim_device="cuda:0", rl_device="cuda:0",
                            headless=True, force_render=False,
                            overrides=["task.env.terrain.terrainType=trimesh", "task.env.terrain.numLevels=4",
                                       "task.env.terrain.numTerrains=8"])
    assert env.custom_origins and env.sim.kernel_variant == 2  # the lane team's TERR form
    gen = torch.Generator(device="cuda:0").manual_seed(3)
    falls = 0
    for t in range(300):
        a = 0.3 * (2 * torch.rand((n, 12), device="cuda:0", generator=gen) - 1)
        obs, rew, reset, extras = env.step(a)
        falls += int(reset.sum())
        if t % 50 == 0:
            assert torch.isfinite(obs["obs"]).all() and torch.isfinite(rew).all()
    h = env.measured_heights
    assert h.shape == (n, 140) and float(h.abs().max()) > 0.05, "height probes see the terrain"
    # bases stay above the terrain under them (no fall-through): probes around the base
    base_z = env.root_states[:, 2]
    assert float((base_z - h.max(dim=1).values > -0.2).float().mean()) > 0.95
    assert falls < 0.5 * n * 300 / 20


def test_anymal_trimesh_default_map_builds_and_steps(monkeypatch):
    """The full default trimesh map (AnymalTerrain.yaml: 10 levels x 20 terrains -> 1200 x 2000 samples,
    4.8 M triangles): the mesh passes the grid validation (spacing from the whole span, not a float32
    single-cell step) and the robots stand on it."""
    from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
    monkeypatch.setattr(vec_task, "EXISTING_SIM", None)
    import isaacgymenvs
    n = 256
    env = isaacgymenvs.make(seed=42, task="AnymalTerrain", num_envs=n, sim_device="cuda:0", rl_device="cuda:0",
                            headless=True, force_render=False, overrides=["task.env.terrain.terrainType=trimesh"])
    assert tuple(env.height_samples.shape) == (1200, 2000)
    zero = torch.zeros((n, 12), device="cuda:0")
    for _ in range(50):
        obs, rew, reset, extras = env.step(zero)
    assert torch.isfinite(obs["obs"]).all()
    h = env.measured_heights
    assert float((env.root_states[:, 2] - h.max(dim=1).values > -0.2).float().mean()) > 0.95


def test_measure_heights_kernel_matches_torch_get_heights():
    """gt_measure_heights against the reference's torch expression (sample_heights) on the same
    inputs: identical cell choice except on exact index ties."""
    from isaacgymenv_amd import gymtask
    from isaacgymenv_amd.isaacgymenvs.tasks.anymal_terrain import sample_heights
    dev = "cuda:0"
    g = torch.Generator(device="cpu").manual_seed(0)
    rows, cols, n, nh = 640, 800, 4096, 140
    hf = torch.randint(-300, 300, (rows, cols), generator=g, dtype=torch.int16).to(dev)
    root = torch.zeros(n, 13)
    root[:, 0] = torch.rand(n, generator=g) * 40 - 5
    root[:, 1] = torch.rand(n, generator=g) * 50 - 5
    root[:, 2] = torch.rand(n, generator=g)
    q = torch.randn(n, 4, generator=g)
    root[:, 3:7] = q / q.norm(dim=1, keepdim=True)
    root = root.to(dev)
    x = 0.1 * torch.tensor([-8, -7, -6, -5, -4, -3, -2, 2, 3, 4, 5, 6, 7, 8], device=dev)
    y = 0.1 * torch.tensor([-5, -4, -3, -2, -1, 1, 2, 3, 4, 5], device=dev)
    gx, gy = torch.meshgrid(x, y, indexing="ij")
    pts = torch.zeros(n, nh, 3, device=dev)
    pts[:, :, 0] = gx.flatten()
    pts[:, :, 1] = gy.flatten()
    out = torch.empty(n, nh, device=dev)
    rc = gymtask.lib().gt_measure_heights(hf.data_ptr(), rows, cols, 20.0, 0.1, 0.005, root.data_ptr(),
                                          pts.data_ptr(), n, nh, out.data_ptr(),
                                          torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    ref = sample_heights(hf, root[:, 3:7], root, pts, 20, 0.1, 0.005)
    torch.cuda.synchronize()
    mism = (out != ref).float().mean().item()
    assert mism < 1e-4, mism
    # edges of the map clip to the last interior cell
    assert torch.isfinite(out).all()


def test_terrain_query_matches_oracle():
    """Contact generation alone (gs_terrain.h vs the oracle's independent statement) over 200k random
    spheres around the rough mesh: found flag, separation and normal.  Float-vs-double differences may
    flip only exact ties (equidistant surfaces, the back-window edge, the contact_offset edge)."""
    from isaacgymenv_amd.isaacgym import _lib
    ter = H.rough_terrain(seed=5)
    art, flat = H.anymal()
    params = dict(H.ANYMAL_PARAMS, has_ground=0)
    gym, sim = H.make_gpu_sim("anymal", 1, params, terrain=ter)
    rng = np.random.RandomState(0)
    n = 200000
    o = ter["oracle"]
    grid = o["vertices"].reshape(o["rows"], o["cols"], 3)
    c = np.zeros((n, 3))
    c[:, 0] = rng.uniform(o["x0"] + 0.3, o["x0"] + (o["rows"] - 2) * o["hs"] - 0.3, n)
    c[:, 1] = rng.uniform(o["y0"] + 0.3, o["y0"] + (o["cols"] - 2) * o["hs"] - 0.3, n)
    gi = np.clip(np.round((c[:, 0] - o["x0"]) / o["hs"]).astype(int), 0, o["rows"] - 1)
    gj = np.clip(np.round((c[:, 1] - o["y0"]) / o["hs"]).astype(int), 0, o["cols"] - 1)
    c[:, 2] = grid[gi, gj, 2] + rng.uniform(-0.15, 0.2, n)
    r = rng.choice([0.03, 0.06, 0.1], n)
    cd = torch.from_numpy(c.astype(np.float32)).cuda()
    rd = torch.from_numpy(r.astype(np.float32)).cuda()
    out = torch.zeros(n, 5, device="cuda:0")
    _lib.check(_lib.lib().gs_debug_terrain_query(sim.handle, cd.data_ptr(), rd.data_ptr(), n, out.data_ptr(),
                                                 torch.cuda.current_stream().cuda_stream), "terrain query")
    g = out.cpu().numpy().astype(np.float64)
    osim = OracleSim(flat, params, terrain=o)
    ref = osim.terrain_query(c.astype(np.float32).astype(np.float64), r.astype(np.float32).astype(np.float64))
    found_g, found_o = g[:, 0] > 0.5, ref[:, 0] > 0.5
    assert found_o.mean() > 0.3
    flips = (found_g != found_o).mean()
    both = found_g & found_o
    dsep = np.abs(g[both, 1] - ref[both, 1])
    dn = np.abs(g[both, 2:5] - ref[both, 2:5]).max(axis=1)
    assert flips < 2e-4, flips
    assert (dsep > 1e-4).mean() < 5e-4, ((dsep > 1e-4).mean(), dsep.max())
    assert (dn > 1e-3).mean() < 5e-4, ((dn > 1e-3).mean(), dn.max())
