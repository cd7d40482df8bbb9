"""Our task layer (CPU pipeline, torch tail) vs golden fixtures produced by the REFERENCE's code.

Both sides run on tests/fakegym.FakeGym with the same seed, config and actions
(tests/golden/make_golden.py).  Integer/bool outputs (done masks, timeouts,
progress) must be identical; floats within 1e-5 relative.  A match also proves
the torch RNG call order (friction buckets, terrain levels, reset draws, push,
observation noise) is the reference's.
"""
import copy
import os

import numpy as np
import pytest
import torch
import yaml

from isaacgymenv_amd.isaacgym import gymapi
from tests.fakegym import FakeGym

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture
def fake_gym(monkeypatch):
    holder = {}

    def install(fake):
        holder["fake"] = fake
        monkeypatch.setattr(gymapi, "acquire_gym", lambda: fake)
        from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
        monkeypatch.setattr(vec_task, "EXISTING_SIM", None)
        return fake

    return install


def _close(a, b, what, rtol=1e-5, atol=1e-6):
    np.testing.assert_allclose(np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64), rtol=rtol, atol=atol,
                               err_msg=what)


def test_anymal_terrain_matches_reference(fake_gym):
    d = np.load(os.path.join(GOLDEN, "anymal_terrain.npz"))
    fake_gym(FakeGym())
    from isaacgymenv_amd.isaacgymenvs.tasks.anymal_terrain import AnymalTerrain
    cfg = yaml.safe_load(str(d["cfg_yaml"]))
    torch.manual_seed(42)
    env = AnymalTerrain(copy.deepcopy(cfg), "cpu", "cpu", -1, True, False, False)
    _close(env.commands.numpy(), d["init_commands"], "commands after the initial reset (RNG order at init)")
    _close(env.dof_state.numpy(), d["init_dof_state"], "dof state after the initial reset")
    np.testing.assert_array_equal(env.feet_indices.numpy(), d["feet_indices"])
    np.testing.assert_array_equal(env.knee_indices.numpy(), d["knee_indices"])
    _close(env.noise_scale_vec.numpy(), d["noise_scale_vec"], "noise scale vector")
    terms = [str(t) for t in d["terms"]]
    for t in range(d["actions"].shape[0]):
        obs, rew, reset, extras = env.step(torch.from_numpy(d["actions"][t]))
        assert reset.dtype == torch.bool
        np.testing.assert_array_equal(reset.numpy().astype(np.int64), d["reset"][t], err_msg=f"reset step {t}")
        np.testing.assert_array_equal(extras["time_outs"].numpy().astype(np.int64), d["time_outs"][t])
        np.testing.assert_array_equal(env.progress_buf.numpy(), d["progress"][t], err_msg=f"progress step {t}")
        _close(rew.numpy(), d["rew"][t], f"reward step {t}")
        _close(obs["obs"].numpy(), d["obs"][t], f"obs step {t}")
        _close(env.commands.numpy(), d["commands"][t], f"commands step {t}")
        _close(env.feet_air_time.numpy(), d["feet_air_time"][t], f"feet air time step {t}")
        _close(np.stack([env.episode_sums[k].numpy() for k in terms]), d["episode_sums"][t], f"episode sums {t}")
        if d["ep_mask"][t]:
            got = np.array([float(extras["episode"]["rew_" + k]) for k in terms] +
                           [float(extras["episode"]["terrain_level"])])
            _close(got, d["ep_extras"][t], f"extras episode step {t}", rtol=1e-5, atol=1e-7)


def test_anymal_terrain_long_matches_reference(fake_gym):
    """Default pushInterval_s (push at step 749) and episodeLength_s (done at progress 999 -> step 998),
    64 envs x 1010 steps on the fake, compared at the fixture's stored steps (make_golden.KEEP_LONG)."""
    d = np.load(os.path.join(GOLDEN, "anymal_terrain_long.npz"))
    fake_gym(FakeGym(base_contact_p=2e-5))  # make_golden.LONG_FAKE
    from isaacgymenv_amd.isaacgymenvs.tasks.anymal_terrain import AnymalTerrain
    cfg = yaml.safe_load(str(d["cfg_yaml"]))
    assert cfg["env"]["learn"]["pushInterval_s"] == 15 and cfg["env"]["learn"]["episodeLength_s"] == 20
    torch.manual_seed(42)
    env = AnymalTerrain(copy.deepcopy(cfg), "cpu", "cpu", -1, True, False, False)
    steps = [int(x) for x in d["steps"]]
    assert 749 in steps and 998 in steps and steps[-1] >= 1000
    rng = np.random.RandomState(7)
    actions = (2 * rng.rand(steps[-1] + 1, env.num_envs, 12) - 1).astype(np.float32)
    np.testing.assert_array_equal(actions[steps], d["actions"])
    terms = [str(t) for t in d["terms"]]
    pos = {s_: i for i, s_ in enumerate(steps)}
    for t in range(steps[-1] + 1):
        env.extras.pop("episode", None)
        obs, rew, reset, extras = env.step(torch.from_numpy(actions[t]))
        if t not in pos:
            continue
        i = pos[t]
        np.testing.assert_array_equal(reset.numpy().astype(np.int64), d["reset"][i], err_msg=f"reset step {t}")
        np.testing.assert_array_equal(extras["time_outs"].numpy().astype(np.int64), d["time_outs"][i])
        np.testing.assert_array_equal(env.progress_buf.numpy(), d["progress"][i], err_msg=f"progress step {t}")
        _close(rew.numpy(), d["rew"][i], f"reward step {t}")
        _close(obs["obs"].numpy(), d["obs"][i], f"obs step {t}")
        _close(env.commands.numpy(), d["commands"][i], f"commands step {t}")
        _close(np.stack([env.episode_sums[k].numpy() for k in terms]), d["episode_sums"][i], f"episode sums {t}")
        if d["ep_mask"][i]:
            got = np.array([float(extras["episode"]["rew_" + k]) for k in terms] +
                           [float(extras["episode"]["terrain_level"])])
            _close(got, d["ep_extras"][i], f"extras episode step {t}", rtol=1e-5, atol=1e-7)
    # the envs still in their first episode reset at progress 999 = step 998 (anymal_terrain.py:299)
    first = d["progress"][pos[997]] == 998
    assert first.sum() > 32 and d["reset"][pos[998]][first].all() and not d["time_outs"][pos[998]].any()


def test_cartpole_matches_reference(fake_gym):
    d = np.load(os.path.join(GOLDEN, "cartpole.npz"))
    fake_gym(FakeGym(seed=777, dof_drift=1.0))
    from isaacgymenv_amd.isaacgymenvs.tasks.cartpole import Cartpole
    cfg = yaml.safe_load(str(d["cfg_yaml"]))
    torch.manual_seed(42)
    env = Cartpole(copy.deepcopy(cfg), "cpu", "cpu", -1, True, False, False)
    for t in range(d["actions"].shape[0]):
        obs, rew, reset, extras = env.step(torch.from_numpy(d["actions"][t]))
        assert reset.dtype == torch.int64
        np.testing.assert_array_equal(reset.numpy(), d["reset"][t], err_msg=f"reset step {t}")
        np.testing.assert_array_equal(extras["time_outs"].numpy().astype(np.int64), d["time_outs"][t])
        _close(obs["obs"].numpy(), d["obs"][t], f"obs step {t}")
        _close(rew.numpy(), d["rew"][t], f"reward step {t}")


def test_ant_matches_reference(fake_gym):
    d = np.load(os.path.join(GOLDEN, "ant.npz"))
    fake_gym(FakeGym(seed=4242, dof_drift=2.0, z_drift=0.02))
    from isaacgymenv_amd.isaacgymenvs.tasks.ant import Ant
    cfg = yaml.safe_load(str(d["cfg_yaml"]))
    torch.manual_seed(42)
    env = Ant(copy.deepcopy(cfg), "cpu", "cpu", -1, True, False, False)
    _close(env.joint_gears.numpy(), d["joint_gears"], "motor gears from the MJCF actuators")
    _close(env.dof_limits_lower.numpy(), d["dof_limits_lower"], "ordered lower limits")
    _close(env.dof_limits_upper.numpy(), d["dof_limits_upper"], "ordered upper limits")
    _close(env.initial_dof_pos.numpy(), d["initial_dof_pos"], "initial dof positions")
    _close(env.initial_root_states.numpy(), d["initial_root_states"], "initial root states")
    np.testing.assert_array_equal(env.extremities_index.numpy(), d["extremities_index"])
    assert d["reset"].sum() > 10 and d["time_outs"].sum() > 0, "fixture must hold falls and timeouts"
    for t in range(d["actions"].shape[0]):
        obs, rew, reset, extras = env.step(torch.from_numpy(d["actions"][t]))
        assert reset.dtype == torch.int64
        np.testing.assert_array_equal(reset.numpy(), d["reset"][t], err_msg=f"reset step {t}")
        np.testing.assert_array_equal(extras["time_outs"].numpy().astype(np.int64), d["time_outs"][t])
        np.testing.assert_array_equal(env.progress_buf.numpy(), d["progress"][t], err_msg=f"progress step {t}")
        _close(obs["obs"].numpy(), d["obs"][t], f"obs step {t}")
        _close(rew.numpy(), d["rew"][t], f"reward step {t}")
        _close(env.potentials.numpy(), d["potentials"][t], f"potentials step {t}")
        _close(env.prev_potentials.numpy(), d["prev_potentials"][t], f"previous potentials step {t}")
        _close(extras["true_objective"].numpy(), d["true_objective"][t], f"true objective step {t}")
        _close(env.dof_state.numpy(), d["dof_state"][t], f"dof state step {t}")
        _close(env.root_states.numpy(), d["root_states"][t], f"root states step {t}")


def test_anymal_trimesh_matches_reference(fake_gym):
    """Trimesh AnymalTerrain: terrain map, custom origins, curriculum levels,
    height probes and the 188-wide observation against the reference's own task code (both on
    our terrain_utils restatement, since Isaac Gym's is absent)."""
    d = np.load(os.path.join(GOLDEN, "anymal_trimesh.npz"))
    fake_gym(FakeGym(seed=99, xy_drift=0.25))
    from isaacgymenv_amd.isaacgymenvs.tasks.anymal_terrain import AnymalTerrain
    cfg = yaml.safe_load(str(d["cfg_yaml"]))
    np.random.seed(42)
    torch.manual_seed(42)
    env = AnymalTerrain(copy.deepcopy(cfg), "cpu", "cpu", -1, True, False, False)
    np.testing.assert_array_equal(env.height_samples.numpy(), d["height_samples"])
    _close(env.terrain_origins.numpy(), d["terrain_origins"], "terrain origins")
    _close(env.env_origins.numpy(), d["init_env_origins"], "env origins at init")
    _close(env.root_states.numpy(), d["init_root_states"], "root states after the initial reset")
    np.testing.assert_array_equal(env.terrain_levels.numpy(), d["init_levels"])
    np.testing.assert_array_equal(env.terrain_types.numpy(), d["init_types"])
    assert len(set(d["levels"][-1].tolist())) > 1 and d["reset"].sum() > 0
    for t in range(d["actions"].shape[0]):
        obs, rew, reset, extras = env.step(torch.from_numpy(d["actions"][t]))
        np.testing.assert_array_equal(reset.numpy().astype(np.int64), d["reset"][t], err_msg=f"reset step {t}")
        np.testing.assert_array_equal(env.terrain_levels.numpy(), d["levels"][t], err_msg=f"levels step {t}")
        _close(env.env_origins.numpy(), d["env_origins"][t], f"env origins step {t}")
        _close(env.measured_heights.numpy(), d["heights"][t], f"heights step {t}")
        _close(env.root_states.numpy(), d["root_states"][t], f"root states step {t}")
        _close(obs["obs"].numpy(), d["obs"][t], f"obs step {t}")
        _close(rew.numpy(), d["rew"][t], f"reward step {t}")


def test_useful_hound_matches_reference(fake_gym):
    """UsefulHound: 24 links with kept fixed joints, link indices, arm OSC
    torques over the Jacobian / mass matrix, termination on trunk, thigh and shoulder contacts, the
    204-wide observation and the RNG order, against the reference's own task code on the fake."""
    d = np.load(os.path.join(GOLDEN, "useful_hound.npz"))
    fake_gym(FakeGym(seed=555))
    from isaacgymenv_amd.isaacgymenvs.tasks.useful_hound import UsefulHound
    cfg = yaml.safe_load(str(d["cfg_yaml"]))
    torch.manual_seed(42)
    env = UsefulHound(copy.deepcopy(cfg), "cpu", "cpu", -1, True, False, False)
    _close(env.commands.numpy(), d["init_commands"], "commands after the initial reset (RNG order at init)")
    _close(env.dof_state.numpy(), d["init_dof_state"], "dof state after the initial reset")
    _close(env.root_states.numpy(), d["init_root_states"], "root states after the initial reset")
    for k in ("feet_indices", "knee_indices", "base_indices"):
        np.testing.assert_array_equal(getattr(env, k).numpy(), d[k], err_msg=k)
    assert env.eef_index == int(d["eef_index"])
    _close(env.noise_scale_vec.numpy(), d["noise_scale_vec"], "noise scale vector")
    _close(env.houndarm_dof_lower_limits.numpy(), d["arm_lower"], "arm lower limits")
    _close(env.houndarm_dof_upper_limits.numpy(), d["arm_upper"], "arm upper limits")
    _close(env._houndarm_effort_limits.numpy(), d["arm_effort"], "arm effort limits")
    terms = [str(t) for t in d["terms"]]
    assert d["reset"].sum() > 0
    for t in range(d["actions"].shape[0]):
        obs, rew, reset, extras = env.step(torch.from_numpy(d["actions"][t]))
        assert reset.dtype == torch.bool
        np.testing.assert_array_equal(reset.numpy().astype(np.int64), d["reset"][t], err_msg=f"reset step {t}")
        np.testing.assert_array_equal(extras["time_outs"].numpy().astype(np.int64), d["time_outs"][t])
        np.testing.assert_array_equal(env.progress_buf.numpy(), d["progress"][t], err_msg=f"progress step {t}")
        _close(env.torques.numpy(), d["torques"][t], f"torques (legs PD + arm OSC) step {t}", rtol=1e-4, atol=1e-4)
        _close(env.dof_state.numpy(), d["dof_state"][t], f"dof state step {t}")
        _close(env.commands.numpy(), d["commands"][t], f"commands step {t}")
        _close(env.feet_air_time.numpy(), d["feet_air_time"][t], f"feet air time step {t}")
        _close(obs["obs"].numpy(), d["obs"][t], f"obs step {t}")
        _close(rew.numpy(), d["rew"][t], f"reward step {t}")
        ep = extras.get("episode")
        assert int(ep is not None) == int(d["ep_mask"][t])
        if ep is not None:
            got = [float(ep["rew_" + k]) for k in terms] + [float(ep["terrain_level"])]
            _close(got, d["ep_extras"][t], f"episode extras step {t}")
        env.extras.pop("episode", None)
