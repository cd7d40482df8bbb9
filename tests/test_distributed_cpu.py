"""Multi-rank path on CPU (gloo, world_size 2): env sharding is independent per rank (seed + rank,
no data-path collective) and bench.py's timed region takes the max over ranks."""
import copy
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from isaacgymenv_amd.isaacgym import gymapi
    from tests.fakegym import FakeGym
    fake = FakeGym()
    gymapi.acquire_gym = lambda: fake
    from isaacgymenv_amd.isaacgymenvs.utils.utils import set_seed
    from isaacgymenv_amd.isaacgymenvs.tasks.anymal_terrain import AnymalTerrain
    import bench
    d = np.load(os.path.join(ROOT, "tests", "golden", "anymal_terrain.npz"))
    cfg = yaml.safe_load(str(d["cfg_yaml"]))
    seed = set_seed(42, rank=rank)
    env = AnymalTerrain(copy.deepcopy(cfg), "cpu", "cpu", -1, True, False, False)
    a = torch.zeros(env.num_envs, 12)

    def step():
        env.step(a)
        if rank == 1:
            import time
            time.sleep(0.01)  # uneven ranks: the max must be the slow one

    el = bench.timed_region(step, 5, 1, world)
    q.put((rank, seed, el, env.commands.clone().numpy()))
    dist.destroy_process_group()


def test_two_rank_gloo_shards_and_timing():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda x: x[0])
    (r0, s0, t0, c0), (r1, s1, t1, c1) = res
    assert (s0, s1) == (42, 43)                      # seed + rank (train.py:120-123)
    assert not np.allclose(c0, c1)                   # independent shards draw different commands
    assert t0 == t1 and t0 >= 5 * 0.01               # both ranks report the max (the slow rank)


def test_multi_gpu_env_creator_maps_local_rank(monkeypatch):
    from isaacgymenv_amd.isaacgymenvs.utils import rlgames_utils
    from isaacgymenv_amd.isaacgymenvs import tasks
    seen = {}

    class Dummy:
        def __init__(self, cfg, rl_device, sim_device, **kw):
            seen.update(cfg=cfg, rl=rl_device, sim=sim_device)

    monkeypatch.setitem(tasks.isaacgym_task_map, "Dummy", Dummy)
    monkeypatch.setenv("LOCAL_RANK", "3")
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("WORLD_SIZE", "8")
    cfg = {}
    rlgames_utils.get_rlgames_env_creator(0, cfg, "Dummy", "cuda:0", "cuda:0", -1, True, multi_gpu=True)()
    assert seen["sim"] == "cuda:3" and seen["rl"] == "cuda:3" and cfg["rank"] == 3


def _bench_setup_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    import bench
    w, r, lr = bench.dist_setup("gloo")  # bench.py's own N-rank setup (the box passes "nccl" = RCCL)
    el = bench.timed_region(lambda: __import__("time").sleep(0.002 * (1 + r)), 4, 1, w)
    ppo = {"allreduce_bytes_per_minibatch": 2094692}
    info = bench.collective_info(w, ppo)
    q.put((r, w, lr, el, info))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_bench_rank_setup_and_collective_report(world):
    """bench.py's _main N-rank handling on CPU (gloo): RANK / LOCAL_RANK / WORLD_SIZE from torch.distributed.run's
    environment, the max-over-ranks timed region, and the collective report of the JSON line (VERDICT r05 item 8:
    the world size the process group really has, the PPO all-reduce bytes per minibatch)."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_setup_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r for r, *_ in res] == list(range(world))
    assert all(w == world and lr == r for r, w, lr, _, _ in res)
    els = {el for *_, el, _ in res}
    assert len(els) == 1 and els.pop() >= 4 * 0.002 * world  # every rank reports the slowest rank's time
    info = res[0][4]
    assert info["backend"] == "gloo" and info["world_size"] == world
    assert info["ppo_allreduce_bytes_per_minibatch"] == 2094692
