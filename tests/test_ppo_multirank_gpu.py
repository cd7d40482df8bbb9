"""The shipped multi-rank learner path, run on the GPU.

Two ranks as two processes on cuda:0 (RCCL refuses two ranks on one device, so the collectives are gloo's,
on the same CUDA tensors the RCCL path all-reduces).  Each rank runs A2CAgent with multi_gpu=True on its own
Cartpole env (seed 42 + rank, reference train.py:120-123): the first epoch eagerly (calc_gradients: local
gradient, flat all-reduce, optimizer step, KL all-reduce), then `_capture_graphs` builds the N-rank form --
three HIP graphs per minibatch around the gradient and KL all-reduces (rl/a2c_continuous.py _capture_graphs /
_run_minibatch) -- which epochs 2 and 3 replay.  Checked:
  * after every epoch the two ranks hold bit-identical parameters (rank 0's broadcast at construction plus
    the averaged gradient: reference AnymalTerrainPPO.yaml:51 multi_gpu, rl_games' gradient all-reduce);
  * in a replayed minibatch the all-reduced flat gradient is exactly the sum of the two ranks' local
    gradients, and the step applies their mean (the graph after the all-reduce divides by the world size);
  * the replayed graphs really are the three-graph form.
RCCL itself and the 8-GPU curve stay unmeasured here (the driver's multi-GPU run is the only 8-rank run).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

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
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import isaacgymenv_amd  # noqa: F401  (HIP runtime settings before the runtime initialises)
        from isaacgymenv_amd.isaacgymenvs.config import compose
        from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
        from isaacgymenv_amd.rl import A2CAgent, PpoConfig
        import isaacgymenvs
        vec_task.EXISTING_SIM = None
        cfg = compose("config", ["task=Cartpole"])
        env = isaacgymenvs.make(seed=42 + rank, task="Cartpole", num_envs=512, sim_device="cuda:0",
                                rl_device="cuda:0", headless=True, force_render=False)
        pcfg = PpoConfig.from_train_cfg(cfg["train"], multi_gpu=True)
        torch.manual_seed(100 + rank)  # different local init: the broadcast must make the ranks equal
        agent = A2CAgent(env, pcfg, device="cuda:0", seed=42 + rank)
        assert agent.multi_gpu and agent.world_size == world and agent.rank == rank
        flat = lambda: torch.cat([p.detach().reshape(-1) for p in agent.params]).cpu().numpy()  # noqa: E731
        params = [flat()]
        agent.train_epoch()  # eager, then _capture_graphs
        params.append(flat())
        forms = [len(g) for g in agent._mb_graphs]
        probe = {}
        orig = agent._run_minibatch

        def run_minibatch(i):
            if probe or i != 0:
                return orig(i)
            g1, g2, g3, kl = agent._mb_graphs[i]
            g1.replay()
            probe["local"] = agent.flat_grad.cpu().numpy().copy()
            dist.all_reduce(agent.flat_grad, op=dist.ReduceOp.SUM)
            probe["reduced"] = agent.flat_grad.cpu().numpy().copy()
            g2.replay()
            probe["applied"] = agent.flat_grad.cpu().numpy().copy()
            dist.all_reduce(kl, op=dist.ReduceOp.SUM)
            g3.replay()

        agent._run_minibatch = run_minibatch
        agent.train_epoch()  # replayed graphs around the all-reduces
        params.append(flat())
        agent._run_minibatch = orig
        agent.train_epoch()
        params.append(flat())
        torch.cuda.synchronize()
        q.put((rank, params, forms, probe, agent.epoch_stats()))
    except Exception as exc:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, None, None, traceback.format_exc() + repr(exc)))
    finally:
        dist.destroy_process_group()


def test_two_rank_learner_graphs_match_world_one_mean():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = {}
        for _ in range(world):
            r, params, forms, probe, stats = q.get(timeout=240)
            assert params is not None, stats
            res[r] = (params, forms, probe, stats)
    finally:
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    (p0, f0, pr0, s0), (p1, f1, pr1, s1) = res[0], res[1]
    assert f0 == f1 and all(f == 4 for f in f0), f0  # (g1, g2, g3, kl) per minibatch
    # the local inits differed; the broadcast at construction made them equal, every epoch keeps them equal
    for e, (a, b) in enumerate(zip(p0, p1)):
        np.testing.assert_array_equal(a, b, err_msg=f"parameters differ between ranks after epoch {e}")
    assert np.abs(p0[-1] - p0[0]).max() > 0, "the learner moved"
    # the replayed minibatch: all-reduced gradient = sum of the two ranks' local gradients (bit-exact for two
    # terms), and the graph after the all-reduce leaves their mean for the step
    assert np.abs(pr0["local"] - pr1["local"]).max() > 0, "ranks saw different experience"
    np.testing.assert_array_equal(pr0["reduced"], pr0["local"] + pr1["local"])
    np.testing.assert_array_equal(pr1["reduced"], pr0["reduced"])
    mean = (pr0["local"] + pr1["local"]) / np.float32(2.0)
    # (after the step the flat gradient buffer holds the mean the optimizer consumed -- clipping rescales
    # in the optimizer pass, not in the buffer)
    np.testing.assert_allclose(pr0["applied"], mean, rtol=1e-6, atol=0)
    assert np.isfinite(s0["kl"]) and abs(s0["kl"] - s1["kl"]) <= 1e-7 + 1e-5 * abs(s0["kl"])
