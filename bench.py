#!/usr/bin/env python3
"""Benchmark: AnymalTerrain VecTask.step throughput (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--num-envs 4096] [--no-cpu-baseline]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one ``VecTask.step(actions)`` of AnymalTerrain (default config:
terrainType plane, 4096 envs per GPU, seed 42 + rank) with synthetic uniform
actions in [-1, 1): 5 physics substeps (decimation 4 + controlFrequencyInv 1),
the post-physics tail, resets, observation noise.  Envs shard across ranks with
no data-path collective (weak scaling); the only collectives are the barrier and
the max-over-ranks of the timed region.

The rank-0 JSON line carries:
  roofline     -- the fused physics kernel (gs_sim_pd_step): SURVEY.md 8(d)'s algorithmic HBM
                  bytes of the env step per launch / its average HIP-event duration on the launch
                  stream (the kernel-scoped bytes beside it);
  cpu_baseline -- the product's CPU pipeline (sim_device=cpu pipeline=cpu: libgymsim's host
                  backend + the task's torch tail) stepping a bounded sample of the same workload
                  on every usable host CPU and on 4 threads;
  other_configs-- env-steps/s of the other BASELINE.json configs on one GPU (Ant 4096, AnymalTerrain
                  trimesh 4096, UsefulHound 4096), same timed-region rules, --other-steps steps each;
  ppo          -- PPO samples/s (the metric's second half): the rl_games-compatible learner
                  (isaacgymenv_amd/rl, AnymalTerrainPPO.yaml) over the same envs, one warm-up
                  epoch then --ppo-epochs timed epochs (rollout + GAE kernel + 5 x 6 minibatch
                  updates); with N ranks every minibatch all-reduces the 2.09 MB flat gradient
                  over RCCL.  value = horizon * envs * ranks * epochs / max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import isaacgymenv_amd  # noqa: E402,F401  (HIP runtime settings before the runtime initialises)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured float4 copy
FP32_VECTOR_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 (vector)


# algorithmic HBM bytes of one AnymalTerrain env step (plane), every mutable
# per-env buffer of the step read once and written once: reads 1,136 B (actions 48, root 52,
# dof_state 96, last_actions 48, last_dof_vel 48, commands 16, feet_air_time 16, progress 8,
# episode_sums 52, pre-drawn obs noise 752) + writes 1,298 B (obs 752, rew 4, reset 1, timeout 1,
# progress 8, root 52, dof_state 96, contact forces 156, torques 48, last_actions 48,
# last_dof_vel 48, feet_air_time 16, episode_sums 52, commands 16).
STEP_BYTES_PER_ENV = 2434


def physics_kernel_bytes_per_env(nd=12, nb=13, ns=9):
    """Kernel-scoped algorithmic HBM bytes one env moves through gs_sim_pd_step alone (DESIGN.md
    section 5), reported beside the step-scoped figure.

    reads : SoA state (13 + 2 nd) f32, actions nd, dof tensor (q, qd) 2 nd, shape friction ns
    writes: SoA state (13 + 2 nd), torques nd, dof tensor 2 nd, root tensor 13,
            contact forces SoA 3 nb + AoS 3 nb
    """
    state = 13 + 2 * nd
    reads = state + nd + 2 * nd + ns
    writes = state + nd + 2 * nd + 13 + 6 * nb
    return 4 * (reads + writes)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--num-envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="wall budget of the CPU baseline sample")
    ap.add_argument("--kernel-launches", type=int, default=50, help="launches timed for the roofline figure")
    ap.add_argument("--other-steps", type=int, default=100,
                    help="timed steps of each other BASELINE config (Ant, trimesh AnymalTerrain, UsefulHound); 0 = skip")
    ap.add_argument("--others", default="Ant,AnymalTerrain,UsefulHound",
                    help="comma list of the other configs to time (A/B runs of one of them)")
    ap.add_argument("--ppo-epochs", type=int, default=5,
                    help="timed PPO epochs (AnymalTerrainPPO.yaml: horizon 24 x envs samples each); 0 = skip")
    ap.add_argument("--physx-solver-type", type=int, default=None,
                    help="override task.sim.physx.solver_type for an A/B (default: the config's, TGS)")
    return ap.parse_args()


def host_cpu_info():
    """The host the CPU baseline ran on: logical CPUs (nproc), the CPUs this process may run on
    (affinity), the cgroup CPU quota, and the CPU model (lscpu's "Model name")."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(float(q) / float(per)))
    except (OSError, ValueError):
        pass
    info["cgroup_cpus"] = quota
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    info["model"] = model
    info["usable"] = min(x for x in (info["affinity"], quota) if x)
    return info


def cpu_baseline(num_envs: int, seconds: float):
    """The product's CPU pipeline (sim_device=cpu pipeline=cpu: libgymsim's host backend + the task's
    torch tail on the CPU) stepping the same AnymalTerrain workload, on every host CPU this process may
    use and, beside it, on 4 threads (the reference CPU pipeline's physx.num_threads: 4,
    cfg/config.yaml:30-32).  Bounded sample: ~`seconds` of stepping per thread count."""
    info = host_cpu_info()
    threads = info["usable"]
    main = _cpu_sample(num_envs, seconds, threads)
    four = _cpu_sample(num_envs, seconds / 2, 4) if threads != 4 else main
    main["sample"] += (f"; on 4 threads (reference PhysX CPU num_threads 4): {four['value']:.0f} env-steps/s; host: "
                       f"{info['model']}, nproc {info['nproc']}, affinity {info['affinity']} CPUs, cgroup quota "
                       f"{info['cgroup_cpus']} CPUs")
    main["threads4_value"] = four["value"]
    main["host"] = info
    return main


def _cpu_sample(num_envs: int, seconds: float, threads: int):
    """VecTask.step of AnymalTerrain (plane) on the CPU pipeline: physics in libgymsim's host backend on
    `threads` threads (physx.num_threads), the post-physics tail in torch on `threads` threads."""
    import torch
    import isaacgymenvs
    from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    vec_task.EXISTING_SIM = None
    try:
        env = isaacgymenvs.make(seed=42, task="AnymalTerrain", num_envs=num_envs, sim_device="cpu", rl_device="cpu",
                                graphics_device_id=-1, headless=True, force_render=False,
                                overrides=["pipeline=cpu", f"num_threads={threads}"])
        assert env.sim.host and env.sim.cparams.num_threads == threads
        gen = torch.Generator().manual_seed(1234)
        pool = torch.empty((16, env.num_envs, env.num_actions)).uniform_(-1.0, 1.0, generator=gen)
        env.reset()
        for i in range(2):
            env.step(pool[i])
        steps, t0 = 0, time.perf_counter()
        while True:
            env.step(pool[steps % 16])
            steps += 1
            el = time.perf_counter() - t0
            if el >= seconds and steps >= 3:
                break
    finally:
        torch.set_num_threads(prev)
        vec_task.EXISTING_SIM = None
    return {"value": num_envs * steps / el, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"product CPU pipeline (sim_device=cpu pipeline=cpu: libgymsim host backend, same solver "
                      f"source as the HIP kernels, + the AnymalTerrain torch tail): {num_envs} envs x {steps} "
                      f"VecTask.step calls (5 simulates each, tail included) in {el:.1f} s on {threads} threads"}


def timed_region(step, steps: int, warmup: int, world: int, sync=lambda: None) -> float:
    """W untimed steps, then exactly K timed steps bracketed by barrier + device sync on both
    sides; returns the MAX over ranks of the elapsed wall time (seconds)."""
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


FP32_MATRIX_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, 64 cyc/SIMD
FP16_MATRIX_PEAK_TFLOPS = 2500.0  # dense bf16/f16 MFMA


def ppo_leg(env, device, rank, world, epochs, task="AnymalTerrain"):
    import torch
    from isaacgymenv_amd.isaacgymenvs.config import compose
    from isaacgymenv_amd.rl import A2CAgent, PpoConfig
    train = compose("config", ["task=AnymalTerrain"])["train"]
    pcfg = PpoConfig.from_train_cfg(train, multi_gpu=world > 1)
    agent = A2CAgent(env, pcfg, device=device, seed=42 + rank)
    agent.env_reset()
    agent.train_epoch()  # warm-up: allocator, hipBLASLt heuristics, RCCL communicator; HIP graph capture
    # phase split of one (untimed) epoch, synchronised between the phases
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    returns, values = agent.play_steps()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    agent.model.train()
    agent.prepare_dataset(returns, values)
    for _ in range(pcfg.mini_epochs):
        for i in range(agent.num_minibatches):
            agent._run_minibatch(i)
    agent.model.eval()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    elapsed = timed_region(agent.train_epoch, epochs, 0, world, sync=torch.cuda.synchronize)
    samples = agent.batch_size * world * epochs
    st = agent.epoch_stats()
    # GEMM roofline of the two phases: 2*in*out flops per sample per Linear layer forward; the update
    # runs forward + backward (input and weight gradients: ~3x the forward) over every sample mini_epochs times
    fwd = sum(2 * m.in_features * m.out_features for m in agent.model.modules() if isinstance(m, torch.nn.Linear))
    roll_flops = fwd * agent.batch_size
    upd_flops = 3 * fwd * agent.batch_size * pcfg.mini_epochs
    roll_tf = roll_flops / (t1 - t0) / 1e12
    upd_tf = upd_flops / (t2 - t1) / 1e12
    gemm = {"flops_per_sample_forward": fwd,
            "rollout": {"flops": roll_flops, "achieved_tflops": roll_tf, "peak_tflops": FP32_MATRIX_PEAK_TFLOPS,
                        "frac": roll_tf / FP32_MATRIX_PEAK_TFLOPS, "dtype": "f32",
                        "note": "rollout time includes the env steps (VecTask.step x horizon)"},
            "update": {"flops": upd_flops, "achieved_tflops": upd_tf, "peak_tflops": FP16_MATRIX_PEAK_TFLOPS,
                       "frac": upd_tf / FP16_MATRIX_PEAK_TFLOPS, "dtype": "fp16 autocast"}}
    return {"metric": f"PPO samples/sec {task} (rl_games a2c_continuous, AnymalTerrainPPO.yaml)",
            "value": samples / elapsed, "unit": "samples/s", "epochs": epochs,
            "ms_per_epoch": 1e3 * elapsed / epochs, "samples_per_epoch": agent.batch_size * world,
            "rollout_ms": 1e3 * (t1 - t0), "update_ms": 1e3 * (t2 - t1),
            "minibatches_per_epoch": pcfg.mini_epochs * agent.num_minibatches,
            "allreduce_bytes_per_minibatch": agent.num_params * 4 if world > 1 else 0,
            "dtype": "f32 rollout, fp16 autocast update (mixed_precision: True)",
            "last_kl": st["kl"], "last_lr": st["lr"], "gemm_roofline": gemm}


OTHER_CONFIGS = [  # BASELINE.json configs beside the headline one (one GPU, 4096 envs each); the last field:
    # also time PPO on it (BASELINE config 3 is "AnymalTerrain + PPO, heightfield contacts")
    ("Ant", "Ant num_envs=4096 (MJCF articulation, flat-ground contacts, 1 simulate/step)", [], False),
    ("AnymalTerrain", "AnymalTerrain num_envs=4096 trimesh heightfield (5 simulates/step)",
     ["task.env.terrain.terrainType=trimesh"], True),
    ("UsefulHound", "UsefulHound num_envs=4096 (quadruped + 6-DoF arm OSC, 18 DoF, 24 links, 5 simulates/step)", [],
     False),
]


def other_config_leg(task, desc, overrides, num_envs, steps, warmup, device, rank, world, ppo_epochs=0):
    """env-steps/s of another BASELINE config (same timed-region rules) and the average duration of its
    physics launch (HIP events around gym.simulate on the launch stream)."""
    import torch
    import isaacgymenvs
    from isaacgymenv_amd.isaacgymenvs.tasks.base import vec_task
    vec_task.EXISTING_SIM = None
    env = isaacgymenvs.make(seed=42 + rank, task=task, num_envs=num_envs, sim_device=device, rl_device=device,
                            graphics_device_id=-1, headless=True, force_render=False, overrides=overrides)
    gen = torch.Generator(device=device)
    gen.manual_seed(4321 + rank)
    n_batches = max(1, min(steps + warmup, 256))
    pool = torch.empty((n_batches, env.num_envs, env.num_actions), device=device).uniform_(-1.0, 1.0, generator=gen)
    env.reset()
    it = [0]

    def step():
        env.step(pool[it[0] % n_batches])
        it[0] += 1

    elapsed = timed_region(step, steps, warmup, world, sync=torch.cuda.synchronize)
    stream = torch.cuda.current_stream(device)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    stream.synchronize()
    ev0.record(stream)
    for _ in range(20):
        env.gym.simulate(env.sim)
    ev1.record(stream)
    ev1.synchronize()
    out = {"task": task, "workload": desc, "value": env.num_envs * world * steps / elapsed, "unit": "env-steps/s",
           "steps": steps, "ms_per_step": 1e3 * elapsed / steps, "simulate_kernel_ms": ev0.elapsed_time(ev1) / 20,
           "kernel_variant": env.gym.amd_kernel_variant(env.sim)}
    if ppo_epochs > 0:
        out["ppo"] = ppo_leg(env, device, rank, world, ppo_epochs, task=f"{task} trimesh")
    del env, pool
    vec_task.EXISTING_SIM = None
    torch.cuda.empty_cache()
    return out


def main():
    # the driver reads ONE JSON line from rank 0's stdout: every other print (set_seed, rank banners,
    # the task layer) goes to stderr
    import contextlib
    out = sys.stdout
    with contextlib.redirect_stdout(sys.stderr):
        line = _main()
    if line is not None:
        print(json.dumps(line), file=out, flush=True)


def dist_setup(backend: str = "nccl"):
    """One process per GPU (torch.distributed.run sets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*): joins the
    process group when WORLD_SIZE > 1 -- "nccl" is RCCL over xGMI on the box; the CPU tests pass "gloo" -- and
    returns (world, rank, local_rank).  The env shards (num_envs per rank) are independent: the only collectives
    are the timed region's barrier / max-over-ranks and the PPO leg's gradient all-reduce."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    return world, rank, local_rank


def collective_info(world: int, ppo) -> dict:
    """What the N-rank run exchanges: the backend and world size of the process group, and the
    PPO learner's one flat-gradient all-reduce per minibatch (2,094,692 B for AnymalTerrainPPO's network)."""
    import torch.distributed as dist
    on = world > 1 and dist.is_initialized()
    return {"backend": (("rccl" if dist.get_backend() == "nccl" else dist.get_backend()) if on else None),
            "world_size": dist.get_world_size() if on else 1,
            "env_data_path": "none (num_envs shards per rank, no exchange; barrier + max-over-ranks time only)",
            "ppo_allreduce_bytes_per_minibatch": (ppo or {}).get("allreduce_bytes_per_minibatch")}


def _main():
    args = parse()
    import torch
    import torch.distributed as dist
    world, rank, local_rank = dist_setup()
    device = f"cuda:{local_rank}"

    import isaacgymenvs
    from isaacgymenv_amd.isaacgymenvs.utils.utils import set_seed
    set_seed(42, rank=rank)
    ov = [] if args.physx_solver_type is None else [f"task.sim.physx.solver_type={args.physx_solver_type}"]
    env = isaacgymenvs.make(seed=42 + rank, task="AnymalTerrain", num_envs=args.num_envs, sim_device=device,
                            rl_device=device, graphics_device_id=-1, headless=True, force_render=False, overrides=ov)
    N, A = env.num_envs, env.num_actions
    gen = torch.Generator(device=device)
    gen.manual_seed(1234 + rank)
    env.reset()
    # the synthetic policy output: distinct action batches generated up front and resident in HBM
    # (<= 1024 batches, cycled), so the timed region is VecTask.step alone
    n_batches = max(1, min(args.steps + args.warmup, 1024))
    pool = torch.empty((n_batches, N, A), device=device).uniform_(-1.0, 1.0, generator=gen)
    it = [0]

    def step():
        env.step(pool[it[0] % n_batches])
        it[0] += 1

    elapsed = timed_region(step, args.steps, args.warmup, world, sync=torch.cuda.synchronize)

    # ---- roofline of the dominant kernel: HIP events on the launch stream around each fused physics launch
    # of `kernel_launches` more VecTask.step calls (same workload as the timed region: the tail's resets keep
    # the state mix, so self-contacts and contact counts are the bench's own)
    stream = torch.cuda.current_stream(device)
    evs = []
    inner = env.fused_physics_step

    def timed_launch(actions):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        inner(actions)
        e1.record(stream)
        evs.append((e0, e1))

    env.fused_physics_step = timed_launch
    for _ in range(args.kernel_launches):
        step()
    env.fused_physics_step = inner
    torch.cuda.synchronize()
    assert len(evs) == args.kernel_launches, "the fused physics launch did not run once per step"
    kernel_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    variant = env.gym.amd_kernel_variant(env.sim)
    kernel_name = {1: "k_pd_step<Topo_anymal_c>", 2: "k_pd_step_team<Topo_anymal_c>"}.get(variant, str(variant))
    solver_type = int(env.sim.cparams.solver_type)
    solver = ("TGS" if solver_type == 1 and variant == 2 else "PGS") + f" (physx.solver_type {solver_type}, cfg/config.yaml:31)"
    # roofline basis: SURVEY.md 8(d)'s step-scoped algorithmic bytes (2,434 B per env step) per launch of
    # the dominant kernel; the kernel-scoped bytes (what gs_sim_pd_step alone moves) beside it
    bytes_per_launch = STEP_BYTES_PER_ENV * N
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
    kbytes_per_launch = physics_kernel_bytes_per_env() * N
    kachieved = kbytes_per_launch / (kernel_ms * 1e-3) / 1e9

    ppo = None
    if args.ppo_epochs > 0:
        ppo = ppo_leg(env, device, rank, world, args.ppo_epochs)
    others = []
    if args.other_steps > 0:
        del env
        for task, desc, ov, with_ppo in OTHER_CONFIGS:
            if task not in args.others.split(","):
                continue
            others.append(other_config_leg(task, desc, ov, args.num_envs, args.other_steps, 20, device, rank, world,
                                           ppo_epochs=min(args.ppo_epochs, 2) if with_ppo else 0))

    if rank == 0:
        traffic, traffic_note = None, None
        pmc = os.path.join(ROOT, "profiles", "pmc_pd_step.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                d = json.load(f)
            if d.get("num_envs") == N:
                traffic = d.get("hbm_bytes_per_launch")
                traffic_note = d.get("note")
        # secondary roofline (SURVEY.md 8d "report both"): counted FP32 VALU FLOPs of the same kernel
        valu = None
        vj = os.path.join(ROOT, "profiles", "valu_pd_step.json")
        if os.path.exists(vj):
            with open(vj) as f:
                d = json.load(f)
            if d.get("num_envs") == N:
                fl = d["fp32_flops_per_launch"]
                ach = fl / (kernel_ms * 1e-3) / 1e12
                valu = {"bound": "valu", "achieved": ach, "peak": FP32_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": ach / FP32_VECTOR_PEAK_TFLOPS, "flops_per_launch": fl,
                        "flops_per_env_step": d["fp32_flops_per_env_step"],
                        "valu_busy_frac": d["busy_frac_valu"], "wait_frac": d["wait_frac"]}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(N, args.cpu_seconds)
        total_env_steps = N * world * args.steps
        line = {
            "metric": "env-steps/sec AnymalTerrain 4096 envs/GPU",
            "value": total_env_steps / elapsed,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (uniform random actions in [-1,1) pre-generated in HBM, seed 1234+rank; random-init sim state via reset_idx)",
            "config": {"workload": "AnymalTerrain VecTask.step, terrainType plane (AnymalTerrain.yaml default), "
                                   "5 physics substeps/step, obs noise on",
                       "num_envs_per_gpu": N, "global_num_envs": N * world, "parallelism": f"dp{world}",
                       "solver": solver},
            "roofline": {"bound": "hbm", "kernel": f"gs_sim_pd_step ({kernel_name})",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_note": traffic_note, "kernel_ms": kernel_ms,
                         "bytes_per_launch": bytes_per_launch,
                         "basis": f"SURVEY.md 8(d): {STEP_BYTES_PER_ENV} B per env step x {N} envs per launch",
                         "kernel_scoped": {"bytes_per_launch": kbytes_per_launch, "achieved": kachieved,
                                           "frac": kachieved / HBM_PEAK_GBS,
                                           "basis": "gs_sim_pd_step's own reads + writes, DESIGN.md section 5"},
                         "valu": valu},
            "cpu_baseline": cpu,
            "ppo": ppo,
            "other_configs": others,
            "collective": collective_info(world, ppo),
        }
    else:
        line = None
    if world > 1:
        dist.destroy_process_group()
    return line


if __name__ == "__main__":
    main()
