"""Replay of the r04f GPU failure: UsefulHound, random states seed 13 spread 0.5,
actions RandomState(2), the fused 4 x PD + 1 sequence, env 111 at error/spread 2.25.

CPU only (host backend = the same gs_solver.h / gs_pairs.h source as the kernels, and the fp64 / fp32 oracle):
  1. the whole 4 x PD + 1 sequence: host backend vs oracle, per field in tolerance units;
  2. substep by substep from the oracle's own trajectory: one substep of the host backend and of the fp32 oracle
     from the same fp64 start, against the fp64 oracle's next state (where does a single substep depart?);
  3. an ensemble of perturbed fp64 oracle runs (fp32-rounding-sized perturbations of the start): the
     distribution of each final field, the self-contact pool per substep along each run (which pair switches);
  4. where the host-backend run sits inside that distribution (rank / quantile).

    python tools/probes/hound_env111_replay.py [--env 111] [--ensemble 256] [--out profiles/r05_hound_env111.txt]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.oracle import OracleSim  # noqa: E402
from tests import helpers as H  # noqa: E402

KP, KD, SCALE, TLIM = 80.0, 2.0, 0.5, 80.0
DEFAULT = np.array([0.0, 0.7854, -1.5708] * 4 + [0.0] * 6)
TOL = dict(H.STATE_TOL, tau=(0.5, 1e-2))


def pd_torque(act, q, qd):
    return np.clip(KP * (SCALE * act + DEFAULT - q) - KD * qd, -TLIM, TLIM)


def oracle_traj(flat, root, dof, mu, act, bits=64, decimation=4, extra=1):
    """States after every substep of the 4 x PD + 1 sequence (the first torque from the start dof state, as
    the fused kernel's stale dof tensor equals it here), plus each substep's torque and the final contacts."""
    dt = np.float64 if bits == 64 else np.float32
    c = lambda a: np.array(a, dtype=dt, order="C")  # a copy: the oracle steps it in place  # noqa: E731
    sim = OracleSim(flat, H.HOUND_PARAMS, real_bits=bits)
    r, d, m = c(root), c(dof), c(mu)
    cf = np.zeros((root.shape[0], flat["nr"], 3), dt)
    states, taus, pools = [(r.astype(np.float64).copy(), d.astype(np.float64).copy())], [], []
    q, qd = d[:, :, 0].astype(np.float64).copy(), d[:, :, 1].astype(np.float64).copy()
    tau = None
    for i in range(decimation + extra):
        if i < decimation:
            tau = pd_torque(act, q, qd)
        pools.append(sim.self_contacts(r, d, m))
        taus.append(tau.copy())
        sim.simulate(r, d, c(tau), m, cf)
        q, qd = d[:, :, 0].astype(np.float64).copy(), d[:, :, 1].astype(np.float64).copy()
        states.append((r.astype(np.float64).copy(), d.astype(np.float64).copy()))
    return states, taus, cf.astype(np.float64), pools


def fields(root, dof, cf=None, tau=None):
    out = dict(pose=root[:, :7], vel=root[:, 7:], q=dof[:, :, 0], qd=dof[:, :, 1])
    if cf is not None:
        out["cf"] = cf
    if tau is not None:
        out["tau"] = tau
    return out


def ratios(a, d):
    n = next(iter(d.values())).shape[0]
    return H._field_ratios(a, d, TOL, n)


def host_full(n, root, dof, mu, act):
    gym, sim = H.make_host_sim("hound", n, H.HOUND_PARAMS, threads=4)
    H.load_state_into(sim, root, dof, mu)
    gym.refresh_dof_state_tensor(sim)
    torques = torch.empty((n, 18))
    gym.amd_pd_decimation_step(sim, torch.from_numpy(act.astype(np.float32)),
                               torch.from_numpy(DEFAULT.astype(np.float32)), KP, KD, SCALE, TLIM, 4, 1, torques)
    g_root, g_dof = H.read_state(sim, 18)
    return fields(g_root, g_dof, sim.contact_tensor.double().numpy().reshape(n, 24, 3), torques.double().numpy())


def host_one(n, root, dof, mu, tau):
    gym, sim = H.make_host_sim("hound", n, H.HOUND_PARAMS, threads=4)
    H.load_state_into(sim, root, dof, mu)
    sim.dof_force.copy_(torch.from_numpy(tau.astype(np.float32).reshape(-1)))
    gym.simulate(sim)
    return H.read_state(sim, 18)


def pool_sig(pool, e):
    cont, cnt = pool
    k = int(cnt[e])
    return tuple((int(cont[e, j, 8]), int(cont[e, j, 9])) for j in range(k)), cont[e, :k, 6].copy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", type=int, default=111)
    ap.add_argument("--ensemble", type=int, default=256)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    lines = []

    def say(s=""):
        print(s, flush=True)
        lines.append(s)

    n = 256
    art, flat = H.hound()
    root, dof, tau0, mu = H.hound_states(n, seed=13, spread=0.5)
    act = np.random.RandomState(2).uniform(-1.0, 1.0, (n, 18))
    e = a.env
    sl = slice(e, e + 1)
    states, taus, cf, pools = oracle_traj(flat, root[sl], dof[sl], mu[sl], act[sl])
    ref = fields(*states[-1], cf, taus[-1])

    # 1. the whole sequence on the host backend (all 256 envs, as the GPU test ran)
    hf = host_full(n, root, dof, mu, act)
    hf_e = {k: v[sl] for k, v in hf.items()}
    r = ratios(hf_e, ref)
    say(f"env {e}: 4 x PD + 1, host backend vs fp64 oracle (tolerance units): "
        + ", ".join(f"{k} {float(v[0]):.3g}" for k, v in r.items()))
    s32, t32, cf32, _ = oracle_traj(flat, root[sl], dof[sl], mu[sl], act[sl], bits=32)
    r32 = ratios(fields(*s32[-1], cf32, t32[-1]), ref)
    say(f"env {e}: 4 x PD + 1, fp32 oracle vs fp64 oracle: " + ", ".join(f"{k} {float(v[0]):.3g}" for k, v in r32.items()))

    # 2. substep by substep from the fp64 trajectory
    say("")
    say("substep-by-substep (one substep from the fp64 oracle's own state k, against its state k+1):")
    for k in range(5):
        r0, d0 = states[k]
        rr, dd = states[k + 1]
        want = fields(rr, dd)
        hr, hd = host_one(1, r0, d0, mu[sl], taus[k])
        o32 = OracleSim(flat, H.HOUND_PARAMS, real_bits=32)
        c = lambda x: np.ascontiguousarray(x, dtype=np.float32)  # noqa: E731
        r32_, d32_ = c(r0), c(d0)
        o32.simulate(r32_, d32_, c(taus[k]), c(mu[sl]))
        rh = ratios(fields(hr, hd), want)
        ro = ratios(fields(r32_.astype(np.float64), d32_.astype(np.float64)), want)
        sig, sep = pool_sig(pools[k], 0)
        say(f"  substep {k}: host {max(float(v[0]) for v in rh.values()):.3g} "
            f"({', '.join(f'{f} {float(v[0]):.2g}' for f, v in rh.items())}); fp32 oracle "
            f"{max(float(v[0]) for v in ro.values()):.3g}; self pool {sig} sep {np.round(sep * 1e3, 3).tolist()} mm")

    # 3. perturbed fp64 ensemble
    say("")
    rng = np.random.RandomState(0)
    ens = []
    sigs = {}
    for t in range(a.ensemble):
        pr, pd = H.perturbed(root[sl], dof[sl], np.array([0]), rng)
        st, ta, c_, pl = oracle_traj(flat, pr, pd, mu[sl], act[sl])
        ens.append(ratios(fields(*st[-1], c_, ta[-1]), ref))
        key = tuple(pool_sig(p, 0)[0] for p in pl)
        sigs.setdefault(key, []).append(t)
    say(f"perturbed fp64 oracle ensemble ({a.ensemble} runs, positions 1e-6, velocities 1e-5): deviation from the "
        "unperturbed run in tolerance units")
    for f in ref:
        v = np.array([float(x[f][0]) for x in ens])
        rank = float((v < float(r[f][0])).mean())
        say(f"  {f:5s}: median {np.median(v):.3g}, p90 {np.quantile(v, 0.9):.3g}, max of first 16 "
            f"{v[:16].max():.3g}, max {v.max():.3g}; host backend {float(r[f][0]):.3g} (quantile {rank:.3f}); "
            f"fp32 oracle {float(r32[f][0]):.3g}")
    say(f"distinct self-contact pool sequences over the 5 substeps: {len(sigs)}")
    for key, runs in sorted(sigs.items(), key=lambda kv: -len(kv[1]))[:6]:
        say(f"  {len(runs):4d} runs: " + " | ".join(str(s) for s in key))
    say(f"unperturbed: " + " | ".join(str(pool_sig(p, 0)[0]) for p in pools))
    if a.out:
        with open(a.out, "w") as fh:
            fh.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
