"""The oracle's TGS restatement the lane team's TGS is checked against (solver_type 3) stays stable where plain
sub-step push-out (solver_type 1) diverged (profiles/r04_tgs_divergence.txt, profiles/r05_tgs_study.json): a short
locomotion rollout under random actions keeps every env finite and the feet out of the ground."""
import numpy as np

from oracle.oracle import OracleSim
from tests import helpers as H


def test_oracle_tgs_locomotion_rollout_is_stable():
    import tools.tgs_study as S
    art, flat = H.anymal()
    n, steps = 16, 40
    root, dof, mu, default = S.start_states(art, flat, n, seed=3)
    acts = np.random.RandomState(7).uniform(-1, 1, (steps, n, 12))
    traj, info = S.rollout(flat, dict(H.ANYMAL_PARAMS, solver_type=3), root, dof, mu, default, acts, 2)
    assert np.isfinite(traj).all()
    assert info["pen_max"] < 0.03
