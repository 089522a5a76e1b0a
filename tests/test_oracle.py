"""The CPU oracle (oracle/mgs_oracle.c): the checker the GPU path is compared
with.  Pinned here by (1) the reference's own known answer for the physics,
Robotiq's recorded closed state `state_close` (mgs/cli/config/gripper/
robotiq_2f_85.yaml:11, values copied as data below), (2) its arithmetic
primitives, (3) determinism and solver consistency."""
import copy

import numpy as np
import pytest

# state_close (robotiq_2f_85.yaml:11): right driver, coupler, spring link,
# follower, then the left chain, after a long ctrl=255 close in free space.
KAT_JOINTS = np.array([7.93116751e-01, 3.48441304e-04, 7.89591521e-01, -7.76735418e-01,
                       7.93117030e-01, 3.47173334e-04, 7.89598436e-01, -7.76696653e-01])


def free_close(env, solver, noslip, nsteps):
    from oracle import oracle as O
    from mgs.util.geo.transforms import SE3Pose
    cm = copy.copy(env.model)
    cm.options = dict(env.model.options)
    cm.options["solver"] = solver
    om = O.OracleModel(cm)
    om.desc.noslip_iterations = noslip
    pose = SE3Pose(np.array([[0.0, 0.0, 0.0]]), np.array([[1.0, 0, 0, 0]]), "wxyz")
    q, mp, mq, _ = env.initial_state(pose, np.zeros((1, 8)))
    q[0, 17] = 0.4      # object out of reach, as in the recorded state
    tr, nc, qv = om.trace(q[0], mp[0], mq[0], np.array([255.0]), nsteps)
    return tr, qv


@pytest.mark.parametrize("solver", ["Newton", "PGS"])
def test_state_close_known_answer(env, solver):
    """Free-space close settles within 1.5e-3 rad of MuJoCo's recorded state
    (noslip off: MuJoCo reached rest, |qvel| ~ 1e-14)."""
    tr, qv = free_close(env, solver, noslip=0, nsteps=4000)
    assert np.abs(tr[-1, 7:15] - KAT_JOINTS).max() < 1.5e-3
    assert np.abs(qv).max() < (1e-9 if solver == "Newton" else 1e-4)   # PGS: 100 iterations, not converged


def test_state_close_with_noslip(env):
    """With the reference's noslip_iterations=2 (gravityless_object_grasping.py:41)
    the close comes to rest at the recorded state.  Before MuJoCo's costChange
    rule was restated (a block update that raises the dual cost by > 1e-10 is
    undone), noslip kept the pad1-pad1 edge contact in a limit cycle at
    |qvel| = 0.19 rad/s; now the residual is the unregularised noslip sweep's
    jitter on the two redundant edge contacts, < 1e-6 rad/s."""
    tr, qv = free_close(env, "Newton", noslip=2, nsteps=4000)
    assert np.abs(tr[-1, 7:15] - KAT_JOINTS).max() < 1.5e-3
    assert np.abs(qv).max() < 2e-6
    v = np.abs(np.diff(tr[2000:, 7:15], axis=0)).max() / 1e-3      # finite-difference joint speed
    assert v < 2e-6


def test_pgs_cost_change_revert_noslip_free_close(env):
    """PGS main solver + noslip, same rest criterion (PGS at 100 iterations is
    not converged, so the bound is the solver's, not the revert rule's)."""
    tr, qv = free_close(env, "PGS", noslip=2, nsteps=4000)
    assert np.abs(tr[-1, 7:15] - KAT_JOINTS).max() < 1.5e-3
    assert np.abs(qv).max() < 1e-3


def test_sincos_and_tree_primitives():
    from oracle import oracle as O
    x = np.concatenate([np.linspace(-30, 30, 4001), np.array([0.0, 1e-300, -1e-8, np.pi / 2, np.pi])])
    s, c = O.sincos(x)
    assert np.abs(s - np.sin(x)).max() < 4e-16 * 30
    assert np.abs(c - np.cos(x)).max() < 4e-16 * 30
    rng = np.random.default_rng(0)
    for n in [1, 2, 3, 7, 16, 20, 33, 64]:
        a, b = rng.standard_normal(64), rng.standard_normal(64)
        leaf = np.zeros(64)
        P = 1
        while P < n:
            P *= 2
        leaf[:n] = a[:n] * b[:n]
        s_ = 1
        v = leaf[:P].copy()
        while s_ < P:
            v = v + v[np.arange(P) ^ s_]
            s_ *= 2
        assert O.tree_dot(a, b, n) == v[0]


def test_rollout_deterministic_across_threads(env, candidates, oracle_model):
    from conftest import plan_for
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    free = oracle_model.collision_free(q, mp, mq, nthreads=4)
    idx = np.nonzero(free)[0][:12]
    plan = plan_for(env, poses[idx], J[idx])
    r1 = oracle_model.rollout(plan, nthreads=1)
    r4 = oracle_model.rollout(plan, nthreads=4)
    for k in r1:
        assert np.array_equal(r1[k], r4[k]), k


def test_collision_free_fraction(env, candidates, oracle_model):
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    free = oracle_model.collision_free(q, mp, mq, nthreads=4)
    assert 0.05 < free.mean() < 0.5
    part = oracle_model.collision_free(q, mp, mq, predicate="partition", nthreads=4)
    assert np.all(part >= free)        # gripper-object contact implies any contact


def test_newton_and_pgs_agree_on_labels(env, candidates):
    """Same convex problem, two solvers: labels agree on most candidates."""
    from conftest import plan_for
    from oracle import oracle as O
    poses, J = candidates
    res = {}
    for solver in ["Newton", "PGS"]:
        cm = copy.copy(env.model)
        cm.options = dict(env.model.options)
        cm.options["solver"] = solver
        om = O.OracleModel(cm)
        q, mp, mq, _ = env.initial_state(poses, J)
        idx = np.nonzero(om.collision_free(q, mp, mq, nthreads=4))[0]
        res[solver] = om.rollout(plan_for(env, poses[idx], J[idx]), nthreads=4)["label"]
    assert (res["Newton"] == res["PGS"]).mean() >= 0.85


def test_empty_batch(env, oracle_model):
    from conftest import plan_for
    from mgs.util.geo.transforms import SE3Pose
    poses = SE3Pose(np.zeros((0, 3), np.float32), np.zeros((0, 4), np.float32), "wxyz")
    q, mp, mq, _ = env.initial_state(poses, np.zeros((0, 8)))
    assert oracle_model.collision_free(q, mp, mq).shape == (0,)


def _guard_plan(env, candidates, oracle_model, n=4):
    """n collision-free candidates (the rollouts the pipeline runs), two of them
    given a bad initial state"""
    from conftest import plan_for
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    idx = np.nonzero(oracle_model.collision_free(q, mp, mq))[0][:n]
    plan = plan_for(env, poses[idx], J[idx])
    plan.qpos_init = plan.qpos_init.copy()
    plan.qpos_init[1, 17] = np.nan        # object x: a NaN state
    plan.qpos_init[2, 0] = 2e10           # gripper x beyond mjMAXVAL
    return plan


def test_divergence_guard_oracle(env, candidates, oracle_model):
    """MuJoCo's mj_checkPos / mj_checkVel / mj_checkAcc (NaN or |x| > 1e10) stop a
    candidate: label 0, fail step = the step that produced the bad state, flag
    MGS_FLAG_DIVERGED in stats[:, 2]; healthy candidates are untouched."""
    from mgs.core.abi import MGS
    plan = _guard_plan(env, candidates, oracle_model)
    r = oracle_model.rollout(plan)
    div = MGS["MGS_FLAG_DIVERGED"]
    assert list(r["stats"][:, 2] & div) == [0, div, div, 0]
    assert not r["label"][1] and not r["label"][2]
    assert r["fail_step"][1] == 0 and r["fail_step"][2] == 0
    clean = oracle_model.rollout(plan.subset([0, 3]))
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(clean[k], r[k][[0, 3]])


@pytest.mark.parametrize("horizon,n", [("h200", 160), ("ref8000", 3)])
def test_separation_certificates_are_exact(env, candidates, oracle_model, horizon, n):
    """Pairs skipped by a separation certificate (kernel / oracle cert_check)
    are pairs MPR would miss: rollouts with the skipping turned off give the
    same labels, fail steps, object poses and contact / row statistics, bit
    for bit, and the skipping removes narrowphase support calls"""
    import ctypes
    from conftest import plan_for
    from oracle import oracle as O
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    idx = np.nonzero(oracle_model.collision_free(q, mp, mq, nthreads=8))[0][:n]
    plan = plan_for(env, poses[idx], J[idx], horizon)
    L = O.lib()
    L.oracle_set_cull.argtypes = [ctypes.c_int]
    try:
        L.oracle_set_cull(0)
        off = oracle_model.rollout(plan, nthreads=8)
    finally:
        L.oracle_set_cull(1)
    on = oracle_model.rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(on[k], off[k]), k
