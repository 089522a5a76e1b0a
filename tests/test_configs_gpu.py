"""The two secondary BASELINE configs on the device, against the oracle.

C5 — Shadow Hand on a settled 5-object clutter pile (tests/golden/
clutter_scene_shadow.npz, made by tests/golden/make_clutter_scene.py): the
reference's ClutterTableEnv.grasp_collision_mask (mgs/env/clutter_table.py:
330-367) and grasp_stable_mask (:272-321) with the Shadow close
(mgs/gripper/shadow.py:379-410), nv 58, through the wide library.  The
capacity-escalation path (GravitylessObjectGrasping.rollout semantics: a
candidate whose contacts or rows overflow is re-run from its initial state at
twice the capacity) is forced by starting at 16 contacts, and the escalated
result must equal the oracle run at the full capacity.

C4 — Allegro hand on a GSO-format object (Synthetic_Mug_Body; the loader is
mgs/obj/gso.py:70-160 in the reference): collision mask and the h200 rollout
(mgs/gripper/allegro.py:354-357) bit-exact against the oracle.
"""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SHADOW_SCENE = os.path.join(HERE, "golden", "clutter_scene_shadow.npz")


def _init_torch():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass


def _in_bounds(p):
    return (np.abs(p[:, 0]) < 0.25) & (np.abs(p[:, 1]) < 0.25) & (p[:, 2] > 0) & (p[:, 2] < 1)


@pytest.fixture(scope="module")
def senv():
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_clutter_scene import make_env
    env = make_env("ShadowHand")
    env.set_state(np.load(SHADOW_SCENE)["state"])
    return env


@pytest.fixture(scope="module")
def scand(senv):
    """hand candidates of every pile object, posed by its settled pose (gen_scene.py:59-66)."""
    from mgs.sampler.antipodal import hand_candidates
    from mgs.util.geo.transforms import SE3Pose
    H, J = [], []
    for k, o in enumerate(senv.objects):
        h, j, _ = hand_candidates(o, 32, senv.gripper, seed=k)
        H.append((senv.get_obj_pose(o.name) @ SE3Pose.from_mat(h)).to_mat())
        J.append(j)
    return SE3Pose.from_mat(np.concatenate(H).astype(np.float32)), np.concatenate(J)


def test_shadow_pile_oracle(senv, scand):
    """CPU: the C5 model and the oracle's mask / short rollout are sane."""
    from oracle import oracle as O
    poses, J = scand
    st = senv.get_state()
    assert senv.model.nv == 28 + 6 * 5
    q, mp, mq = senv._initial_qpos(poses, J, st)
    om = O.OracleModel(senv.model_for(st), ncon_max=senv.ncon_max, nefc_max=256)
    free = om.collision_free(q, mp, mq, predicate="partition_incl", nthreads=8) & _in_bounds(poses.pos)
    assert 4 <= free.sum() < len(free)
    idx = np.nonzero(free)[0][:3]
    r = om.rollout(senv.stable_plan(poses[idx], J[idx], st, nstep_lift=60, close_steps=60), nthreads=8)
    assert r["stats"][:, 0].max() > 16           # the pile has more contacts than the forced start capacity
    assert r["stats"][:, 2].max() == 0


@pytest.mark.gpu
def test_shadow_pile_gpu_parity(senv, scand):
    _init_torch()
    from oracle import oracle as O
    poses, J = scand
    st = senv.get_state()
    eng = senv.engine_for_state(st)
    assert os.path.basename(eng.lib._name) == "libmgs_gpu_wide.so"
    om = O.OracleModel(senv.model_for(st), ncon_max=senv.ncon_max, nefc_max=eng.desc.nefc_max)
    mask = senv.grasp_collision_mask(poses, J)
    q, mp, mq = senv._initial_qpos(poses, J, st)
    ref = om.collision_free(q, mp, mq, predicate="partition_incl", nthreads=8) & _in_bounds(poses.pos)
    assert np.array_equal(mask, ref)
    idx = np.nonzero(mask)[0][:8]
    plan = senv.stable_plan(poses[idx], J[idx], st, nstep_lift=200, close_steps=200)
    rg, ro = eng.rollout(plan), om.rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(rg[k], ro[k]), k
    lab = senv.grasp_stable_mask(poses[idx], J[idx], st, nstep_lift=200, close_steps=200, enough_stable=2)
    from conftest import full_capacity_oracle
    rf = full_capacity_oracle(senv, st).rollout(plan, nthreads=8)     # the env escalates past its capacity
    assert lab.sum() == min(2, int(rf["label"].sum()))


@pytest.mark.gpu
def test_shadow_pile_reference_schedule_parity(senv, scand):
    """C5 at the reference's own schedule: close 3000 + lift 3000 steps
    (clutter_table.py:277,307) on two pile candidates through the env's own
    rollout (main capacity, escalation past it), bit-exact against the oracle
    at the escalation's full capacity"""
    _init_torch()
    from conftest import full_capacity_oracle
    poses, J = scand
    st = senv.get_state()
    idx = np.nonzero(senv.grasp_collision_mask(poses, J))[0][:2]
    plan = senv.stable_plan(poses[idx], J[idx], st)
    assert plan.nsteps == [3000, 3000]
    rg, ro = senv.rollout(plan, st), full_capacity_oracle(senv, st).rollout(plan, nthreads=2)
    assert rg["overflow"] == 0 and (ro["stats"][:, 2] == 0).all()
    for k in ("label", "fail_step", "obj_qpos"):
        assert np.array_equal(rg[k], ro[k]), k


@pytest.mark.gpu
def test_shadow_pile_capacity_escalation(senv, scand):
    """start at 16 contacts: the first pass overflows, the escalated result is
    the oracle's at full capacity."""
    _init_torch()
    from mgs.env.clutter_table import ClutterTableEnv
    from oracle import oracle as O
    poses, J = scand
    st = senv.get_state()
    small = ClutterTableEnv.from_dict(senv.to_dict(), ncon_max=16)
    idx = np.nonzero(senv.grasp_collision_mask(poses, J))[0][:6]
    plan = small.stable_plan(poses[idx], J[idx], st, nstep_lift=100, close_steps=100)
    first = small.engine_for_state(st).rollout(plan)
    assert (first["stats"][:, 2] != 0).any()
    res = small.rollout(plan, st)
    assert res["overflow"] == 0
    from conftest import full_capacity_oracle
    ro = full_capacity_oracle(senv, st).rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos"):
        assert np.array_equal(res[k], ro[k]), k


@pytest.mark.gpu
def test_shadow_pile_rotation_and_escalation(senv, scand):
    """the wide build's in-launch rotation (G in HBM, four rows per lane): a
    work-queue grid of 3 workgroups over the pile candidates with a yield every
    7 steps, starting at 16 contacts so the escalation continues the capped
    candidates from their records -- every output equals one workgroup per
    candidate without rotation, candidates yielded and no ring spin expired"""
    _init_torch()
    from mgs.env.clutter_table import ClutterTableEnv
    poses, J = scand
    st = senv.get_state()
    small = ClutterTableEnv.from_dict(senv.to_dict(), ncon_max=16)
    idx = np.nonzero(senv.grasp_collision_mask(poses, J))[0][:8]
    plan = small.stable_plan(poses[idx], J[idx], st, nstep_lift=60, close_steps=60)
    # the main engine (16 contacts) and the escalation's (32 .. 128): the
    # capped candidates stop within a few steps at 16, so the later stages
    # are the ones that run long enough to rotate
    engines = [small.engine_for_state(st, ncon_max=c) for c in (16, 32, 64, 128)]
    L = engines[0].lib

    def stats():
        q = [e.queue_stats() for e in engines]
        return sum(a for a, _ in q), sum(b for _, b in q)
    prev = L.mgs_rollout_queue(-1)
    try:
        L.mgs_rollout_queue(0)
        one = small.rollout(plan, st, yield_every=0)
        y0, s0 = stats()
        L.mgs_rollout_queue(3)
        rot = small.rollout(plan, st, yield_every=7)
        y1, s1 = stats()
    finally:
        L.mgs_rollout_queue(prev)
    assert len(idx) > 3
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(rot[k], one[k]), k
    assert y1 > y0 and s1 == s0 == 0


@pytest.fixture(scope="module")
def genv():
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.selector import get_gripper
    from mgs.obj.gso import ObjectGSO
    from mgs.obj.selector import get_object
    obj = get_object("Synthetic_Mug_Body")
    assert isinstance(obj, ObjectGSO)
    return GravitylessObjectGrasping(get_gripper({"name": "AllegroGripper"}), obj)


@pytest.fixture(scope="module")
def gcand(genv):
    from mgs.sampler.antipodal import hand_candidates
    from mgs.util.geo.transforms import SE3Pose
    H, J, _ = hand_candidates(genv.obj, 512, genv.gripper, seed=3)
    return SE3Pose.from_mat(H), J


def test_allegro_gso_oracle(genv, gcand):
    from conftest import plan_for
    from oracle import oracle as O
    poses, J = gcand
    # full capacity (the last stage of the env's escalation, 64 contacts / 256
    # rows is beyond it): multiccd contacts of a hand grasp fit, nothing capped
    om = O.OracleModel(genv.model, ncon_max=64, nefc_max=256)
    q, mp, mq, _ = genv.initial_state(poses, J)
    free = om.collision_free(q, mp, mq, nthreads=8)
    assert 16 <= free.sum() < len(free)
    idx = np.nonzero(free)[0][:16]
    r = om.rollout(plan_for(genv, poses[idx], J[idx]), nthreads=8)
    assert r["stats"][:, 2].max() == 0


@pytest.mark.gpu
def test_allegro_gso_gpu_parity(genv, gcand):
    _init_torch()
    from conftest import plan_for
    from oracle import oracle as O
    poses, J = gcand
    om = O.OracleModel(genv.model, ncon_max=genv.ncon_max, nefc_max=genv.nefc_max)
    mask = genv.grasp_collision_mask(poses, J)
    q, mp, mq, _ = genv.initial_state(poses, J)
    assert np.array_equal(mask, om.collision_free(q, mp, mq, nthreads=8))
    idx = np.nonzero(mask)[0][:96]
    plan = plan_for(genv, poses[idx], J[idx])
    rg, ro = genv.engine.rollout(plan), om.rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(rg[k], ro[k]), k
    mask2, stable = genv.evaluate(poses, J, horizon="h200", enough_stable=5)
    assert np.array_equal(mask2, mask)
    assert stable.sum() <= 5 and np.all(stable[idx] <= ro["label"])
