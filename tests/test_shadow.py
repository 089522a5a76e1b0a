"""Shadow Hand x object (config C5's gripper).

CPU: model structure (25 gripper bodies incl. the mocap, 36 collision geoms
of five types, 22 frictionloss joints, 4 coupled tendons, 18 servos; SURVEY.md
§8 table), the reference's 22 -> 18 joint-target mapping _qpos_to_qacc
(shadow.py:444-455, restated independently below) and its close targets
(shadow.py:383-408), and oracle rollouts that grasp.
GPU: mask and rollout bit-exact against the oracle through the C-ABI, with
contact-capacity escalation (the hand makes > 20 contacts on some steps)."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def senv():
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_object
    return GravitylessObjectGrasping(get_gripper({"name": "ShadowHand"}), get_object("005_tomato_soup_can"))


@pytest.fixture(scope="module")
def scand(senv):
    from mgs.sampler.antipodal import hand_candidates
    from mgs.util.geo.transforms import SE3Pose
    H, J, _ = hand_candidates(senv.obj, 256, senv.gripper, seed=0)
    return SE3Pose.from_mat(H), J


def test_shadow_model(senv):
    cm = senv.model
    assert (cm.nv, cm.nu, cm.nmocap) == (34, 18, 1)
    ground = cm.geom_names.index("geom:ground")
    assert ground == 36
    assert int((cm.dof_frictionloss > 0).sum()) == 22
    assert int((cm.geom_radius[:ground] > 0).sum()) == 13        # 8 finger + 2 thumb capsules, 3 thumb spheres


def test_shadow_ctrl_mapping(senv):
    g = senv.gripper
    q = np.arange(22, dtype=float)
    ff, mf, rf, lf, th = q[0:4], q[4:8], q[8:12], q[12:17], q[17:22]
    expect = np.concatenate([th, ff[:2], [ff[2] + ff[3]], mf[:2], [mf[2] + mf[3]], rf[:2], [rf[2] + rf[3]],
                             lf[:3], [lf[3] + lf[4]]])
    assert np.array_equal(g._qpos_to_qacc(q), expect)
    assert np.allclose(g.close_ctrl(None)[:5], [0.07708, 1.21, 0.2023, 0.6614, 0.0102])
    names = senv.model.actuator_names
    assert names[:5] == [f"rh_A_THJ{k}" for k in (5, 4, 3, 2, 1)] and names[7] == "rh_A_FFJ0"


def test_shadow_oracle_grasps(senv, scand):
    from conftest import plan_for
    from oracle import oracle as O
    poses, J = scand
    om = O.OracleModel(senv.model, ncon_max=senv.ncon_max, nefc_max=senv.nefc_max)
    q, mp, mq, _ = senv.initial_state(poses, J)
    idx = np.nonzero(om.collision_free(q, mp, mq, nthreads=8))[0][:16]
    assert len(idx) == 16
    r = om.rollout(plan_for(senv, poses[idx], J[idx]), nthreads=8)
    assert r["label"].sum() >= 4


@pytest.mark.gpu
def test_shadow_gpu_parity(senv, scand):
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
    from conftest import plan_for
    from oracle import oracle as O
    poses, J = scand
    om = O.OracleModel(senv.model, ncon_max=senv.ncon_max, nefc_max=senv.nefc_max)
    q, mp, mq, _ = senv.initial_state(poses, J)
    fg = senv.engine.collision_free(q, mp, mq)
    assert np.array_equal(fg, om.collision_free(q, mp, mq, nthreads=8))
    idx = np.nonzero(fg)[0][:64]
    plan = plan_for(senv, poses[idx], J[idx])
    rg, ro = senv.engine.rollout(plan), om.rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(rg[k], ro[k]), k
    # escalated results equal the oracle at the wider capacity
    res = senv.rollout(plan)
    ov = np.nonzero(rg["stats"][:, 2])[0]
    if len(ov):
        ow = O.OracleModel(senv.model, ncon_max=40, nefc_max=senv.engine_for(40).desc.nefc_max).rollout(
            plan.subset(ov), nthreads=8)
        for k in ("label", "fail_step", "obj_qpos", "stats"):
            assert np.array_equal(res[k][ov], ow[k]), k
