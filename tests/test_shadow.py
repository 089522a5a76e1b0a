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


def test_shadow_free_close_known_answer(senv):
    """Free-space close (object out of reach) with close_gripper_at's servo
    targets (shadow.py:379-410 through _qpos_to_qacc, :444-455) against
    shadow.yaml:10 qpos_close, which those targets equal for the first and
    middle fingers and the thumb (ring and little finger targets differ from
    the yaml and are not compared).  A position servo with gain kp stops where
    its torque kp * error no longer beats the joints' frictionloss (0.01 per
    joint), so every unobstructed servo ends within floss * (joints it drives)
    / kp of its target: FFJ4 / FFJ3 / MFJ4 / thumb joints per joint, the J1 + J2
    sums of the FF and MF tendon servos.  MFJ3 (target 1.475) curls the middle
    proximal into the palm and rests short of it on that contact."""
    from oracle import oracle as O
    from mgs.util.geo.transforms import SE3Pose
    cm = senv.model
    g = senv.gripper
    qpos_close = np.array([-0.3464, 1.253, 0.7836, -0.001106, 0.01103, 1.475, 0.6181, 0.0155, -0.2083, 0.3328,
                           0.07129, 0.02873, 0.1829, -0.2676, 0.05465, 0.3892, 0.008468, 0.07708, 1.21, 0.2023,
                           0.6614, 0.0102])
    pose = SE3Pose(np.array([[0.0, 0.0, 0.0]]), np.array([[1.0, 0, 0, 0]]), "wxyz")
    q, mp, mq, _ = senv.initial_state(pose, np.zeros((1, 22)))
    q[0, cm.nq - 7] = 1.0            # object x: far from the hand
    idx = senv.get_joint_idxs(g.get_actuator_joint_names())
    ctrl = g.close_ctrl(None)
    om = O.OracleModel(cm, ncon_max=40)
    tr, nc, qv = om.trace(q[0], mp[0], mq[0], ctrl, 3000)
    qf = tr[-1, idx]
    kp = dict(zip(cm.actuator_names, -np.asarray(cm.actuator_biasprm)[:, 1]))
    floss = 0.01
    assert np.allclose(cm.dof_frictionloss[6:28], floss)
    slack = 1e-3
    single = {0: "rh_A_FFJ4", 1: "rh_A_FFJ3", 4: "rh_A_MFJ4", 17: "rh_A_THJ5", 18: "rh_A_THJ4", 19: "rh_A_THJ3",
              20: "rh_A_THJ2", 21: "rh_A_THJ1"}
    for j, a in single.items():
        assert abs(qf[j] - qpos_close[j]) <= floss / kp[a] + slack, (j, qf[j] - qpos_close[j])
    for (j1, j2), a in (((2, 3), "rh_A_FFJ0"), ((6, 7), "rh_A_MFJ0")):
        err = (qf[j1] + qf[j2]) - (qpos_close[j1] + qpos_close[j2])
        assert abs(err) <= 2 * floss / kp[a] + slack, (a, err)
    # MFJ3: short of its target, held by the palm
    assert qpos_close[5] - qf[5] > 0.05
    _, _, _, _, gg = om.contacts(tr[-1], mp[0], mq[0])
    pairs = {tuple(sorted((cm.body_names[cm.geom_bodyid[a]], cm.body_names[cm.geom_bodyid[b]]))) for a, b in gg}
    assert ("rh_mfproximal", "rh_palm") in pairs
