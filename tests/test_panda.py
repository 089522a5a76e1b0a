"""Franka Panda gripper x object (config C3's gripper).

CPU: model compile, the host bookkeeping the reference defines for the Panda
(width_to_joints / _clamp_width, panda.py:217-223,264-266; b2c panda.py:190-193;
close ctrl panda.py:225-241), and a physics known answer from the reference's
own config: `qpos_close: [0.0, -0.04]` (mgs/cli/config/gripper/panda.yaml:7),
the fingers' closed joint values, reached by the oracle's free-space close.
GPU: mask and rollout bit-exact against the oracle through the C-ABI."""
import numpy as np
import pytest

# reference panda.yaml:6-7 (data): open and closed finger joints
QPOS_OPEN = np.array([0.04, 0.00])
QPOS_CLOSE = np.array([0.0, -0.04])


@pytest.fixture(scope="module")
def penv():
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_object
    return GravitylessObjectGrasping(get_gripper({"name": "PandaGripper"}), get_object("003_cracker_box"))


@pytest.fixture(scope="module")
def pcand(penv):
    from mgs.sampler.antipodal import panda_candidates
    from mgs.util.geo.transforms import SE3Pose
    H, J, W = panda_candidates(penv.obj, 1024, seed=0)
    return SE3Pose.from_mat(H), np.asarray(J, np.float64), W


@pytest.fixture(scope="module")
def pom(penv):
    from oracle import oracle as O
    return O.OracleModel(penv.model, ncon_max=penv.ncon_max, nefc_max=penv.nefc_max)


def test_panda_model_sizes(penv):
    cm = penv.model
    # hand free joint (7/6) + 2 slide fingers + object free joint (7/6)
    assert (cm.nq, cm.nv, cm.nu, cm.nmocap) == (16, 14, 2, 1)
    assert cm.geom_names.index("geom:ground") == 13          # 1 hand hull + 2 x (hull + 5 pads)
    assert penv.get_joint_idxs(["finger_joint1", "finger_joint2"]) == [7, 8]


def test_panda_host_bookkeeping(penv, pcand):
    g = penv.gripper
    w = np.array([-1.0, 0.0, 0.01, 0.05, 0.055, 0.2])
    q1, q2 = g.width_to_joints(g._clamp_width(w))
    cw = np.clip(w + 0.025, 0.003, 0.08)
    assert np.array_equal(q1, np.clip(cw / 2, 0, 0.04)) and np.array_equal(q2, np.clip(-0.04 + cw / 2, -0.04, 0))
    poses, J, W = pcand
    q, mp, mq, proc = penv.initial_state(poses[:4], J[:4])
    assert np.array_equal(q[:, 7:9], J[:4])
    b2c = g.base_to_contact_transform()
    assert np.allclose(b2c.quat, [0.70710677, 0, 0, 0.70710677]) and np.allclose(b2c.pos, [0, 0, -0.102])
    assert np.array_equal(mp, proc.pos.astype(np.float64))
    assert np.array_equal(g.close_ctrl(None), QPOS_CLOSE)


def test_panda_free_close_known_answer(penv):
    """Free-space close (object out of reach) settles on panda.yaml's qpos_close
    up to the static deadband the fingers' frictionloss (1 N) leaves against the
    position servo (kp 1000): |q - q_close| <= 1 N / 1000 N/m = 1 mm."""
    from mgs.util.geo.transforms import SE3Pose
    from oracle import oracle as O
    om = O.OracleModel(penv.model)
    pose = SE3Pose(np.array([[0.0, 0.0, 0.0]]), np.array([[1.0, 0, 0, 0]]), "wxyz")
    q, mp, mq, _ = penv.initial_state(pose, QPOS_OPEN[None])
    q[0, 9] = 0.4          # object x: far from the fingers
    tr, nc, qv = om.trace(q[0], mp[0], mq[0], QPOS_CLOSE, 3000)
    assert np.abs(tr[-1, 7:9] - QPOS_CLOSE).max() <= 1.0 / 1000 + 1e-9
    assert np.abs(qv).max() < 1e-6


def test_panda_oracle_rollout_sane(penv, pcand, pom):
    from conftest import plan_for
    poses, J, _ = pcand
    q, mp, mq, _ = penv.initial_state(poses, J)
    free = pom.collision_free(q, mp, mq, nthreads=8)
    assert 0.005 < free.mean() < 0.5
    idx = np.nonzero(free)[0][:16]
    r = pom.rollout(plan_for(penv, poses[idx], J[idx]), nthreads=8)
    assert r["label"].any()
    # stable grasps keep the object between the fingers: it stays within 10 cm of the hand
    ok = r["label"]
    assert np.all(np.isfinite(r["obj_qpos"][ok]))


@pytest.mark.gpu
def test_panda_gpu_parity(penv, pcand, pom):
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
    from conftest import plan_for
    poses, J, _ = pcand
    q, mp, mq, _ = penv.initial_state(poses, J)
    fg = penv.engine.collision_free(q, mp, mq)
    assert np.array_equal(fg, pom.collision_free(q, mp, mq, nthreads=8))
    idx = np.nonzero(fg)[0]
    plan = plan_for(penv, poses[idx], J[idx])
    rg, ro = penv.engine.rollout(plan), pom.rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(rg[k], ro[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("obj_id", ["005_tomato_soup_can", "010_potted_meat_can", "017_orange", "061_foam_brick"])
def test_panda_ycb_set_gpu_parity(obj_id):
    """C3 covers the YCB set: every shipped YCB-format object besides the
    cracker box (test_panda_gpu_parity), mask and h200 rollouts bit-exact
    against the oracle through the C-ABI (with the env's capacity escalation)"""
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
    from conftest import plan_for
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_object
    from mgs.sampler.antipodal import panda_candidates
    from mgs.util.geo.transforms import SE3Pose
    from oracle import oracle as O
    env = GravitylessObjectGrasping(get_gripper({"name": "PandaGripper"}), get_object(obj_id))
    H, J, _ = panda_candidates(env.obj, 512, seed=1)
    poses, J = SE3Pose.from_mat(H), np.asarray(J, np.float64)
    q, mp, mq, _ = env.initial_state(poses, J)
    om = O.OracleModel(env.model, ncon_max=env.ncon_max, nefc_max=env.nefc_max)
    fg = env.engine.collision_free(q, mp, mq)
    assert np.array_equal(fg, om.collision_free(q, mp, mq, nthreads=8))
    idx = np.nonzero(fg)[0][:96]
    assert len(idx) >= 8
    plan = plan_for(env, poses[idx], J[idx])
    rg = env.rollout(plan, max_ncon=env.ncon_max, on_capacity="capped")
    ro = om.rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(rg[k], ro[k]), k
