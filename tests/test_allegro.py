"""Allegro 16-DoF hand x object (config C4's gripper).

CPU: model structure (22 gripper bodies incl. the mocap, 17 boxes + 4 fingertip
capsules, 16 position servos), the reference's host
bookkeeping (close ctrl = close_pose, allegro.py:275-294,354-357; the composed
base-to-contact transform, allegro.py:296-302, recomputed here with scipy as
the reference does), and oracle rollouts that grasp.
GPU: mask and rollout bit-exact against the oracle through the C-ABI (this
exercises the rounded fingertip capsules on the device)."""
import numpy as np
import pytest
from scipy.spatial.transform import Rotation


@pytest.fixture(scope="module")
def aenv():
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_object
    return GravitylessObjectGrasping(get_gripper({"name": "AllegroGripper"}), get_object("005_tomato_soup_can"))


@pytest.fixture(scope="module")
def acand(aenv):
    from mgs.sampler.antipodal import hand_candidates
    from mgs.util.geo.transforms import SE3Pose
    H, J, _ = hand_candidates(aenv.obj, 512, aenv.gripper, seed=0)
    return SE3Pose.from_mat(H), J


@pytest.fixture(scope="module")
def aom(aenv):
    from oracle import oracle as O
    return O.OracleModel(aenv.model, ncon_max=aenv.ncon_max, nefc_max=aenv.nefc_max)


def test_allegro_model(aenv):
    cm = aenv.model
    assert (cm.nv, cm.nu, cm.nmocap) == (28, 16, 1)
    assert cm.nbody == 25                      # world + 22 gripper bodies + ground + object
    ground = cm.geom_names.index("geom:ground")
    assert ground == 21
    assert int((cm.geom_radius[:ground] > 0).sum()) == 4       # fingertip capsules
    assert np.allclose(sorted(cm.geom_radius[:ground][cm.geom_radius[:ground] > 0]), 0.012)


def test_allegro_host_bookkeeping(aenv, acand):
    g = aenv.gripper
    b2c = g.base_to_contact_transform()
    th = -np.pi / 2
    R = Rotation.from_quat([0, np.sin(th / 2), 0, np.cos(th / 2)])
    assert np.allclose(b2c.pos, R.apply([-0.08, 0.0, 0.01]), atol=1e-7)
    assert np.allclose(b2c.quat, [np.cos(th / 2), 0, np.sin(th / 2), 0], atol=1e-7)
    assert np.array_equal(g.close_ctrl(None), [-0.08, 0.95, 1, 0.95, 0, 0.95, 1.2, 0.85, 0.08, 0.95, 1.2, 0.9,
                                              1.4, 0.55, 0.29, 1.45])
    poses, J = acand
    q, mp, mq, proc = aenv.initial_state(poses[:3], J[:3])
    idx = aenv.get_joint_idxs(g.get_actuator_joint_names())
    assert np.array_equal(q[:, idx], J[:3])


def test_allegro_free_close_known_answer(aenv, aom):
    """Free-space close (object out of reach) against allegro.yaml:7 qpos_close,
    which close_gripper_at sends as the servo targets (allegro.py:354-357):
    the unobstructed first and ring fingers settle on it exactly (position
    servos, no gravity); the thumb (target 1.4 clamped to its ctrlrange 1.396)
    meets the middle finger, so those two chains rest short of it on that one
    contact.  The hand comes to rest."""
    from mgs.util.geo.transforms import SE3Pose
    close = np.array([-0.08, 0.95, 1, 0.95, 0, 0.95, 1.2, 0.85, 0.08, 0.95, 1.2, 0.9, 1.4, 0.55, 0.29, 1.45])
    pose = SE3Pose(np.array([[0.0, 0.0, 0.0]]), np.array([[1.0, 0, 0, 0]]), "wxyz")
    q, mp, mq, _ = aenv.initial_state(pose, np.zeros((1, 16)))
    q[0, 23] = 1.0          # object x: far from the hand
    tr, nc, qv = aom.trace(q[0], mp[0], mq[0], close, 3000)
    qf = tr[-1, 7:23]
    assert np.abs(qf[0:4] - close[0:4]).max() < 1e-9          # first finger
    assert np.abs(qf[8:12] - close[8:12]).max() < 1e-9        # ring finger
    assert np.abs(qf[4:8] - close[4:8]).max() < 1e-2          # middle finger, held by the thumb
    assert np.abs(qf[12:16] - close[12:16]).max() < 1.5e-2    # thumb
    assert nc[-1] == 1
    assert np.abs(qv).max() < 1e-9


def test_allegro_oracle_grasps(aenv, acand, aom):
    from conftest import plan_for
    poses, J = acand
    q, mp, mq, _ = aenv.initial_state(poses, J)
    free = aom.collision_free(q, mp, mq, nthreads=8)
    idx = np.nonzero(free)[0][:32]
    assert len(idx) >= 16
    # full capacity (the env escalates past its main capacity; multiccd makes
    # more than 20 contacts on some hand grasps)
    from oracle import oracle as O
    r = O.OracleModel(aenv.model, ncon_max=64, nefc_max=256).rollout(plan_for(aenv, poses[idx], J[idx]), nthreads=8)
    assert r["label"].sum() >= 4
    assert r["stats"][:, 2].max() == 0


@pytest.mark.gpu
def test_allegro_gpu_parity(aenv, acand, aom):
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
    from conftest import plan_for
    poses, J = acand
    q, mp, mq, _ = aenv.initial_state(poses, J)
    fg = aenv.engine.collision_free(q, mp, mq)
    assert np.array_equal(fg, aom.collision_free(q, mp, mq, nthreads=8))
    idx = np.nonzero(fg)[0][:128]
    plan = plan_for(aenv, poses[idx], J[idx])
    rg, ro = aenv.engine.rollout(plan), aom.rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(rg[k], ro[k]), k
