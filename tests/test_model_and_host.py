"""Model compiler (the MjModel.from_xml_string replacement) and the host-side
mirror of the reference interface."""
import numpy as np
import pytest


def test_robotiq_env_sizes(env):
    cm = env.model
    # Robotiq x object nq 22, nv 20, nbody 18, collision geoms 15 + K (K = 1)
    assert (cm.nq, cm.nv, cm.nbody, cm.nmocap, cm.nu) == (22, 20, 18, 1, 1)
    assert len(cm.geom_bodyid) == 16
    assert sum({0: 3, 1: 6, 2: 1}[int(t)] for t in cm.eq_type) == 13      # 2 connect + weld + joint
    assert len(cm.pair_geom1) == 95


def test_option_merge_order(env):
    o = env.model.options
    # env XML then gripper <option>: impratio 3 -> 10, noslip 1 -> 2 (gravityless_object_grasping.py:36-42)
    assert o["impratio"] == 10.0
    assert o["noslip_iterations"] == 2
    assert o["tolerance"] == 1e-8 and o["noslip_tolerance"] == 1e-8
    assert o["cone"] == "elliptic" and o["integrator"] == "implicitfast"
    assert list(o["gravity"]) == [0.0, 0.0, 0.0]


def test_geom_partition(env):
    cm = env.model
    side = np.asarray(cm.geom_side)
    names = cm.geom_names
    assert side[names.index("geom:ground")] == 0
    assert all(side[i] < 0 for i, n in enumerate(names) if n.startswith(("right_", "left_")))
    assert side[-1] > 0                       # object geoms after the ground


def test_invweights(env):
    cm = env.model
    biw, diw = cm.body_invweight0, cm.dof_invweight0
    assert biw.shape == (cm.nbody, 2) and diw.shape == (cm.nv,)
    assert np.all(biw[0] == 0)
    mocap = list(cm.body_mocapid).index(0)
    assert np.all(biw[mocap] == 0)            # world-welded
    assert np.all(diw > 0)
    obj = cm.body_names.index("003_cracker_box") if "003_cracker_box" in cm.body_names else cm.nbody - 1
    # free body alone: translational inverse weight = 1 / mass
    assert biw[obj, 0] == pytest.approx(1.0 / cm.body_mass[obj], rel=1e-9)


def test_apply_enough_stable():
    from mgs.env.gravityless_object_grasping import apply_enough_stable
    lab = np.array([1, 0, 1, 1, 0, 1], bool)
    assert apply_enough_stable(lab, None).tolist() == lab.tolist()
    assert apply_enough_stable(lab, 2).tolist() == [True, False, True, False, False, False]
    assert apply_enough_stable(lab, 0).tolist() == [False] * 6


def test_horizons():
    from mgs.env.gravityless_object_grasping import HORIZONS
    h = HORIZONS["h200"]
    assert h["close_steps"] + h["nstep_lift"] + 4 * h["shake_steps"] == 200
    r = HORIZONS["ref8000"]
    assert r["close_steps"] + r["nstep_lift"] + 4 * r["shake_steps"] == 8000


def test_input_validation_mirrors_reference(env, candidates):
    poses, J = candidates
    with pytest.raises(ValueError, match="must match number of joint configurations"):
        env.grasp_collision_mask(poses[:3], J[:2])
    with pytest.raises(ValueError, match="incorrect dimension"):
        env.grasp_collision_mask(poses[:2], J[:2, :5])
    with pytest.raises(ValueError, match="must match number of joint configurations"):
        env.grasp_stability_evaluation_from_joints(poses[:3], J[:2])


def test_plan_layout(env, candidates):
    from conftest import plan_for
    poses, J = candidates
    plan = plan_for(env, poses[:5], J[:5])
    assert plan.horizon == 200
    assert plan.qpos_init.shape == (5, env.model.nq)
    assert plan.phase_start.shape == (5, 5, 3) and plan.phase_target.shape == (5, 5, 3)
    # left shake restarts from the pre-right position (gravityless_object_grasping.py:264-272)
    assert np.array_equal(plan.phase_start[:, 4], plan.phase_start[:, 3])


def test_gso_loader_format():
    """ObjectGSO (reference mgs/obj/gso.py:28-160): GoogleScannedObjects/<id>/ with
    info.yml, model.obj as the sampling mesh, same include body as YCB."""
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.selector import get_gripper
    from mgs.obj.gso import ObjectGSO
    from mgs.obj.selector import get_object
    o = get_object("Synthetic_Mug_Body", name="mug")
    assert isinstance(o, ObjectGSO) and o.obj_file_path.endswith("GoogleScannedObjects/Synthetic_Mug_Body/model.obj")
    env = GravitylessObjectGrasping(get_gripper({"name": "PandaGripper"}), o)
    cm = env.model
    assert cm.jnt_names[-1] == "mug:joint" and cm.nv == 14
    g = cm.geom_names.index("geom:ground")
    assert len(cm.geom_names) == g + 2 and cm.pair_condim.max() == 4


def test_se3_pose_against_reference_golden():
    """SE3Pose from_mat / @ / to_mat / inverse bit-exact against the reference's
    own SE3Pose (tests/golden/se3_golden.npz, tests/golden/make_se3_golden.py;
    reference transforms.py:79-121, operations.py:20-112), including inverse's
    mutation of the receiver with float64 values."""
    import os
    from mgs.util.geo.transforms import SE3Pose
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "se3_golden.npz"))
    a = SE3Pose.from_mat(g["H"])
    assert np.array_equal(a.pos, g["a_pos"]) and np.array_equal(a.quat, g["a_quat"])
    assert np.array_equal(a.to_mat(), g["a_mat"])
    b = SE3Pose(g["b_pos"], g["b_quat"], "wxyz")
    ab = a @ b
    assert np.array_equal(ab.pos, g["ab_pos"]) and np.array_equal(ab.quat, g["ab_quat"])
    c = SE3Pose(np.copy(a.pos), np.copy(a.quat), "wxyz")
    inv = c.inverse()
    assert np.array_equal(inv.pos, g["inv_pos"]) and np.array_equal(inv.quat, g["inv_quat"])
    assert c.pos.dtype == g["self_pos"].dtype and np.array_equal(c.pos, g["self_pos"])
    assert c.quat.dtype == g["self_quat"].dtype and np.array_equal(c.quat, g["self_quat"])


def test_from_mat_fast_path_equals_scipy():
    """SE3Pose.from_mat's batch path (Newton polar factor + Markley, rows at
    risk handed to scipy) returns scipy's from_matrix(...).as_quat(canonical=
    False) float32 rounding row for row: float32 pose products (the API's
    `poses @ b2c`), float64 rotations (all rows at risk: scipy's own path),
    identities and axis permutations (scipy skips its SVD)."""
    from scipy.spatial.transform import Rotation
    from mgs.util.geo import transforms as T
    n = 40000
    A = Rotation.random(n, random_state=11).as_matrix().astype(np.float32)
    B = Rotation.random(n, random_state=12).as_matrix().astype(np.float32)
    R32 = np.einsum("...ij,...jk->...ik", A, B)
    R64 = Rotation.random(500, random_state=13).as_matrix()
    Rax = Rotation.from_euler("zx", np.arange(400).reshape(200, 2) * 90, degrees=True).as_matrix().astype(np.float32)
    for R in (R32, R64, Rax, np.concatenate([Rax, R32[:300]])):
        want = Rotation.from_matrix(R).as_quat(canonical=False).astype(np.float32)
        assert np.array_equal(T._fast_quat(R).astype(np.float32), want)
    H = np.tile(np.eye(4, dtype=np.float32), (n, 1, 1))
    H[:, :3, :3] = R32
    assert np.array_equal(T.SE3Pose.from_mat(H).quat, T._xyzw_to_wxyz(T._scipy_quat(R32)).astype(np.float32))
    with pytest.raises(ValueError):
        T.SE3Pose.from_mat(-H)
    # to_mat's batch path (scipy's from_quat(...).as_matrix() products in its
    # order) against scipy, random and axis-aligned quaternions
    for R in (R32, Rax):
        q = Rotation.from_matrix(R).as_quat(canonical=False).astype(np.float32)
        want = Rotation.from_quat(np.copy(q)).as_matrix().astype(np.float32)
        assert np.array_equal(T._fast_mat(q), want)
        assert np.array_equal(T.SE3Pose(np.zeros((len(q), 3)), q, "xyzw").to_mat()[:, :3, :3], want)


def test_eig3_mesh_frame():
    """mgs.core.mjcf.eig3 (MuJoCo's mju_eig3 restated, the mesh compiler's
    principal axes): eigenvalues in decreasing order, the quaternion's matrix
    diagonalises the tensor to MuJoCo's own stopping rule (cosine within 1e-12
    of 1, i.e. off-diagonals ~1e-6 relative), and a degenerate (axisymmetric)
    tensor gets a fixed frame: the identity for an already diagonal one"""
    from mgs.core.mjcf import eig3, quat2mat
    rng = np.random.default_rng(0)
    for _ in range(300):
        A = rng.standard_normal((3, 3))
        A = A @ A.T
        ev, q = eig3(A)
        V = quat2mat(q)
        D = V.T @ A @ V
        assert np.abs(D - np.diag(np.diag(D))).max() < 1e-5 * np.abs(A).max()
        assert np.allclose(ev, np.sort(np.linalg.eigvalsh(A))[::-1], atol=1e-9 * np.abs(A).max())
    ev, q = eig3(np.diag([3.0, 2.0, 2.0]))
    assert np.array_equal(q, [1.0, 0.0, 0.0, 0.0]) and np.array_equal(ev, [3.0, 2.0, 2.0])
    ev, q = eig3(np.diag([1.0, 2.0, 2.0]))        # sorted by quarter turns
    assert np.allclose(ev, [2.0, 2.0, 1.0])
    assert np.allclose(quat2mat(q).T @ np.diag([1.0, 2.0, 2.0]) @ quat2mat(q), np.diag(ev), atol=1e-12)
