"""ClutterTableEnv: grasp_collision_mask and
grasp_stable_mask over a settled 5-object pile (tests/golden/clutter_scene.npz,
made by tests/golden/make_clutter_scene.py on the oracle).

CPU: the scene-dict / integration-state round trip, the reference's host rules
(in-bounds box :344-354, the inclusive collision predicate vs the strict lift
predicate :237-270, the (t + 1) % 100 lift cadence :313), and that the oracle's
lifted grasps hold objects.  GPU: both methods bit-exact against the oracle
through the wide library (4 constraint rows per lane, G rows in HBM)."""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SCENE = os.path.join(HERE, "golden", "clutter_scene.npz")


@pytest.fixture(scope="module")
def cenv():
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_clutter_scene import make_env
    z = np.load(SCENE)
    env = make_env()
    env.set_state(z["state"])
    return env


@pytest.fixture(scope="module")
def ccand(cenv):
    """antipodal Robotiq grasps of every object in its own frame, posed by the
    settled object pose (gen_scene.py:59-66: o2w @ pose)."""
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose
    H, J = [], []
    for k, o in enumerate(cenv.objects):
        h, j, _ = robotiq_candidates(o, 48, seed=k)
        o2w = cenv.get_obj_pose(o.name)
        H.append((o2w @ SE3Pose.from_mat(h)).to_mat())
        J.append(j)
    return SE3Pose.from_mat(np.concatenate(H).astype(np.float32)), np.concatenate(J)


def test_state_layout_and_dict_roundtrip(cenv):
    from mgs.env.clutter_table import ClutterTableEnv
    cm = cenv.model
    # reference layout: gripper (22 -> 15 qpos) + camera free joint + 5 objects
    assert cenv.ref_nq == cm.nq + 7 and cenv.ref_nv == cm.nv + 6
    assert cm.nv == 14 + 6 * 5
    s = cenv.get_state()
    assert s.shape == (cenv.state_size(),)
    d = cenv.to_dict()
    e2 = ClutterTableEnv.from_dict(d)
    assert np.array_equal(e2.get_state(), s)
    assert cm.geom_names.index("geom:table") < cm.geom_names.index("geom:camera")


def test_collision_mask_rules(cenv, ccand):
    from oracle import oracle as O
    poses, J = ccand
    p = poses.pos
    inb = (np.abs(p[:, 0]) < 0.25) & (np.abs(p[:, 1]) < 0.25) & (p[:, 2] > 0) & (p[:, 2] < 1)
    q, mp, mq = cenv._initial_qpos(poses, J, cenv.get_state())
    om = O.OracleModel(cenv.model, ncon_max=cenv.ncon_max, nefc_max=256)
    incl = om.collision_free(q, mp, mq, predicate="partition_incl", nthreads=8)
    strict = om.collision_free(q, mp, mq, predicate="partition", nthreads=8)
    anyc = om.collision_free(q, mp, mq, predicate="any", nthreads=8)
    # gripper-table contacts count as collisions for the mask, not for the lift check
    assert np.all(incl <= strict) and np.all(anyc <= incl)
    assert 0 < (incl & inb).sum() < len(inb)


def test_stable_plan_cadence(cenv, ccand):
    poses, J = ccand
    plan = cenv.stable_plan(poses[:2], J[:2], cenv.get_state())
    assert plan.nsteps == [3000, 3000] and plan.check_every == [0, 100] and plan.check_offset == [0, 1]
    assert np.allclose(plan.phase_target[:, 1, 2] - plan.phase_start[:, 1, 2], 0.3)
    assert plan.check_at_end == [0, 0]


def test_oracle_stable_grasps_hold(cenv, ccand):
    from oracle import oracle as O
    poses, J = ccand
    st = cenv.get_state()
    q, mp, mq = cenv._initial_qpos(poses, J, st)
    om = O.OracleModel(cenv.model_for(st), ncon_max=cenv.ncon_max, nefc_max=256)
    free = om.collision_free(q, mp, mq, predicate="partition_incl", nthreads=8)
    idx = np.nonzero(free)[0][:12]
    plan = cenv.stable_plan(poses[idx], J[idx], st, nstep_lift=600, close_steps=600)
    r = om.rollout(plan, nthreads=8)
    assert len(idx) == 12 and r["label"].sum() >= 4
    assert np.all(np.isin(r["fail_step"][~r["label"]], 600 + np.arange(99, 600, 100)))


@pytest.mark.gpu
def test_clutter_gpu_parity(cenv, ccand):
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
    from oracle import oracle as O
    poses, J = ccand
    st = cenv.get_state()
    eng = cenv.engine_for_state(st)
    om = O.OracleModel(cenv.model_for(st), ncon_max=cenv.ncon_max, nefc_max=eng.desc.nefc_max)
    mask = cenv.grasp_collision_mask(poses, J)
    p = poses.pos
    inb = (np.abs(p[:, 0]) < 0.25) & (np.abs(p[:, 1]) < 0.25) & (p[:, 2] > 0) & (p[:, 2] < 1)
    q, mp, mq = cenv._initial_qpos(poses, J, st)
    ref = om.collision_free(q, mp, mq, predicate="partition_incl", nthreads=8) & inb
    assert np.array_equal(mask, ref)
    idx = np.nonzero(mask)[0][:24]
    plan = cenv.stable_plan(poses[idx], J[idx], st, nstep_lift=600, close_steps=600)
    rg, ro = eng.rollout(plan), om.rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "stats"):
        assert np.array_equal(rg[k], ro[k]), k
    lab = cenv.grasp_stable_mask(poses[idx], J[idx], st, nstep_lift=600, close_steps=600, enough_stable=3)
    from conftest import full_capacity_oracle
    rf = full_capacity_oracle(cenv, st).rollout(plan, nthreads=8)     # the env escalates past its capacity
    assert lab.sum() == min(3, int(rf["label"].sum()))


def test_scene_file_roundtrip(cenv, tmp_path):
    from mgs.env.selector import get_env_from_dict, load_scene, save_scene
    save_scene(tmp_path / "scene.npz", cenv.to_dict())
    sd = load_scene(tmp_path / "scene.npz")
    e2 = get_env_from_dict({"name": "ClutterTable"}, sd)
    assert np.array_equal(e2.get_state(), cenv.get_state())
    assert e2.object_names == cenv.object_names and type(e2.gripper) is type(cenv.gripper)


@pytest.mark.gpu
def test_eval_grasps_cli(cenv, ccand, tmp_path, monkeypatch):
    """eval_grasps.py:13-82 on a scene directory: success rate = stable / all."""
    from mgs.cli import eval_grasps
    from mgs.env.selector import save_scene
    from oracle import oracle as O
    poses, J = ccand
    d = tmp_path / "Robotiq2f85Gripper" / "scene_000"
    d.mkdir(parents=True)
    save_scene(d / "scene.npz", cenv.to_dict())
    sel = np.arange(0, len(J), 4)
    np.savez(d / "inference_grasps.npz", pose=poses[sel].to_mat(), joints=J[sel])
    monkeypatch.setenv("MGS_INPUT_DIR", str(tmp_path))
    eval_grasps.run(["id=0", "lift_steps=300"])
    import json
    res = json.load(open(d / "grasp_evaluation.json"))
    # oracle: the same pipeline (inverse b2c, then the env's own b2c, mask, stable)
    from mgs.util.geo.transforms import SE3Pose
    b2c_inv = cenv.gripper.base_to_contact_transform().inverse().to_mat()
    P = SE3Pose.from_mat(np.einsum("nij,jk->nik", poses[sel].to_mat(), b2c_inv))
    st = cenv.get_state()
    eng = cenv.engine_for_state(st)
    om = O.OracleModel(cenv.model_for(st), ncon_max=cenv.ncon_max, nefc_max=eng.desc.nefc_max)
    q, mp, mq = cenv._initial_qpos(P, J[sel], st)
    p = P.pos
    inb = (np.abs(p[:, 0]) < 0.25) & (np.abs(p[:, 1]) < 0.25) & (p[:, 2] > 0) & (p[:, 2] < 1)
    free = om.collision_free(q, mp, mq, predicate="partition_incl", nthreads=8) & inb
    idx = np.nonzero(free)[0]
    lab = om.rollout(cenv.stable_plan(P[idx], J[sel][idx], st, nstep_lift=300, close_steps=300), nthreads=8)["label"]
    assert res["success_rate"] == pytest.approx(lab.sum() / len(sel)) and res["num_objects"] == 5


def test_oversized_pile_fails_clearly():
    """the kernels hold at most 128 dofs (any count up to that runs, through a
    specialised code object where the libraries have no instantiation, two
    dofs per lane past 64); a pile beyond it is refused when the env is built,
    with the largest pile size in the message (not at the first simulation)"""
    from mgs.env.clutter_table import ClutterTableEnv
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.obj.selector import get_object
    from mgs.util.geo.transforms import SE3Pose
    grip = GripperRobotiq2f85(SE3Pose(np.array([5.0, 5.0, 1.0]), np.array([1.0, 0, 0, 0]), "wxyz"))
    objs = [get_object("003_cracker_box") for _ in range(20)]
    for i, o in enumerate(objs):
        o.name = f"o{i}"
    with pytest.raises(ValueError, match="piles of at most 19 free objects"):
        ClutterTableEnv(grip, objs)


from mgs.core.shipped import SPREAD_PILES, spread_pile  # noqa: E402  (the shipped pile scenes)


@pytest.mark.gpu
@pytest.mark.parametrize("gripper,objects", SPREAD_PILES)
def test_any_pile_size_gpu_parity(gripper, objects):
    """piles of 3 (Robotiq) and 4 (Panda) objects: nv 32, a dof count no
    library instantiates, runs through a model-specialised code object, bit-exact
    against the oracle (mask and a close + lift rollout)"""
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
    from mgs.core.engine import supported_nvs
    from mgs.sampler.antipodal import hand_candidates, panda_candidates, robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose
    from oracle import oracle as O
    env = spread_pile(gripper, objects)
    st = env.get_state()
    assert env.model.nv == 32 and 32 not in supported_nvs()
    eng = env.engine_for_state(st)
    assert eng.specialized()
    H, J = [], []
    for k, o in enumerate(env.objects):
        if gripper == "PandaGripper":
            h, j = panda_candidates(o, 24, seed=k, gripper=env.gripper)[:2]
        else:
            h, j = robotiq_candidates(o, 24, seed=k)[:2]
        H.append((env.get_obj_pose(o.name) @ SE3Pose.from_mat(h)).to_mat())
        J.append(j)
    poses = SE3Pose.from_mat(np.concatenate(H).astype(np.float32))
    J = np.concatenate(J).astype(np.float64)
    om = O.OracleModel(env.model_for(st), ncon_max=env.ncon_max, nefc_max=eng.desc.nefc_max)
    mask = env.grasp_collision_mask(poses, J)
    q, mp, mq = env._initial_qpos(poses, J, st)
    ref = om.collision_free(q, mp, mq, predicate="partition_incl", nthreads=8) & env.in_bounds(poses)
    assert np.array_equal(mask, ref)
    idx = np.nonzero(mask)[0][:8]
    assert len(idx) >= 2
    plan = env.stable_plan(poses[idx], J[idx], st, nstep_lift=150, close_steps=150)
    rg, ro = eng.rollout(plan), om.rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(rg[k], ro[k]), k
