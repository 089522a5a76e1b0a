"""mgs.cli drop-ins (reference mgs/cli/*.py): Hydra-style config composition,
the grasp-set file format, and (GPU) the gen_grasps / filter_to_stable
pipelines against the oracle."""
import os

import numpy as np
import pytest


def test_compose_defaults_and_overrides():
    from mgs.cli._hydra import compose
    c = compose("filter_to_stable", ["gripper=panda", "id=2", "horizon=h200"])
    assert c.gripper.name == "PandaGripper" and c.id == 2 and c.horizon == "h200"
    assert compose("gen_grasp_candidates").gripper.name == "Robotiq2f85Gripper"
    with pytest.raises(ValueError):
        compose("filter_to_stable", ["gripper=nope"])


def test_gen_grasp_candidates_file_format(tmp_path, monkeypatch):
    from mgs.cli import gen_grasp_candidates
    monkeypatch.setenv("MGS_OUTPUT_DIR", str(tmp_path))
    gen_grasp_candidates.run(["gripper=panda", "id=0", "num_grasps=32", "sampler=host"])
    z = np.load(tmp_path / "PandaGripper" / "003_cracker_box" / "candidates.npz")
    assert z["pose"].shape == (32, 4, 4) and z["pose"].dtype == np.float32
    assert z["joints"].shape == (32, 2)
    assert np.allclose(z["pose"][:, 3], [0, 0, 0, 1])


@pytest.mark.gpu
def test_gen_grasps_and_filter_to_stable(tmp_path, monkeypatch):
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
    from conftest import plan_for
    from mgs.cli import filter_to_stable, gen_grasps
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping, apply_enough_stable
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_object
    from mgs.util.geo.transforms import SE3Pose
    from oracle import oracle as O
    monkeypatch.setenv("MGS_OUTPUT_DIR", str(tmp_path))
    monkeypatch.setenv("MGS_INPUT_DIR", str(tmp_path))
    gen_grasps.run(["id=0", "num_grasps=256", "horizon=h200", "enough_stable=20"])    # device sampler
    d = tmp_path / "Robotiq2f85Gripper" / "003_cracker_box"
    cand = np.load(d / "candidates.npz")
    stable = np.load(d / "stable_grasps.npz")
    env = GravitylessObjectGrasping(get_gripper({"name": "Robotiq2f85Gripper"}), get_object("003_cracker_box"))
    om = O.OracleModel(env.model, ncon_max=env.ncon_max, nefc_max=env.nefc_max)
    P = SE3Pose.from_mat(cand["pose"])
    q, mp, mq, _ = env.initial_state(P, cand["joints"])
    free = om.collision_free(q, mp, mq, nthreads=8)
    idx = np.nonzero(free)[0]
    lab = apply_enough_stable(om.rollout(plan_for(env, P[idx], cand["joints"][idx]), nthreads=8)["label"], 20)
    # files hold SE3Pose.to_mat() of the processed poses, as the reference writes them
    assert np.array_equal(stable["pose"], P[idx[lab]].to_mat())
    # the reference's filter_to_stable on the same candidates file
    filter_to_stable.run(["id=0", "horizon=h200"])
    cf = np.load(d / "candidates_collision_free.npz")
    assert np.array_equal(cf["pose"], P[idx].to_mat())
