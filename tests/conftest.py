import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mj-grasp-sim_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X; runs the HIP engine through the C-ABI")


def pytest_runtest_setup(item):
    """GPU tests start the HIP runtime through torch first (the engine's device
    count is read after it), whichever GPU test of a selection runs first"""
    if item.get_closest_marker("gpu") is not None:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()


@pytest.fixture(scope="session")
def env():
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.obj.selector import get_object
    from mgs.util.geo.transforms import SE3Pose
    grip = GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz"))
    return GravitylessObjectGrasping(grip, get_object("003_cracker_box"))


@pytest.fixture(scope="session")
def candidates(env):
    """256 seeded antipodal candidates (poses as SE3Pose, joints zeros(8))."""
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose
    H, J, W = robotiq_candidates(env.obj, 256, seed=0)
    return SE3Pose.from_mat(H), np.asarray(J, np.float64)


@pytest.fixture(scope="session")
def oracle_model(env):
    from oracle import oracle as O
    return O.OracleModel(env.model, ncon_max=env.ncon_max, nefc_max=env.nefc_max)


def full_capacity_oracle(env, state):
    """the oracle at a clutter env's last escalation capacity (128 contacts,
    256 rows: sliced_rollout's max_ncon and the wide library's rows), which a
    run escalated from the env's main capacity equals bit for bit"""
    from oracle import oracle as O
    return O.OracleModel(env.model_for(state), ncon_max=128, nefc_max=256)


def plan_for(env, poses, joints, horizon="h200"):
    from mgs.env.gravityless_object_grasping import HORIZONS
    h = HORIZONS[horizon]
    return env.rollout_plan(poses, joints, nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                            close_steps=h["close_steps"], lift_check_every=h["lift_check_every"])
