"""Host-side schedule vs the reference harness (tests/golden/harness_golden.npz,
made by tests/golden/make_golden.py from the reference's own
GravitylessObjectGrasping / GripperRobotiq2f85 / SE3Pose under a recording
mujoco stand-in).  Pins: float32 pose processing, the joint-index quirk, the
initial qpos, the per-step mocap pose and ctrl of close/lift/back/right/left,
the check points, early exits and labels under a scripted contact oracle.
Physics is not involved (MuJoCo is absent): parity of the physics itself is
covered against the oracle in test_gpu_parity.py."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "harness_golden.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


@pytest.fixture(scope="module")
def gplan(env, gold):
    from mgs.util.geo.transforms import SE3Pose
    poses = SE3Pose.from_mat(gold["poses"])
    return env.rollout_plan(poses, gold["joints"], nstep_lift=int(gold["nstep_lift"]),
                            shake_steps=int(gold["shake_steps"]), close_steps=int(gold["close_steps"]),
                            lift_check_every=100)


def expand(plan, i):
    """Per-step control exactly as the rollout kernel forms it (mgs_kernels.hip
    mgs_rollout_kernel / oracle_rollout): mocap = start + (target - start) * (t / n)."""
    rows = []
    for p, n in enumerate(plan.nsteps):
        ps, pt = plan.phase_start[i, p], plan.phase_target[i, p]
        for t in range(n):
            pos = ps + (pt - ps) * (float(t) / float(n))
            rows.append(np.concatenate([pos, plan.mocap_quat[i], plan.ctrl[p]]))
    return np.array(rows)


def checks_and_exit(plan, lose_after):
    """The kernel's check schedule (global step count after which the contact
    predicate is read) and its early exit under 'contact lost after step k'."""
    checks, g = [], 0
    for p, n in enumerate(plan.nsteps):
        ce = plan.check_every[p]
        for t in range(n):
            g += 1
            if ce > 0 and t > 0 and t % ce == 0:
                checks.append(g)
                if lose_after >= 0 and g > lose_after:
                    return checks, False, g
        if plan.check_at_end[p]:
            checks.append(g)
            if lose_after >= 0 and g > lose_after:
                return checks, False, g
    return checks, True, g


def test_initial_qpos_matches_reference(env, gold):
    from mgs.util.geo.transforms import SE3Pose
    q, mp, mq, _ = env.initial_state(SE3Pose.from_mat(gold["poses"]), gold["joints"])
    assert np.array_equal(q, gold["qpos0"])


def test_joint_index_quirk(env):
    idxs = env.get_joint_idxs(env.gripper.get_actuator_joint_names())
    assert idxs == [7, 8, 15, 10, 11, 12, 15, 14]


def test_per_step_controls_bit_exact(gplan, gold):
    for i in range(len(gold["labels"])):
        n = int(gold["nsteps"][i])
        ref = gold["traj"][i, :n]
        mine = expand(gplan, i)[:n]
        assert np.array_equal(mine, ref), f"candidate {i}: first diff at step {np.argmax((mine != ref).any(1))}"


def test_check_points_labels_and_exits(gplan, gold):
    for i in range(len(gold["labels"])):
        checks, label, nsteps = checks_and_exit(gplan, int(gold["lose_after"][i]))
        ref_checks = [c for c in gold["checks"][i] if c >= 0]
        assert checks == ref_checks, i
        assert label == bool(gold["labels"][i]), i
        assert nsteps == int(gold["nsteps"][i]), i


def test_schedule_shape(gplan, gold):
    assert gplan.nsteps == [3000, int(gold["nstep_lift"]), int(gold["shake_steps"]), int(gold["shake_steps"]),
                            2 * int(gold["shake_steps"])]
    assert gplan.horizon == gold["traj"].shape[1]
