"""Host-side schedules vs the reference harness beyond Robotiq x gravityless
(tests/golden/harness_grippers_golden.npz, harness_clutter_golden.npz, made by
tests/golden/make_golden_more.py from the reference's own env / gripper
classes under a recording mujoco stand-in; no physics involved).

  * Panda, Allegro, Shadow close_gripper_at + lift + shake: initial qpos and
    every step's mocap pose and ctrl, bit for bit.
  * ClutterTableEnv: the collision mask (workspace box + the inclusive gripper
    predicate) and the stable mask (scene state, close, 0.3 m lift, the
    (t + 1) % 100 cadence, the strict gripper predicate, enough_stable) on
    scripted contacts, with the kernels' predicate (oracle_contact_predicate)
    and the plan's check schedule."""
import json
import os

import numpy as np
import pytest

from test_golden_harness import expand

HERE = os.path.dirname(os.path.abspath(__file__))
GRIP = os.path.join(HERE, "golden", "harness_grippers_golden.npz")
CLUT = os.path.join(HERE, "golden", "harness_clutter_golden.npz")
NAMES = {"panda": "PandaGripper", "allegro": "AllegroGripper", "shadow": "ShadowHand"}


@pytest.mark.parametrize("key", ["panda", "allegro", "shadow"])
def test_gripper_close_lift_shake_schedule(key):
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_object
    from mgs.util.geo.transforms import SE3Pose
    g = np.load(GRIP)
    env = GravitylessObjectGrasping(get_gripper({"name": NAMES[key]}), get_object("003_cracker_box"))
    poses = SE3Pose.from_mat(g[f"{key}_poses"])
    J = g[f"{key}_joints"]
    q, _, _, _ = env.initial_state(poses, J)
    assert np.array_equal(q, g[f"{key}_qpos0"])
    plan = env.rollout_plan(poses, J, nstep_lift=int(g["nstep_lift"]), shake_steps=int(g["shake_steps"]),
                            close_steps=3000)
    for i in range(len(J)):
        n = int(g[f"{key}_nsteps"][i])
        assert n == plan.horizon
        ref = g[f"{key}_traj"][i, :n]
        mine = expand(plan, i)
        assert mine.shape == ref.shape
        assert np.array_equal(mine, ref), f"{key} candidate {i}: first diff at step {np.argmax((mine != ref).any(1))}"


@pytest.fixture(scope="module")
def clutter():
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_clutter_scene import make_env
    from oracle import oracle as O
    g = np.load(CLUT)
    env = make_env()
    env.set_state(g["state"])
    cm = env.model
    om = O.OracleModel(cm)
    gbody = [cm.body_names[b] for b in cm.geom_bodyid]
    ids = {"G": cm.geom_names.index("right_pad1"), "O": gbody.index("obj0"), "O2": gbody.index("obj1")}

    def pairs(spec):
        return [[ids[a] if a in ids else cm.geom_names.index(a), ids[b] if b in ids else cm.geom_names.index(b)]
                for a, b in spec]
    return env, om, g, pairs


def test_clutter_collision_mask_rules(clutter):
    from oracle import oracle as O
    from mgs.util.geo.transforms import SE3Pose
    env, om, g, pairs = clutter
    poses = SE3Pose.from_mat(g["poses"])
    inb = env.in_bounds(poses)
    scripts = json.loads(str(g["mask_contacts"]))
    mine = [bool(inb[i]) and not O.contact_predicate(om, pairs(scripts[i]), "partition_incl")
            for i in range(len(scripts))]
    assert mine == g["mask"].tolist()
    assert not all(mine) and any(mine)


def _scripted_rollout(plan, i, om, close_pairs, lift_pairs, lose, pairs):
    """the kernel's check schedule (check after step t of a phase if
    check_every > 0 and (t + off) > 0 and (t + off) % check_every == 0) on a
    scripted contact list; returns (label, steps, check steps)"""
    from oracle import oracle as O
    close = plan.nsteps[0]
    g, checks = 0, []
    for p, n in enumerate(plan.nsteps):
        ce, off = plan.check_every[p], plan.check_offset[p]
        for t in range(n):
            g += 1
            if ce > 0 and (t + off) > 0 and (t + off) % ce == 0:
                checks.append(g)
                if g <= close:
                    cs = close_pairs
                elif lose >= 0 and g > close + lose:
                    cs = []
                else:
                    cs = lift_pairs
                if not O.contact_predicate(om, pairs(cs), "partition"):
                    return False, g, checks
        if plan.check_at_end[p]:
            raise AssertionError("the clutter lift has no end-of-phase check")
    return True, g, checks


def test_clutter_stable_mask_schedule(clutter):
    from mgs.env.gravityless_object_grasping import apply_enough_stable
    from mgs.util.geo.transforms import SE3Pose
    env, om, g, pairs = clutter
    poses = SE3Pose.from_mat(g["poses"])
    J = g["joints"]
    st = g["state"]
    scripts = json.loads(str(g["stable_contacts"]))
    plan = env.stable_plan(poses, J, st, nstep_lift=int(g["nstep_lift"]), close_steps=int(g["close_steps"]))
    q, _, _ = env._initial_qpos(poses, J, st)
    labels = []
    for i, (cc, lc, lose) in enumerate(scripts):
        assert np.array_equal(q[i], env._reduce(g["qpos0"][i], "q")), i
        n = int(g["nsteps"][i])
        ref = g["traj"][i, :n]
        assert np.array_equal(expand(plan, i)[:n], ref), i
        lab, steps, checks = _scripted_rollout(plan, i, om, cc, lc, lose, pairs)
        assert lab == bool(g["labels"][i]), i
        assert steps == n, i
        assert checks == [c for c in g["checks"][i] if c >= 0 and c > int(g["close_steps"])], i
        labels.append(lab)
    assert not all(labels) and any(labels)
    assert apply_enough_stable(np.array(labels), int(g["enough_stable"])).tolist() == \
        g["enough_stable_labels"].tolist()
