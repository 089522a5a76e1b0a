"""Robotiq free-space close against the reference's recorded closed state
(state_close, mgs/cli/config/gripper/robotiq_2f_85.yaml:11): is the offset of
the oracle's rest state a trajectory effect (friction-stick equilibria) or a
model effect?  Runs the oracle (CPU) from perturbed starts / close profiles
and with perturbed contact and constraint parameters, and prints the rest
joints against the recorded ones.  Output: profiles/r03_state_close_experiment.txt
    python tools/state_close_experiment.py"""
import copy
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mj-grasp-sim_amd")]

# state_close joints (right driver, coupler, spring link, follower, then left)
KAT = np.array([7.93116751e-01, 3.48441304e-04, 7.89591521e-01, -7.76735418e-01,
                7.93117030e-01, 3.47173334e-04, 7.89598436e-01, -7.76696653e-01])


def main():
    from oracle import oracle as O
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.obj.selector import get_object
    from mgs.util.geo.transforms import SE3Pose
    env = GravitylessObjectGrasping(GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz")),
                                    get_object("003_cracker_box"))
    pose = SE3Pose(np.array([[0.0, 0.0, 0.0]]), np.array([[1.0, 0, 0, 0]]), "wxyz")
    q0, mp, mq, _ = env.initial_state(pose, np.zeros((1, 8)))
    q0 = q0[0]
    q0[17] = 0.4       # object out of reach, as in the recorded state
    rows = []

    def run(cm, q, label, n=6000, pre=None):
        om = O.OracleModel(cm)
        if pre is not None:
            tr, _, _ = om.trace(q, mp[0], mq[0], np.array([pre]), 1500)
            q = tr[-1].copy()
        tr, nc, qv = om.trace(q, mp[0], mq[0], np.array([255.0]), n)
        j = tr[-1, 7:15]
        rows.append((label, j))
        d = j - KAT
        print(f"{label:46s} driver {d[0]:+.2e} {d[4]:+.2e}  spring {d[2]:+.2e} {d[6]:+.2e}  "
              f"follower {d[3]:+.2e} {d[7]:+.2e}  |qvel| {np.abs(qv).max():.1e}  ncon {nc[-1]}")

    cm = env.model
    print("rest joints minus state_close (rad), oracle, 6 s of ctrl=255 in free space\n")
    print("-- trajectory: perturbed starts and close profiles --")
    run(cm, q0.copy(), "open start")
    for k, dj in [(7, 0.05), (11, 0.05), (7, 0.2), (11, 0.2), (9, 0.05), (13, -0.05)]:
        q = q0.copy()
        q[k] += dj
        run(cm, q, f"start qpos[{k}] {dj:+}")
    for c in (200.0, 230.0):
        run(cm, q0.copy(), f"1.5 s at ctrl {c:.0f}, then 255", pre=c)
    J = np.array([r[1] for r in rows])
    print("spread over these starts (max - min):", np.array2string(J.max(0) - J.min(0), precision=7))
    print("\n-- model: one parameter changed at a time --")
    bb = cm.pair_kind == 1
    v = copy.copy(cm); v.pair_kind = np.zeros_like(cm.pair_kind)
    run(v, q0.copy(), "box pairs through MPR + clipping (not box-box)")
    for tc in (0.002, 0.008):
        v = copy.copy(cm); ps = cm.pair_solref.copy(); ps[bb, 0] = tc; v.pair_solref = ps
        run(v, q0.copy(), f"pad contact solref timeconst {tc}")
    for w in (0.0005, 0.002):
        v = copy.copy(cm); si = cm.pair_solimp.copy(); si[bb, 2] = w; v.pair_solimp = si
        run(v, q0.copy(), f"pad contact solimp width {w}")
    for tc in (0.01, 0.04):
        v = copy.copy(cm); es = cm.eq_solref.copy(); es[:, 0] = tc; v.eq_solref = es
        run(v, q0.copy(), f"equality solref timeconst {tc}")
    for ir in (3.0, 30.0):
        v = copy.copy(cm); v.options = dict(cm.options, impratio=ir)
        run(v, q0.copy(), f"impratio {ir}")
    for ks in (0.045, 0.055):
        v = copy.copy(cm); st = cm.jnt_stiffness.copy(); st[st > 0] = ks; v.jnt_stiffness = st
        run(v, q0.copy(), f"spring-link stiffness {ks}")


if __name__ == "__main__":
    main()
