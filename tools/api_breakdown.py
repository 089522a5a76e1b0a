"""Where the drop-in API's time goes for one 8192-candidate filter_to_stable
call (mgs/cli/filter_to_stable.py:39-50): host pose processing, the mask
launch, the stability call's plan building, its rollout launch(es), the rest.
GPU box; prints one line per stage (median of 5 calls after 2 warm-up calls).

    python tools/api_breakdown.py [yield_every]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mj-grasp-sim_amd")]


def main():
    import numpy as np
    import torch
    torch.cuda.init()
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping, HORIZONS
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.obj.selector import get_object
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose
    env = GravitylessObjectGrasping(GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz")),
                                    get_object("003_cracker_box"))
    if len(sys.argv) > 1:
        env.YIELD_EVERY = int(sys.argv[1])
    h = HORIZONS["h200"]
    H, J, _ = robotiq_candidates(env.obj, 8192, seed=0)
    poses = SE3Pose.from_mat(H)
    rows = []
    for it in range(7):
        t = [time.perf_counter()]
        q, mp, mq, _ = env.initial_state(poses, J)
        t.append(time.perf_counter())
        mask = env.engine.collision_free(q, mp, mq)
        t.append(time.perf_counter())
        idx = np.nonzero(mask)[0]
        plan = env.rollout_plan(poses[idx], J[idx], nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                                close_steps=h["close_steps"], lift_check_every=h["lift_check_every"])
        t.append(time.perf_counter())
        res = env.rollout(plan)
        t.append(time.perf_counter())
        if it >= 2:
            rows.append(np.diff(t) * 1e3)
    m = np.median(np.array(rows), 0)
    names = ["initial_state (host SE3, 8192)", "collision_free (upload, launch, download)",
             "rollout_plan (host SE3 + schedule, %d)" % len(idx), "env.rollout (rotation every %d steps)" % env.YIELD_EVERY]
    for n, v in zip(names, m):
        print(f"{n:48s} {v:8.2f} ms")
    print(f"{'total':48s} {m.sum():8.2f} ms  -> {8192 / m.sum() * 1e3:.0f} candidates/s; "
          f"last rollout kernel {res.get('kernel_ms', float('nan')):.1f} ms")


if __name__ == "__main__":
    main()
