"""Diagnostic: how many rollout workgroups a CU holds at once.  The same
collision-free headline candidate copied N times (identical work per wave),
rollout kernel time against N: a step in the time appears where N passes the
number of resident slots (CUs x workgroups per CU)."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "mj-grasp-sim_amd"))


def main():
    import torch
    torch.cuda.init()
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping, HORIZONS
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.obj.selector import get_object
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose
    os.environ.setdefault("MGS_SPECIALIZE", "1")
    env = GravitylessObjectGrasping(GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz")),
                                    get_object("003_cracker_box"))
    H, J, _ = robotiq_candidates(env.obj, 256, seed=2)
    P = SE3Pose.from_mat(H)
    q, mp, mq, _ = env.initial_state(P, J)
    eng = env.engine
    free = np.nonzero(eng.collision_free(q, mp, mq))[0]
    h = HORIZONS["h200"]
    plan1 = env.rollout_plan(P[free[:8]], J[free[:8]], nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                             close_steps=h["close_steps"], lift_check_every=h["lift_check_every"])
    r = eng.rollout(plan1)
    k = int(np.argmax(r["fail_step"] < 0)) if (r["fail_step"] < 0).any() else 0     # one that runs all steps
    print("lds bytes per candidate", eng.lds_bytes(), "specialised", eng.specialized())
    for n in [256, 512, 768, 769, 900, 1024, 1025, 1280, 1536, 2048]:
        plan = plan1.subset(np.full(n, k))
        ms = []
        for _ in range(2):
            eng.rollout(plan)
            ms.append(eng.last_kernel_ms())
        print(f"N={n:5d} kernel_ms={min(ms):8.2f}", flush=True)


if __name__ == "__main__":
    main()
