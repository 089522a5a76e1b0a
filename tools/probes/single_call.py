"""One drop-in API rollout launch (GPU box): the collision-free subset of the
headline's 8192-candidate batch (1173 rollouts), median kernel ms of 5
launches -- the critical path of the API call (tools/probes/critical_path_probe.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    h = HORIZONS["h200"]
    H, J, _ = robotiq_candidates(env.obj, 8192, seed=0)
    poses = SE3Pose.from_mat(H)
    idx = np.nonzero(env.grasp_collision_mask(poses, J))[0]
    plan = env.rollout_plan(poses[idx], J[idx], nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                            close_steps=h["close_steps"], lift_check_every=h["lift_check_every"])
    ks = [env.rollout(plan)["kernel_ms"] for _ in range(6)][1:]
    r = env.rollout(plan)
    print(f"single call: {len(idx)} rollouts, kernel {np.median(ks):.2f} ms (min {min(ks):.2f}), "
          f"stable {int(r['label'].sum())}, specialised {env.engine.specialized()}")


if __name__ == "__main__":
    main()
