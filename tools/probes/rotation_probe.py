"""In-launch rotation on the drop-in API's rollout call (GPU box): the
collision-free subset of one 8192-candidate batch (the filter_to_stable
pattern), env.rollout with yield_every 0 / 8 / 16 / 32 / 64; prints the
rollout kernel's duration, the launch grid, and the fail-step histogram."""
import os
import sys
import time

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
    mask = env.grasp_collision_mask(poses, J)
    idx = np.nonzero(mask)[0]
    plan = env.rollout_plan(poses[idx], J[idx], nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                            close_steps=h["close_steps"], lift_check_every=h["lift_check_every"])
    n = len(idx)
    print(f"rollouts {n}, grid {env.engine.rollout_grid(n)}")
    ref = None
    for y in (0, 8, 16, 32, 64, 0):
        ts, ks = [], []
        for it in range(4):
            t0 = time.perf_counter()
            r = env.rollout(plan, yield_every=y)
            ts.append(time.perf_counter() - t0)
            ks.append(r["kernel_ms"])
        if ref is None:
            ref = r
            fs = r["fail_step"]
            steps = np.where(fs < 0, plan.horizon, fs + 1)
            print("executed steps per rollout: mean %.1f, full-length %d of %d; candidate-steps %d"
                  % (steps.mean(), int((fs == -1).sum()), n, int(steps.sum())))
        same = all(np.array_equal(r[k], ref[k]) for k in ("label", "fail_step", "obj_qpos", "stats"))
        print(f"yield_every {y:3d}: env.rollout {1e3 * np.median(ts):7.2f} ms, kernel {np.median(ks):7.2f} ms "
              f"(min {min(ks):.2f}), outputs identical {same}")


if __name__ == "__main__":
    main()
