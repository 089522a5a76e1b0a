"""Critical path of one drop-in API rollout launch (GPU box): the collision-free
subset of one 8192-candidate batch; each candidate's solo latency (a launch of
that candidate alone) for the heaviest ones by solver work and for a spread of
typical ones, against the whole launch's duration."""
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
    mask = env.grasp_collision_mask(poses, J)
    idx = np.nonzero(mask)[0]
    plan = env.rollout_plan(poses[idx], J[idx], nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                            close_steps=h["close_steps"], lift_check_every=h["lift_check_every"])
    eng = env.engine
    whole = [eng.rollout(plan)["kernel_ms"] for _ in range(3)]
    r = eng.rollout(plan)
    st = r["stats"]
    fs = r["fail_step"]
    steps = np.where(fs < 0, plan.horizon, fs + 1)
    print(f"whole launch ({len(idx)} rollouts): {np.median(whole):.2f} ms")
    cost = st[:, 5].astype(float)      # sum of constraint rows over the executed steps
    order = np.argsort(-cost)
    pick = list(order[:12]) + list(order[len(order) // 4::len(order) // 8][:6])
    print(" cand  steps  iters  sum_ncon  sum_nefc   solo ms   us/step")
    solo = []
    for c in pick:
        sub = plan.subset(np.array([c]))
        ms = np.median([eng.rollout(sub)["kernel_ms"] for _ in range(3)])
        solo.append(ms)
        print(f"{c:5d} {steps[c]:6d} {st[c, 3]:6d} {st[c, 4]:9d} {st[c, 5]:9d} {ms:9.2f} {1e3 * ms / steps[c]:9.1f}")
    # every full-length candidate alone would take how long? extrapolate by rows
    a = np.polyfit(cost[pick] / steps[pick], np.array(solo) / steps[pick], 1)
    est = steps * np.polyval(a, cost / steps)
    print(f"per-step solo cost ~ {a[0] * 1e3:.2f} us per row + {a[1] * 1e3:.1f} us; estimated solo latency: "
          f"max {est.max():.1f} ms, 99th pct {np.percentile(est, 99):.1f}, median {np.median(est):.1f}; "
          f"sum / 1024 slots = {est.sum() / 1024:.1f} ms")


if __name__ == "__main__":
    main()
