"""Which headline engine finishes a rollout call of n collision-free candidates
sooner: the G-rows-in-HBM object (eight per CU, the throughput engine) or the
G-rows-in-LDS one (four per CU, shorter steps)?  A call of n <= the resident
slots is one round of rollouts, i.e. the heaviest rollout's latency.  Prints
the median wall time of env.rollout's path (sliced_rollout: escalation and
rotation as the env runs them) per n and engine.  GPU box:
    python tools/probes/latency_engine_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mj-grasp-sim_amd")]


def main():
    import numpy as np
    import torch
    torch.cuda.init()
    from mgs.core.engine import Engine
    from mgs.env.gravityless_object_grasping import HORIZONS, GravitylessObjectGrasping, sliced_rollout
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.obj.selector import get_object
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose
    env = GravitylessObjectGrasping(GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz")),
                                    get_object("003_cracker_box"))
    h = HORIZONS["h200"]
    H, J, _ = robotiq_candidates(env.obj, 8192 * 3, seed=0)
    poses = SE3Pose.from_mat(H)
    q, mp, mq, _ = env.initial_state(poses, J)
    free = np.nonzero(env.engine.collision_free(q, mp, mq))[0]
    engines = {"hbm": Engine(env.model, ncon_max=env.ncon_max, nefc_max=env.nefc_max, g_rows_hbm=True),
               "lds": Engine(env.model, ncon_max=env.ncon_max, nefc_max=env.nefc_max, g_rows_hbm=False,
                             specialize="cached")}
    for name, e in engines.items():
        print(f"{name}: specialised {e.specialized()}, resident grid {e.rollout_grid(4096)}", flush=True)
    for n in (512, 1024, 1173, 1536, 2048, 3072):
        idx = free[:n]
        plan = env.rollout_plan(poses[idx], J[idx], nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                                close_steps=h["close_steps"], lift_check_every=h["lift_check_every"])
        line = [f"n {n:5d}"]
        labels = {}
        for name, e in engines.items():
            ts = []
            for it in range(4):
                t = time.perf_counter()
                r = sliced_rollout(plan, e, env.engine_for, env.ncon_max, 40, 1, yield_every=env.YIELD_EVERY)
                ts.append(time.perf_counter() - t)
            labels[name] = r["label"]
            line.append(f"{name} {np.median(ts[1:]) * 1e3:7.1f} ms")
        line.append("labels equal" if np.array_equal(labels["hbm"], labels["lds"]) else "LABELS DIFFER")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
