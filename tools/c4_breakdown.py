"""Where C4's call time goes (Allegro x GSO mug stand-in, 32768 candidates,
mask + h200 rollouts of the collision-free ones, tools/bench_configs.py c4):
host poses, the mask launch, the plan, the rollout call and its capacity
escalation stages.  GPU box; median of 3 calls after one warm-up.

    python tools/c4_breakdown.py [ncon_max]   (the main engine's contacts, default 20)"""
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mj-grasp-sim_amd")]


def main():
    import numpy as np
    import torch
    torch.cuda.init()
    import mgs.env.gravityless_object_grasping as G
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_object
    from mgs.sampler import antipodal
    from mgs.util.geo.transforms import SE3Pose
    h = G.HORIZONS["h200"]
    g = get_gripper({"name": "AllegroGripper"})
    ncon = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    env = G.GravitylessObjectGrasping(g, get_object("Synthetic_Mug_Body"), ncon_max=ncon)
    H, J, _ = antipodal.hand_candidates(env.obj, 32768, g, seed=0)
    P = SE3Pose.from_mat(H)
    # count the escalation stages of each rollout call
    stages = []
    orig = env.engine_for

    def counting(c):
        e = orig(c)
        inner = e.rollout

        def timed(plan, **kw):
            t = time.perf_counter()
            r = inner(plan, **kw)
            stages.append((c, len(plan.qpos_init), (time.perf_counter() - t) * 1e3, r.get("kernel_ms", float("nan"))))
            return r
        e.rollout = timed
        return e
    env.engine_for = counting
    rows = []
    labels = None
    for it in range(4):
        stages.clear()
        t = [time.perf_counter()]
        q, mp, mq, _ = env.initial_state(P, J)
        t.append(time.perf_counter())
        mask = env.engine.collision_free(q, mp, mq)
        t.append(time.perf_counter())
        idx = np.nonzero(mask)[0]
        plan = env.rollout_plan(P[idx], J[idx], nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                                close_steps=h["close_steps"], lift_check_every=h["lift_check_every"])
        t.append(time.perf_counter())
        res = env.rollout(plan)
        t.append(time.perf_counter())
        if it:
            rows.append(np.diff(t) * 1e3)
        labels = res["label"] if labels is None else labels
        assert np.array_equal(labels, res["label"])
        print(f"call {it}: {len(idx)} rollouts, main launch kernel {res.get('kernel_ms', float('nan')):.1f} ms, "
              f"escalation stages (ncon, rollouts, wall ms, kernel ms): "
              f"{[(c, n, round(w, 1), round(k, 1)) for c, n, w, k in stages]}", flush=True)
    m = np.median(np.array(rows), 0)
    for n, v in zip(["initial_state (host SE3, 32768)", "collision_free (upload, launch, download)",
                     f"rollout_plan ({len(idx)})", "env.rollout (with escalation)"], m):
        print(f"{n:48s} {v:8.2f} ms")
    print(f"{'total':48s} {m.sum():8.2f} ms  -> {32768 / m.sum() * 1e3:.0f} candidates/s")
    print(f"ncon_max {ncon}: {int(labels.sum())} stable of {len(labels)}, label crc32 {zlib.crc32(labels.tobytes()):08x}")


if __name__ == "__main__":
    main()
