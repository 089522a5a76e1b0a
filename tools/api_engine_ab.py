"""Interleaved A/B of the drop-in API's rollout call (the 8192-candidate
filter_to_stable call, mgs/cli/filter_to_stable.py:39-50): which engine and
rotation slice finish the call's 1173 rollouts first, and the host stages.
GPU box; prints one line per variant (median of 5 rounds after 1 warm-up).

    python tools/api_engine_ab.py"""
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
    h = HORIZONS["h200"]
    H, J, _ = robotiq_candidates(env.obj, 8192, seed=0)
    poses = SE3Pose.from_mat(H)
    variants = [("latency engine, yield 32", 1.25, 32), ("latency engine, yield 16", 1.25, 16),
                ("latency engine, yield 64", 1.25, 64), ("main engine, yield 32", 0.0, 32),
                ("main engine, no rotation", 0.0, 0)]
    times = {v[0]: [] for v in variants}
    host = []
    ref = None
    for it in range(6):
        t0 = time.perf_counter()
        q, mp, mq, _ = env.initial_state(poses, J)
        t1 = time.perf_counter()
        mask = env.engine.collision_free(q, mp, mq)
        t2 = time.perf_counter()
        idx = np.nonzero(mask)[0]
        plan = env.rollout_plan(poses[idx], J[idx], nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                                close_steps=h["close_steps"], lift_check_every=h["lift_check_every"])
        t3 = time.perf_counter()
        if it:
            host.append([(t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3])
        for name, rounds, ye in variants:
            env.LATENCY_ROUNDS = rounds
            t = time.perf_counter()
            res = env.rollout(plan, yield_every=ye)
            dt = (time.perf_counter() - t) * 1e3
            if ref is None:
                ref = res["label"].copy()
            assert np.array_equal(res["label"], ref), name
            if it:
                times[name].append(dt)
        print(f"round {it} done", flush=True)
    # the mask call's parts: pageable copies + launch + sync vs the launch alone
    q, mp, mq, _ = env.initial_state(poses, J)
    dq, dmp, dmq = (torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (q, mp, mq))
    dout = torch.zeros(len(q), dtype=torch.uint8, device="cuda")
    tm, td = [], []
    for _ in range(10):
        t = time.perf_counter()
        env.engine.collision_free(q, mp, mq)
        tm.append((time.perf_counter() - t) * 1e3)
        torch.cuda.synchronize()
        t = time.perf_counter()
        env.engine.collision_free_device(len(q), dq.data_ptr(), dmp.data_ptr(), dmq.data_ptr(), dout.data_ptr(),
                                         stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        td.append((time.perf_counter() - t) * 1e3)
    print(f"mask host call {np.median(tm):.2f} ms, device-resident launch + sync {np.median(td):.2f} ms")
    m = np.median(np.array(host), 0)
    print(f"host poses {m[0]:.2f} ms, mask {m[1]:.2f} ms, plan {m[2]:.2f} ms ({len(idx)} rollouts)")
    for name, _, _ in variants:
        r = np.median(times[name])
        print(f"{name:28s} rollout {r:7.2f} ms  -> call {8192 / (m.sum() + r) * 1e3:8.0f} candidates/s")
    print("labels identical across variants")


if __name__ == "__main__":
    main()
