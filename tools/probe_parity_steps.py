"""Probe (GPU): the first step at which the headline rollout leaves the oracle.
Short plans (the close phase cut to k steps) on the seed-0 candidates; per k
the candidates whose stats / object pose differ, with their contact counts."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mj-grasp-sim_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

torch.cuda.init()
from conftest import plan_for  # noqa: E402
from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping  # noqa: E402
from mgs.gripper.robotiq2f85 import GripperRobotiq2f85  # noqa: E402
from mgs.obj.selector import get_object  # noqa: E402
from mgs.sampler.antipodal import robotiq_candidates  # noqa: E402
from mgs.util.geo.transforms import SE3Pose  # noqa: E402
from oracle import oracle as O  # noqa: E402

env = GravitylessObjectGrasping(GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz")),
                                get_object("003_cracker_box"))
H, J, _ = robotiq_candidates(env.obj, 256, seed=0)
poses = SE3Pose.from_mat(H)
J = np.asarray(J, np.float64)
q, mp, mq, _ = env.initial_state(poses, J)
om = O.OracleModel(env.model, ncon_max=env.ncon_max, nefc_max=env.nefc_max)
free = env.engine.collision_free(q, mp, mq)
print("mask equal", np.array_equal(free, om.collision_free(q, mp, mq, nthreads=8)), "specialized",
      env.engine.specialized())
idx = np.nonzero(free)[0]
for eng_name, eng in (("main", env.engine), ("latency", env.latency_engine)):
    if eng is None:
        continue
    for k in (1, 2, 3, 5, 10, 30, 76, 200):
        plan = plan_for(env, poses[idx], J[idx])
        tot = 0
        ns = []
        for p, n in enumerate(plan.nsteps):
            take = max(0, min(n, k - tot))
            ns.append(take)
            tot += take
        keep = [i for i, n in enumerate(ns) if n > 0]
        plan.nsteps = [ns[i] for i in keep]
        plan.check_every = [plan.check_every[i] for i in keep]
        plan.check_at_end = [plan.check_at_end[i] for i in keep]
        plan.ctrl = [plan.ctrl[i] for i in keep]
        plan.phase_start = np.ascontiguousarray(plan.phase_start[:, keep])
        plan.phase_target = np.ascontiguousarray(plan.phase_target[:, keep])
        rg, ro = eng.rollout(plan), om.rollout(plan, nthreads=8)
        bad = np.nonzero((rg["stats"] != ro["stats"]).any(1) | (rg["obj_qpos"] != ro["obj_qpos"]).any(1)
                         | (rg["label"] != ro["label"]))[0]
        print(eng_name, "k", k, "differ", len(bad), "of", len(idx), bad[:6].tolist(), flush=True)
        for b in bad[:3]:
            print("   gpu stats", rg["stats"][b].tolist(), "oracle", ro["stats"][b].tolist(),
                  "dq", float(np.abs(rg["obj_qpos"][b] - ro["obj_qpos"][b]).max()))
        if len(bad):
            break
