"""Probe (GPU): the headline h200 parity block (tests/test_gpu_parity.py
test_rollout_parity_h200, Newton) on the main engine with each listed A/B
code object of mgs/_lib/ab (MGS_SPECIAL_OBJECT; tools/ab_build.py --ghbm),
then on the cached object.  python3 tools/probe_ab_parity.py name [name ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mj-grasp-sim_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

torch.cuda.init()
from conftest import plan_for  # noqa: E402
from mgs.core.engine import Engine  # noqa: E402
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
idx = np.nonzero(om.collision_free(q, mp, mq, nthreads=8))[0]
plan = plan_for(env, poses[idx], J[idx])
ro = om.rollout(plan, nthreads=8)
lib = os.path.join(ROOT, "mj-grasp-sim_amd", "mgs", "_lib", "ab")
for name in sys.argv[1:] + ["(cached)"]:
    if name == "(cached)":
        os.environ.pop("MGS_SPECIAL_OBJECT", None)
    else:
        os.environ["MGS_SPECIAL_OBJECT"] = os.path.join(lib, name + ".hsaco")
    eng = Engine(env.model, ncon_max=env.ncon_max, nefc_max=env.nefc_max, g_rows_hbm=True)
    rg = eng.rollout(plan)
    bad = np.nonzero((rg["stats"] != ro["stats"]).any(1) | (rg["obj_qpos"] != ro["obj_qpos"]).any(1)
                     | (rg["label"] != ro["label"]))[0]
    print(name, "g_rows_hbm", int(eng.desc.g_rows_hbm), "specialized", eng.specialized(), "differ", len(bad), "of",
          len(idx), "labels differ", int((rg["label"] != ro["label"]).sum()), bad[:8].tolist(), flush=True)
    eng.close()
