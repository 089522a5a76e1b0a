"""Diagnostic: per-stage s_memtime breakdown of the wide (clutter) rollout kernel
on the Shadow pile (libmgs_gpu_wide_prof.so, -DMGS_WIDE -DMGS_PROFILE)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "mj-grasp-sim_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import mgs.core.engine as E  # noqa: E402

E.LIB_WIDE_PATH = E.LIB_WIDE_PATH.replace("libmgs_gpu_wide.so", "libmgs_gpu_wide_prof.so")
from make_clutter_scene import make_env  # noqa: E402
from mgs.sampler.antipodal import hand_candidates  # noqa: E402
from mgs.util.geo.transforms import SE3Pose  # noqa: E402
from stage_profile import NAMES, report  # noqa: E402

z = np.load(os.path.join(ROOT, "tests", "golden", "clutter_scene_shadow.npz"))
env = make_env("ShadowHand")
env.set_state(z["state"])
H, J = [], []
for k, o in enumerate(env.objects):
    h, j, _ = hand_candidates(o, 64, env.gripper, seed=k)
    H.append((env.get_obj_pose(o.name) @ SE3Pose.from_mat(h)).to_mat())
    J.append(j)
P = SE3Pose.from_mat(np.concatenate(H).astype(np.float32))
J = np.concatenate(J)
st = env.get_state()
mask = env.grasp_collision_mask(P, J)
idx = np.nonzero(mask)[0][:32]
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
plan = env.stable_plan(P[idx], J[idx], st, nstep_lift=steps, close_steps=steps)
eng = env.engine_for_state(st)
L = eng.lib
L.mgs_prof_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 64)()
L.mgs_prof_read(buf)
r = eng.rollout(plan)
L.mgs_prof_read(buf)
report(buf, r, len(idx), 2 * steps)
