"""Diagnostic: per-stage s_memtime breakdown of the clutter rollout on the
Shadow pile: the profile build (-DMGS_PROFILE) of the pile model's specialised
code object attached in place of the product one.
    python tools/stage_profile_clutter.py [steps] [--compile-only]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "mj-grasp-sim_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from mgs.core import special  # noqa: E402

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
eng = env.engine_for_state(st)
path = special.code_object(eng.lib, eng.desc, profile=True)
if "--compile-only" in sys.argv:
    print(path)
    sys.exit(0)
mask = env.grasp_collision_mask(P, J)
idx = np.nonzero(mask)[0][:32]
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
plan = env.stable_plan(P[idx], J[idx], st, nstep_lift=steps, close_steps=steps)
eng._ck(eng.lib.mgs_model_attach_special(eng._model, path.encode()), "mgs_model_attach_special")
L = eng.lib
L.mgs_model_prof_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 64)()
L.mgs_model_prof_read(eng._model, buf)
r = eng.rollout(plan)
eng._ck(L.mgs_model_prof_read(eng._model, buf), "mgs_model_prof_read")
report(buf, r, len(idx), 2 * steps)
