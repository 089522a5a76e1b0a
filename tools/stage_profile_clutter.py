"""Diagnostic: per-stage s_memtime breakdown of the clutter rollout on the
Shadow pile: the profile build (-DMGS_PROFILE) of the pile model's specialised
code object attached in place of the product one.
    python tools/stage_profile_clutter.py [steps] [candidates per object] [max rollouts] [--compile-only]"""
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

ARGS = [a for a in sys.argv[1:] if not a.startswith("--")]
NPER = int(ARGS[1]) if len(ARGS) > 1 else 64
NMAX = int(ARGS[2]) if len(ARGS) > 2 else 32
z = np.load(os.path.join(ROOT, "tests", "golden", "clutter_scene_shadow.npz"))
env = make_env("ShadowHand")
env.set_state(z["state"])
H, J = [], []
for k, o in enumerate(env.objects):
    h, j, _ = hand_candidates(o, NPER, env.gripper, seed=k)
    H.append((env.get_obj_pose(o.name) @ SE3Pose.from_mat(h)).to_mat())
    J.append(j)
P = SE3Pose.from_mat(np.concatenate(H).astype(np.float32))
J = np.concatenate(J)
st = env.get_state()
if "--compile-only" in sys.argv:
    # the profile object of the engine engine_for_state(st) creates, built here
    # (no device needed): same model, capacity and rows as Engine() sizes them
    from mgs.core import abi
    from mgs.core.engine import default_rows, library_for
    cm = env.model_for(st)
    ne = env.rows_for(cm, env.ncon_max) or default_rows(cm, int(cm.pack(ncon_max=env.ncon_max)[0]["nefc_max"]))
    fields, _, _ = cm.pack(ncon_max=env.ncon_max, nefc_max=ne)
    print(special.code_object(library_for(cm.nv, int(fields["nefc_max"])), abi.make_desc(fields), profile=True))
    sys.exit(0)
eng = env.engine_for_state(st)
path = special.code_object(eng.lib, eng.desc, profile=True)
mask = env.grasp_collision_mask(P, J)
idx = np.nonzero(mask)[0][:NMAX]
steps = int(ARGS[0]) if ARGS else 300
plan = env.stable_plan(P[idx], J[idx], st, nstep_lift=steps, close_steps=steps)
eng._ck(eng.lib.mgs_model_attach_special(eng._model, path.encode()), "mgs_model_attach_special")
L = eng.lib
L.mgs_model_prof_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 64)()
L.mgs_model_prof_read(eng._model, buf)
r = eng.rollout(plan)
eng._ck(L.mgs_model_prof_read(eng._model, buf), "mgs_model_prof_read")
report(buf, r, len(idx), 2 * steps)
