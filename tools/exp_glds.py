"""Experiment: the wide (clutter) kernel with G rows in HBM (libmgs_gpu_wide.so)
vs in LDS (libmgs_gpu_wide_glds.so, -DMGS_G_LDS) on the Shadow pile rollouts
of config C5, same capacities; kernel time, overflow, label agreement."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "mj-grasp-sim_amd"), os.path.join(ROOT, "tests", "golden"), ROOT]
import torch  # noqa: E402
torch.cuda.init()
from make_clutter_scene import make_env  # noqa: E402
from mgs.core import engine as E  # noqa: E402
from mgs.sampler.antipodal import hand_candidates  # noqa: E402
from mgs.util.geo.transforms import SE3Pose  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 600
caps = [(40, 128), (48, 140)]
z = np.load(os.path.join(ROOT, "tests", "golden", "clutter_scene_shadow.npz"))
env = make_env("ShadowHand")
env.set_state(z["state"])
H, J = [], []
for k, o in enumerate(env.objects):
    h, j, _ = hand_candidates(o, 256, env.gripper, seed=k)
    H.append((env.get_obj_pose(o.name) @ SE3Pose.from_mat(h)).to_mat())
    J.append(j)
P = SE3Pose.from_mat(np.concatenate(H).astype(np.float32))
J = np.concatenate(J)
st = env.get_state()
mask = env.grasp_collision_mask(P, J)
idx = np.nonzero(mask)[0]
plan = env.stable_plan(P[idx], J[idx], st, nstep_lift=steps, close_steps=steps)
cm = env.model_for(st)
res = {}
for lib in ["libmgs_gpu_wide.so", "libmgs_gpu_wide_glds.so"]:
    os.environ["MGS_LIB_WIDE"] = lib
    for nc, ne in caps:
        eng = E.Engine(cm, device=0, ncon_max=nc, nefc_max=ne)
        eng.rollout(plan)
        r = eng.rollout(plan)
        res[(lib, nc, ne)] = r
        print(lib, nc, ne, "lds", eng.lds_bytes(), "kernel_ms %.1f" % r["kernel_ms"], "overflow",
              int((r["stats"][:, 2] != 0).sum()), "stable", int(r["label"].sum()), flush=True)
for nc, ne in caps:
    a, b = res[("libmgs_gpu_wide.so", nc, ne)], res[("libmgs_gpu_wide_glds.so", nc, ne)]
    ok = (a["stats"][:, 2] == 0) & (b["stats"][:, 2] == 0)
    print(nc, ne, "identical where no overflow:", all(np.array_equal(a[k][ok], b[k][ok]) for k in ("label", "obj_qpos")))
