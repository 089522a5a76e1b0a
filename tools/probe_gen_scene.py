"""Probe (GPU): the gen_scene CLI test's pipeline with its intermediate
counts -- the settled scene's object poses, the collision-free and stable
grasps and the stable mask's fail steps (tests/test_scene_gen.py::
test_gen_scene_cli)."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mj-grasp-sim_amd")]
import torch  # noqa: E402

torch.cuda.init()
from mgs.cli import gen_scene  # noqa: E402
from mgs.cli._hydra import compose  # noqa: E402
from mgs.env.selector import get_env_from_dict  # noqa: E402
from mgs.obj.selector import get_object  # noqa: E402
from mgs.sampler.antipodal import robotiq_candidates  # noqa: E402
from mgs.util.const import ASSET_PATH  # noqa: E402
from mgs.util.geo.transforms import SE3Pose  # noqa: E402

tmp = tempfile.mkdtemp()
fast = open(os.path.join(ASSET_PATH, "mj-objects", "fast_eta_objects.txt")).read().splitlines()
for k, oid in enumerate(fast):
    h, j, _ = robotiq_candidates(get_object(oid), 256, seed=k)
    d = os.path.join(tmp, "in", "Robotiq2f85Gripper", oid)
    os.makedirs(d)
    np.savez(os.path.join(d, "stable_grasps.npz"), pose=np.asarray(h, np.float32), joints=j)
os.environ["MGS_INPUT_DIR"] = os.path.join(tmp, "in")
for seed in (3, 4, 5):
    cfg = compose("gen_scene", ["gripper=robotiq_2f_85", f"seed={seed}", "num_objects=4", "scene_batch=4",
                                "steps_each=300", "steps_final=2000", "lift_steps=300", "enough_collision_free=4",
                                "enough_stable=1"])
    try:
        sd = gen_scene.gen_stable_scene(cfg, rng=seed)
    except ValueError as e:
        print(seed, "scene:", e)
        continue
    env = get_env_from_dict(cfg.env, sd)
    for n in env.object_names:
        print(seed, n, np.round(env.get_obj_pose(n).pos, 3).tolist())
    P, J = [], []
    for n, oid in zip(env.object_names, env.object_ids):
        p, j = gen_scene.get_grasps(cfg.gripper.name, oid)
        P.append((env.get_obj_pose(n) @ SE3Pose.from_mat(p)).to_mat())
        J.append(j)
    P, J = np.concatenate(P), np.concatenate(J)
    mask = env.grasp_collision_mask(SE3Pose.from_mat(P), J)
    idx = np.nonzero(mask)[0]
    res = env.grasp_stable_mask(SE3Pose.from_mat(P[idx]), J[idx], sd["env_state"]["state"], nstep_lift=300,
                                close_steps=300, return_details=True)
    fs = res["fail_step"]
    print(seed, "collision-free", len(idx), "stable", int(res["label"].sum()), "fail steps",
          np.unique(fs, return_counts=True), "max ncon", int(res["stats"][:, 0].max()) if len(idx) else 0,
          flush=True)
