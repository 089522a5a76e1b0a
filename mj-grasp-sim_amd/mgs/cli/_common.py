"""Shared CLI plumbing: object id from fast_eta_objects.txt, the per-(gripper,
object) directory under MGS_INPUT_DIR / MGS_OUTPUT_DIR, and the grasp-set
npz format (`pose` float32 (N,4,4) contact frames from SE3Pose.to_mat,
`joints` unchanged; reference filter_to_stable.py:32-68)."""
import os

import numpy as np

from mgs.util.const import ASSET_PATH


def object_id(cfg) -> str:
    with open(os.path.join(ASSET_PATH, "mj-objects", "fast_eta_objects.txt")) as f:
        ids = f.read().splitlines()
    return ids[int(cfg.id)]


def grasp_dir(cfg, oid, env_var) -> str:
    base = os.getenv(env_var) or "."
    return os.path.abspath(os.path.join(base, cfg.gripper.name, oid))


def load_grasps(path):
    from mgs.util.geo.transforms import SE3Pose
    g = np.load(path)
    return SE3Pose.from_mat(g["pose"], type="wxyz"), g["joints"]


def save_grasps(path, poses, joints):
    np.savez(path, **{"pose": poses.to_mat(), "joints": joints})


def evaluators(env, cfg):
    """(collision_mask, stable_mask) callables on (poses, joints) of a
    GravitylessObjectGrasping env for this configuration's horizon -- the two
    stages the CLIs shard over ranks (mgs.env.sharding)."""
    kw = horizon_kwargs(cfg)
    return env.grasp_collision_mask, lambda p, j: env.grasp_stability_evaluation_from_joints(p, j, **kw)


def horizon_kwargs(cfg):
    """stability keyword arguments of a named horizon (ref8000 = the reference's)."""
    from mgs.env.gravityless_object_grasping import HORIZONS
    h = HORIZONS[cfg.get("horizon", "ref8000")]
    return dict(nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"], close_steps=h["close_steps"],
                lift_check_every=h["lift_check_every"])
