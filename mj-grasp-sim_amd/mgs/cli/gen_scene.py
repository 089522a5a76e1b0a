"""python -m mgs.cli.gen_scene gripper=<cfg> [object=subset_from_fast] [num_objects=5]
(reference: mgs/cli/gen_scene.py:15-212).

gen_stable_scene (:28-45): draw the objects (mgs.obj.selector.get_objects,
random subsets parked off the drop zone), park the gripper at (5, 5, 1), drop
the objects one by one and settle the pile (ClutterTableEnv.gen_clutter on the
GPU free-simulation entry point mgs_simulate), and reject an unstable pile
(is_stable).  `scene_batch=k` settles k candidate piles at once, one wave
each, and keeps the first stable one (k = 1 is the reference's behaviour).

filter_grasps (:48-159): every object's stable_grasps.npz from
$MGS_INPUT_DIR/<gripper>/<object id>/, posed by the settled object pose; the
clutter collision mask (at least 128 collision-free, else ValueError); then,
unless only_collision_free, a shuffle and the stable mask with
enough_stable = min(128, 32 * num_objects).  As in the reference the shuffle
permutes poses and joints but not the object indices (:113 compares instead of
assigning); `fix_shuffle=true` permutes them too.

main (:162-208): $MGS_OUTPUT_DIR/<gripper>/<hash>/scene.npz (this build's
pickle-free scene format, mgs.env.selector.save_scene) and one
<id>_<name>.npz {pose, joints} per object (plus <id>_<name>_collision.npz with
save_collision_grasps).  A failure prints its message and writes nothing.
"""
import os
import random
from copy import deepcopy

import numpy as np

from mgs.cli._hydra import main
from mgs.env.selector import get_env, get_env_from_dict, save_scene
from mgs.gripper.selector import get_gripper
from mgs.obj.selector import generate_unique_hash, get_objects
from mgs.util.geo.transforms import SE3Pose


def get_grasps(gripper_name, obj_id):
    g = np.load(os.path.join(os.getenv("MGS_INPUT_DIR"), gripper_name, obj_id, "stable_grasps.npz"))
    return g["pose"], g["joints"]


def gen_stable_scene(cfg, rng=None):
    rng = np.random.default_rng(rng)
    obj_list = get_objects(cfg.object, random.Random(int(rng.integers(1 << 62))))
    gripper = get_gripper(cfg.gripper, default_pose=SE3Pose(np.array([5.0, 5.0, 1.0]),
                                                             np.array([1.0, 0.0, 0.0, 0.0]), type="wxyz"))
    env = get_env(cfg.env, gripper=deepcopy(gripper), obj_list=deepcopy(obj_list))
    states = env.gen_clutter_states(int(cfg.get("scene_batch", 1)), rng,
                                    steps_each=int(cfg.get("steps_each", 900)),
                                    steps_final=int(cfg.get("steps_final", 9000)),
                                    ncon_max=cfg.get("settle_ncon"))
    gen_bad = np.asarray(getattr(env, "last_bad_scenes", np.zeros(len(states), bool)), bool)
    stable, _, _ = env.is_stable_states(states)
    stable = stable & ~gen_bad      # truncated / diverged while settling: never saved
    if not stable.any():
        raise ValueError("Scene unstable")
    env.set_state(states[int(np.argmax(stable))])
    return env.to_dict()


def filter_grasps(cfg, scene_def, rng=None):
    rng = np.random.default_rng(rng)
    env = get_env_from_dict(cfg.env, deepcopy(scene_def))
    all_grasps = []
    for obj_name, obj_id in zip(env.object_names, env.object_ids):
        poses, joints = get_grasps(cfg.gripper.name, obj_id)
        o2w = env.get_obj_pose(obj_name)
        all_grasps.append(((o2w @ SE3Pose.from_mat(deepcopy(poses))).to_mat(), joints, obj_name, obj_id))
    P, J, I, obj_map = [], [], [], []
    for idx, (p, j, obj_name, obj_id) in enumerate(all_grasps):
        if len(p) > 0:
            P.append(p)
            J.append(j)
            I.append(np.full(len(p), idx, dtype=np.int32))
            obj_map.append((obj_name, obj_id))
    if not P:
        raise ValueError("No collision free grasps")
    all_poses, all_joints, obj_indices = np.concatenate(P), np.concatenate(J), np.concatenate(I)
    mask = env.grasp_collision_mask(SE3Pose.from_mat(deepcopy(all_poses), type="wxyz"), deepcopy(all_joints))
    if mask.sum() < int(cfg.get("enough_collision_free", 128)):
        raise ValueError("Not enough collision free grasps!")
    cf_p, cf_j, cf_i = all_poses[mask], all_joints[mask], obj_indices[mask]
    col_p, col_j, col_i = all_poses[~mask], all_joints[~mask], obj_indices[~mask]
    if not cfg.only_collision_free:
        perm = rng.permutation(len(cf_p))
        cf_p, cf_j = cf_p[perm], cf_j[perm]
        if cfg.get("fix_shuffle", False):
            cf_i = cf_i[perm]
        enough = cfg.get("enough_stable")
        enough = min(128, int(cfg.num_objects) * 32) if enough is None else int(enough)
        kw = {}
        if cfg.get("lift_steps") is not None:
            kw = dict(nstep_lift=int(cfg.lift_steps), close_steps=int(cfg.lift_steps))
        stable = env.grasp_stable_mask(SE3Pose.from_mat(deepcopy(cf_p), type="wxyz"), deepcopy(cf_j),
                                       deepcopy(scene_def["env_state"]["state"]), enough_stable=enough, **kw)
        if stable.sum() < enough:
            raise ValueError("Not enough stable grasps!")
        rp, rj, ri = cf_p[stable], cf_j[stable], cf_i[stable]
    else:
        rp, rj, ri = cf_p, cf_j, cf_i
    result, neg_result = [], []
    for oi in np.unique(ri):
        m = ri == oi
        obj_name, obj_id = obj_map[oi]
        result.append({"object_id": obj_id, "object_name": obj_name, "pose": rp[m], "joints": rj[m]})
        if cfg.save_collision_grasps:
            cm = col_i == oi
            if cm.sum() > 0:
                neg_result.append({"object_id": obj_id, "object_name": obj_name, "pose": col_p[cm],
                                   "joints": col_j[cm]})
    return result, neg_result


@main("gen_scene")
def run(cfg):
    output_dir = os.getenv("MGS_OUTPUT_DIR")
    input_dir = os.getenv("MGS_INPUT_DIR")
    assert output_dir is not None, "No ouput_dir defined!"
    assert input_dir is not None, "No input_dir defined!"
    output_dir = os.path.join(output_dir, cfg.gripper.name, generate_unique_hash(16))
    rng = np.random.default_rng(cfg.get("seed"))
    try:
        scene_dict = gen_stable_scene(cfg, rng)
        valid, invalid = filter_grasps(cfg, scene_dict, rng)
        os.makedirs(output_dir, exist_ok=True)
        save_scene(os.path.join(output_dir, "scene.npz"), scene_dict)
        for g in valid:
            np.savez(os.path.join(output_dir, g["object_id"] + "_" + g["object_name"]),
                     pose=g["pose"], joints=g["joints"])
        for g in invalid:
            np.savez(os.path.join(output_dir, g["object_id"] + "_" + g["object_name"] + "_collision"),
                     pose=g["pose"], joints=g["joints"])
        return output_dir
    except Exception as e:
        print(e)
        return None


if __name__ == "__main__":
    run()
