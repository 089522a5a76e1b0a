"""python -m mgs.cli.eval_grasps gripper=<cfg> id=<k>
(reference: mgs/cli/eval_grasps.py:13-82).

For scene directory number `id` (sorted) under $MGS_INPUT_DIR/<gripper>/:
load scene.npz (this build's pickle-free scene format, mgs.env.selector.
save_scene) and inference_grasps.npz (contact-frame poses, joints), map the
poses to base frames with the inverse base-to-contact transform as the
reference does (:17-20), run the clutter collision mask and stable mask on the
GPU, and write grasp_evaluation.json {success_rate, num_objects, scene_id}."""
import json
import os

import numpy as np

from mgs.cli._hydra import main
from mgs.env.selector import get_env_from_dict, load_scene
from mgs.env.sharding import cli_device, filter_sharded, init_cli_group
from mgs.util.geo.transforms import SE3Pose


def eval_grasps(cfg, scene_def, grasps, **stable_kw):
    """collision mask, then the stable mask of the collision-free grasps
    (reference :20-36), split over the launch's ranks when WORLD_SIZE > 1"""
    env = get_env_from_dict(cfg.env, scene_def, device=cli_device())
    b2c = env.gripper.base_to_contact_transform().inverse().to_mat()
    pose, joints = grasps
    pose = np.einsum("nij,jk->nik", pose, b2c)
    state = scene_def["env_state"]["state"]
    mask, stable = filter_sharded(env.grasp_collision_mask,
                                  lambda p, j: env.grasp_stable_mask(p, j, state, **stable_kw),
                                  SE3Pose.from_mat(pose, type="wxyz"), joints)
    if mask.sum() == 0:
        return 0.0, {"num_objects": len(env.object_names)}
    return float(stable.sum()) / float(len(pose)), {"num_objects": len(env.object_names)}


@main("eval_grasps")
def run(cfg):
    rank, _ = init_cli_group()
    input_dir = os.getenv("MGS_INPUT_DIR")
    assert input_dir is not None, "No input_dir defined!"
    root = os.path.join(input_dir, cfg.gripper.name)
    scenes = sorted(os.listdir(root))
    scene = scenes[int(cfg.id)]
    d = os.path.join(root, scene)
    scene_def = load_scene(os.path.join(d, "scene.npz"))
    g = np.load(os.path.join(d, "inference_grasps.npz"))
    kw = {}
    if cfg.get("lift_steps") is not None:
        kw = dict(nstep_lift=int(cfg.lift_steps), close_steps=int(cfg.lift_steps))
    rate, aux = eval_grasps(cfg, scene_def, (g["pose"], g["joints"]), **kw)
    if rank != 0:
        return
    res = {"success_rate": float(rate), "num_objects": aux["num_objects"], "scene_id": scene}
    with open(os.path.join(d, "grasp_evaluation.json"), "w") as f:
        json.dump(res, f, indent=2)
    print(f"Evaluation complete: {rate:.2%} success rate")


if __name__ == "__main__":
    run()
