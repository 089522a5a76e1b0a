"""python -m mgs.cli.filter_stable_grasps gripper=<cfg> id=<k> [horizon=...]
(reference: mgs/cli/filter_stable_grasps.py:14-52):
candidates_collision_free.npz -> stable_grasps.npz."""
import os

from mgs.cli._common import grasp_dir, horizon_kwargs, load_grasps, object_id, save_grasps
from mgs.cli._hydra import main
from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
from mgs.gripper.selector import get_gripper
from mgs.obj.selector import get_object


@main("filter_stable_grasps")
def run(cfg):
    oid = object_id(cfg)
    env = GravitylessObjectGrasping(get_gripper(cfg.gripper), get_object(oid))
    d = grasp_dir(cfg, oid, "MGS_INPUT_DIR")
    poses, joints = load_grasps(os.path.join(d, "candidates_collision_free.npz"))
    mask = env.grasp_stability_evaluation_from_joints(poses, joints, **horizon_kwargs(cfg))
    print(sum(mask))
    save_grasps(os.path.join(d, "stable_grasps.npz"), poses[mask], joints[mask])


if __name__ == "__main__":
    run()
