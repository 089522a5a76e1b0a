"""python -m mgs.cli.filter_to_stable gripper=<cfg> id=<k> [horizon=ref8000|h200]
(reference: mgs/cli/filter_to_stable.py:14-71): candidates.npz -> collision
mask -> stability rollout (enough_stable=1000) -> candidates_collision_free.npz
and stable_grasps.npz, every candidate of a stage evaluated at once on the GPU."""
import os

from mgs.cli._common import grasp_dir, horizon_kwargs, load_grasps, object_id, save_grasps
from mgs.cli._hydra import main
from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
from mgs.gripper.selector import get_gripper
from mgs.obj.selector import get_object


@main("filter_to_stable")
def run(cfg):
    oid = object_id(cfg)
    env = GravitylessObjectGrasping(get_gripper(cfg.gripper), get_object(oid))
    d = grasp_dir(cfg, oid, "MGS_INPUT_DIR")
    poses, joints = load_grasps(os.path.join(d, "candidates.npz"))
    mask = env.grasp_collision_mask(poses, joints)
    poses_cf, joints_cf = poses[mask], joints[mask]
    print(sum(mask))
    mm = env.grasp_stability_evaluation_from_joints(poses_cf, joints_cf, enough_stable=1000, **horizon_kwargs(cfg))
    print(sum(mm))
    save_grasps(os.path.join(d, "candidates_collision_free.npz"), poses_cf, joints_cf)
    save_grasps(os.path.join(d, "stable_grasps.npz"), poses_cf[mm], joints_cf[mm])


if __name__ == "__main__":
    run()
