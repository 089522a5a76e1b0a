"""python -m mgs.cli.filter_collision_free_candidates gripper=<cfg> id=<k>
(reference: mgs/cli/filter_collision_free_candidates.py): candidates.npz ->
candidates_collision_free.npz (sharded over the ranks when WORLD_SIZE > 1)."""
import os

from mgs.cli._common import grasp_dir, load_grasps, object_id, save_grasps
from mgs.cli._hydra import main
from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
from mgs.env.sharding import cli_device, init_cli_group, stage_sharded
from mgs.gripper.selector import get_gripper
from mgs.obj.selector import get_object


@main("filter_collision_free_candidates")
def run(cfg):
    rank, _ = init_cli_group()
    oid = object_id(cfg)
    env = GravitylessObjectGrasping(get_gripper(cfg.gripper), get_object(oid), device=cli_device())
    d = grasp_dir(cfg, oid, "MGS_INPUT_DIR")
    poses, joints = load_grasps(os.path.join(d, "candidates.npz"))
    mask = stage_sharded(env.grasp_collision_mask, poses, joints)
    if rank == 0:
        print(sum(mask))
        save_grasps(os.path.join(d, "candidates_collision_free.npz"), poses[mask], joints[mask])


if __name__ == "__main__":
    run()
