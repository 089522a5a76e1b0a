"""python -m mgs.cli.filter_stable_grasps gripper=<cfg> id=<k> [horizon=...]
(reference: mgs/cli/filter_stable_grasps.py:14-52):
candidates_collision_free.npz -> stable_grasps.npz (sharded over the ranks when
WORLD_SIZE > 1)."""
import os

from mgs.cli._common import grasp_dir, horizon_kwargs, load_grasps, object_id, save_grasps
from mgs.cli._hydra import main
from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
from mgs.env.sharding import cli_device, init_cli_group, stage_sharded
from mgs.gripper.selector import get_gripper
from mgs.obj.selector import get_object


@main("filter_stable_grasps")
def run(cfg):
    rank, _ = init_cli_group()
    oid = object_id(cfg)
    env = GravitylessObjectGrasping(get_gripper(cfg.gripper), get_object(oid), device=cli_device())
    d = grasp_dir(cfg, oid, "MGS_INPUT_DIR")
    poses, joints = load_grasps(os.path.join(d, "candidates_collision_free.npz"))
    kw = horizon_kwargs(cfg)
    mask = stage_sharded(lambda p, j: env.grasp_stability_evaluation_from_joints(p, j, **kw), poses, joints)
    if rank == 0:
        print(sum(mask))
        save_grasps(os.path.join(d, "stable_grasps.npz"), poses[mask], joints[mask])


if __name__ == "__main__":
    run()
