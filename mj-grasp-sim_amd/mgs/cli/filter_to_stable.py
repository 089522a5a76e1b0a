"""python -m mgs.cli.filter_to_stable gripper=<cfg> id=<k> [horizon=ref8000|h200]
(reference: mgs/cli/filter_to_stable.py:14-71): candidates.npz -> collision
mask -> stability rollout (enough_stable=1000) -> candidates_collision_free.npz
and stable_grasps.npz, every candidate of a stage evaluated at once on the GPU.

Under a launcher with WORLD_SIZE > 1 (`torchrun --nproc-per-node N -m
mgs.cli.filter_to_stable ...`) the candidates are split over the ranks, one
GPU each (mgs.env.sharding); rank 0 writes the same files."""
import os

from mgs.cli import _common
from mgs.cli._common import grasp_dir, load_grasps, object_id, save_grasps
from mgs.cli._hydra import main
from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
from mgs.env.sharding import cli_device, filter_sharded, init_cli_group
from mgs.gripper.selector import get_gripper
from mgs.obj.selector import get_object


@main("filter_to_stable")
def run(cfg):
    rank, _ = init_cli_group()
    oid = object_id(cfg)
    env = GravitylessObjectGrasping(get_gripper(cfg.gripper), get_object(oid), device=cli_device())
    d = grasp_dir(cfg, oid, "MGS_INPUT_DIR")
    poses, joints = load_grasps(os.path.join(d, "candidates.npz"))
    mask, mm = filter_sharded(*_common.evaluators(env, cfg), poses, joints, enough_stable=1000)
    poses_cf, joints_cf = poses[mask], joints[mask]
    if rank == 0:
        print(sum(mask))
        print(sum(mm))
        save_grasps(os.path.join(d, "candidates_collision_free.npz"), poses_cf, joints_cf)
        save_grasps(os.path.join(d, "stable_grasps.npz"), poses_cf[mm], joints_cf[mm])


if __name__ == "__main__":
    run()
