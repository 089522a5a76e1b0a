"""python -m mgs.cli.gen_grasps gripper=<cfg> id=<k> num_grasps=<n> [horizon=...]

The whole grasp-set pipeline in one process (the north star's gen_grasps):
gen_grasp_candidates (antipodal) -> filter_to_stable (collision mask + close /
lift / shake rollout on the GPU, enough_stable) -> the reference's three files
candidates.npz, candidates_collision_free.npz, stable_grasps.npz under
$MGS_OUTPUT_DIR/<gripper>/<object>/, plus timing on stdout."""
import os
import time

import numpy as np

from mgs.cli import _common
from mgs.cli._common import grasp_dir, object_id, save_grasps
from mgs.cli._hydra import main
from mgs.cli.gen_grasp_candidates import candidates
from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
from mgs.env.sharding import broadcast_from_rank0, cli_device, filter_sharded, init_cli_group
from mgs.gripper.selector import get_gripper
from mgs.obj.selector import get_object
from mgs.util.geo.transforms import SE3Pose


@main("gen_grasps")
def run(cfg):
    rank, world = init_cli_group()
    oid = object_id(cfg)
    gripper = get_gripper(cfg.gripper)
    obj = get_object(oid)
    out = grasp_dir(cfg, oid, "MGS_OUTPUT_DIR")
    t0 = time.perf_counter()
    HJ = None
    if rank == 0:
        # candidates are sampled once (rank 0's GPU) and the evaluation is
        # sharded over the ranks (mgs.env.sharding) when WORLD_SIZE > 1
        os.makedirs(out, exist_ok=True)
        HJ = candidates(gripper, obj, int(cfg.get("num_grasps", 8192)), int(cfg.get("seed", 0)),
                        cfg.get("sampler", "device"), gripper_name=cfg.gripper.name)
        np.savez(os.path.join(out, "candidates.npz"), pose=HJ[0], joints=HJ[1])
    H, J = broadcast_from_rank0(HJ)
    t1 = time.perf_counter()
    env = GravitylessObjectGrasping(gripper, obj, device=cli_device())
    poses = SE3Pose.from_mat(H, type="wxyz")
    es = cfg.get("enough_stable", 1000)
    mask, mm = filter_sharded(*_common.evaluators(env, cfg), poses, J, enough_stable=es)
    pc, jc = poses[mask], J[mask]
    t2 = time.perf_counter()
    if rank != 0:
        return
    save_grasps(os.path.join(out, "candidates_collision_free.npz"), pc, jc)
    save_grasps(os.path.join(out, "stable_grasps.npz"), pc[mm], jc[mm])
    print(f"{len(H)} candidates, {int(mask.sum())} collision-free, {int(mm.sum())} stable; "
          f"sampling {t1 - t0:.2f} s, evaluation {t2 - t1:.2f} s on {world} rank(s) -> {out}")


if __name__ == "__main__":
    run()
