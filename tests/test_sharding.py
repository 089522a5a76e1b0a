"""Multi-process path on CPU (gloo, world size 2): the batch split + gather of
mgs.env.sharding gives exactly the single-process result.  The per-rank
compute here is the oracle (CPU); on GPUs each rank runs the HIP engine."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_evaluate(env):
    """per-rank evaluator for mgs.env.sharding.evaluate_sharded on the CPU: the
    oracle in place of the GPU engine (same signature as env.evaluate)"""
    from oracle import oracle as O
    from conftest import plan_for
    om = O.OracleModel(env.model)

    def evaluate(poses, joints):
        q, mp, mq, _ = env.initial_state(poses, joints)
        mask = om.collision_free(q, mp, mq)
        stable = np.zeros(len(poses), bool)
        idx = np.nonzero(mask)[0]
        if len(idx):
            stable[idx] = om.rollout(plan_for(env, poses[idx], joints[idx]))["label"]
        return mask, stable
    return evaluate


def _worker(rank, world, port, outq):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "mj-grasp-sim_amd"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.env.sharding import evaluate_sharded
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.obj.selector import get_object
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose
    dist.init_process_group("gloo", rank=rank, world_size=world)
    env = GravitylessObjectGrasping(GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz")),
                                    get_object("003_cracker_box"))
    H, J, _ = robotiq_candidates(env.obj, 96, seed=3)
    poses = SE3Pose.from_mat(H)
    # the product entry point: shard bounds, per-rank evaluation, gather, the
    # global enough_stable prefix
    mask, stable = evaluate_sharded(env, poses, J, enough_stable=3, evaluate=_oracle_evaluate(env))
    if rank == 0:
        outq.put({"mask": mask.tolist(), "stable": stable.tolist()})
    dist.destroy_process_group()


def _oracle_evaluators(env, cfg):
    """mgs.cli._common.evaluators with the oracle in place of the GPU engine"""
    from oracle import oracle as O
    from mgs.cli._common import horizon_kwargs
    om = O.OracleModel(env.model, ncon_max=env.ncon_max)
    kw = horizon_kwargs(cfg)

    def mask(p, j):
        q, mp, mq, _ = env.initial_state(p, j)
        return om.collision_free(q, mp, mq)

    def stable(p, j):
        return om.rollout(env.rollout_plan(p, j, **kw))["label"]
    return mask, stable


def _cli_worker(rank, world, port, indir, argv):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "mj-grasp-sim_amd"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world), MGS_INPUT_DIR=indir)
    from mgs.cli import _common, filter_to_stable
    _common.evaluators = _oracle_evaluators
    filter_to_stable.run(argv)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


def test_filter_to_stable_cli_two_ranks_writes_single_rank_files(tmp_path):
    """`torchrun --nproc-per-node 2 -m mgs.cli.filter_to_stable` (WORLD_SIZE 2,
    gloo gather) writes the files of the one-process run"""
    import shutil
    import torch.multiprocessing as mp
    from mgs.cli import gen_grasp_candidates
    src = tmp_path / "cand"
    os.environ["MGS_OUTPUT_DIR"] = str(src)
    try:
        gen_grasp_candidates.run(["id=0", "num_grasps=40", "sampler=host", "seed=5"])
    finally:
        del os.environ["MGS_OUTPUT_DIR"]
    sub = os.path.join("Robotiq2f85Gripper", "003_cracker_box")
    argv = ["id=0", "horizon=h200"]
    ctx = mp.get_context("spawn")
    outs = {}
    for world in (1, 2):
        d = tmp_path / f"w{world}"
        shutil.copytree(src, d)
        port = _free_port()
        procs = [ctx.Process(target=_cli_worker, args=(r, world, port, str(d), argv)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=300)
            assert p.exitcode == 0
        outs[world] = {f: np.load(d / sub / f) for f in ("candidates_collision_free.npz", "stable_grasps.npz")}
    for f in outs[1]:
        for k in ("pose", "joints"):
            assert np.array_equal(outs[1][f][k], outs[2][f][k]), (f, k)
    assert len(outs[1]["candidates_collision_free.npz"]["pose"]) > 0


def test_shard_bounds_cover():
    from mgs.env.sharding import shard_bounds
    for n in [0, 1, 7, 8192, 8193]:
        for w in [1, 2, 3, 8]:
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1


def test_two_rank_gloo_equals_single_process(env):
    import torch.multiprocessing as mp
    from conftest import plan_for
    from mgs.env.gravityless_object_grasping import apply_enough_stable
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    H, J, _ = robotiq_candidates(env.obj, 96, seed=3)
    poses = SE3Pose.from_mat(H)
    om = O.OracleModel(env.model)
    qq, mpos, mq, _ = env.initial_state(poses, J)
    mask = om.collision_free(qq, mpos, mq)
    stable = np.zeros(len(poses), bool)
    idx = np.nonzero(mask)[0]
    stable[idx] = om.rollout(plan_for(env, poses[idx], J[idx]))["label"]
    assert got["mask"] == mask.tolist()
    assert got["stable"] == apply_enough_stable(stable, 3).tolist()
