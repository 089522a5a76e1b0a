"""Clutter piles of more than 64 dofs: two dofs per lane.

The reference draws piles of `num_objects_min`..`num_objects_max` objects with
repetition (mgs/obj/selector.py:124-130); with the Shadow hand (28 dofs) and
six per free object, 7 objects give nv 70 and 10 give nv 88 -- past the 64
lanes of a wave.  Those models run in a specialised code object of the wide
flavour built with -DMGS_DPL=2 (mgs_kernels.hip DofV: lane l owns dofs l and
l + 64; the dof reductions are the oracle's tree_dot over 128 leaves, i.e. the
tree over each half, then their sum).  The piles here are spread on the table
(mgs.core.shipped.spread_pile): parity does not need a settled pile.

CPU: the model, its packing (4-word dof masks), LDS fit, the object's flags,
the refusal past 128 dofs, and the oracle's short rollout.  GPU: collision
mask and a close + lift rollout bit-exact against the oracle for 7 and 10
objects.
"""
import os

import numpy as np
import pytest

from mgs.core.shipped import WIDE_PILE_OBJECTS as OBJS   # their objects are prebuilt by the build


def _init_torch():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass


def _in_bounds(p):
    return (np.abs(p[:, 0]) < 0.25) & (np.abs(p[:, 1]) < 0.25) & (p[:, 2] > 0) & (p[:, 2] < 1)


_ENVS = {}


def pile(n):
    if n not in _ENVS:
        from mgs.core.shipped import spread_pile
        _ENVS[n] = spread_pile("ShadowHand", OBJS[:n])
    return _ENVS[n]


def candidates(env, per_object=8):
    """hand candidates of every pile object, posed by its pose (gen_scene.py:59-66)"""
    from mgs.sampler.antipodal import hand_candidates
    from mgs.util.geo.transforms import SE3Pose
    H, J = [], []
    for k, o in enumerate(env.objects):
        h, j, _ = hand_candidates(o, per_object, env.gripper, seed=k)
        H.append((env.get_obj_pose(o.name) @ SE3Pose.from_mat(h)).to_mat())
        J.append(j)
    return SE3Pose.from_mat(np.concatenate(H).astype(np.float32)), np.concatenate(J)


@pytest.mark.parametrize("n", [7, 10])
def test_pile_model_over_64_dofs(n):
    """nv 28 + 6 n, dof masks of 4 words per body, the specialised object is
    the two-dofs-per-lane build of the wide flavour, the working set fits one
    CU's LDS"""
    from mgs.core import abi, special
    from mgs.core.engine import library_for, lds_bytes_for
    env = pile(n)
    st = env.get_state()
    cm = env.model_for(st)
    assert cm.nv == 28 + 6 * n and cm.nv > 64
    assert cm.nbody <= 64 and len(cm.jnt_type) <= 64
    mask = cm.body_dofmask()
    assert mask.shape == (cm.nbody, 4)
    # every dof's own body carries its bit, dofs past 64 included
    for d in range(cm.nv):
        b = int(cm.dof_bodyid[d])
        assert (int(mask.view(np.uint32)[b, d // 32]) >> (d % 32)) & 1
    nc, ne = env.ncon_max, env.rows_for(cm, env.ncon_max)
    assert lds_bytes_for(cm, nc, ne) <= 160 * 1024
    fields, _, _ = cm.pack(ncon_max=nc, nefc_max=ne)
    lib = library_for(cm.nv, int(fields["nefc_max"]))
    assert lib.mgs_rows_per_lane() == 4 and not lib.mgs_supports_nv(cm.nv)
    _, flags, _ = special.plan(lib, abi.make_desc(fields))
    assert "-DMGS_DPL=2" in flags and "-DMGS_WIDE" in flags


def test_pile_past_128_dofs_refused():
    env = pile(7)
    with pytest.raises(ValueError, match="at most 128 dofs"):
        env._check_kernel(130)


def test_pile_7_oracle_short_rollout():
    """CPU: the oracle's mask and a short close + lift on the 7-object pile
    (nv 70) are sane"""
    from oracle import oracle as O
    env = pile(7)
    st = env.get_state()
    poses, J = candidates(env)
    q, mp, mq = env._initial_qpos(poses, J, st)
    om = O.OracleModel(env.model_for(st), ncon_max=env.ncon_max, nefc_max=256)
    free = om.collision_free(q, mp, mq, predicate="partition_incl", nthreads=8) & _in_bounds(poses.pos)
    assert 2 <= free.sum() < len(free)
    idx = np.nonzero(free)[0][:2]
    r = om.rollout(env.stable_plan(poses[idx], J[idx], st, nstep_lift=40, close_steps=40), nthreads=2)
    assert r["stats"][:, 2].max() == 0
    assert np.isfinite(r["obj_qpos"]).all()


def _gpu_parity(n, steps, ncand):
    from oracle import oracle as O
    env = pile(n)
    st = env.get_state()
    poses, J = candidates(env)
    eng = env.engine_for_state(st)
    assert eng.specialized() and os.path.basename(eng.lib._name) == "libmgs_gpu_wide.so"
    mask = env.grasp_collision_mask(poses, J)
    q, mp, mq = env._initial_qpos(poses, J, st)
    om = O.OracleModel(env.model_for(st), ncon_max=env.ncon_max, nefc_max=eng.desc.nefc_max)
    ref = om.collision_free(q, mp, mq, predicate="partition_incl", nthreads=8) & _in_bounds(poses.pos)
    assert np.array_equal(mask, ref)
    idx = np.nonzero(mask)[0][:ncand]
    assert len(idx) >= 2
    plan = env.stable_plan(poses[idx], J[idx], st, nstep_lift=steps, close_steps=steps)
    rg, ro = eng.rollout(plan), om.rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(rg[k], ro[k]), k


@pytest.mark.gpu
def test_pile_7_objects_gpu_parity():
    """7-object Shadow pile (nv 70): collision mask and a 150 + 150 step close
    + lift, GPU == oracle bit for bit (verdict r4 item 7)"""
    _init_torch()
    _gpu_parity(7, 150, 4)


@pytest.mark.gpu
def test_pile_10_objects_gpu_parity():
    """10-object Shadow pile (nv 88, the reference's largest draws): 60 + 60
    steps, GPU == oracle bit for bit"""
    _init_torch()
    _gpu_parity(10, 60, 3)
