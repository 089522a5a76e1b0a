"""HIP engine vs the oracle, through the C-ABI (libmgs_gpu.so), on an MI355X.

Bar: bit-exact.  The kernels and the oracle follow one arithmetic contract
(-ffp-contract=off, identical operation order, pairwise tree reductions that
mirror the wave's DPP tree, IEEE sqrt/div, polynomial sincos), so labels,
fail steps, final object poses and solver statistics must be identical, not
merely close.  At the full 8192-candidate size the checks are size-independent
properties (permutation invariance, run-to-run determinism, sub-batch
consistency) tied back to the oracle on a slice."""
import copy

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# torch (used here only to hold device buffers for the device-pointer entry
# points) bundles its own HIP runtime; it must initialise before
# libmgs_gpu.so pulls in /opt/rocm's, or torch finds no device.
try:
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
except Exception:  # pragma: no cover - CPU containers
    pass


@pytest.fixture(scope="module")
def eng(env):
    return env.engine


def _variant(env, **opts):
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    e2 = copy.copy(env)
    e2.model = copy.copy(env.model)
    e2.model.options = dict(env.model.options, **opts)
    e2._engine = None
    e2._sim = type(env._sim)(e2)
    return e2


def _assert_same(rg, ro, what=""):
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(rg[k], ro[k]), f"{what}: {k} differs"


def test_arith_probe_exact():
    from mgs.core import engine as E
    from oracle import oracle as O
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(-20, 20, 20000), rng.uniform(-1e-3, 1e-3, 1000), [0.0, np.pi, -np.pi / 2]])
    y = rng.uniform(0.1, 10, len(x))
    g = E.arith_probe(x, y)
    s, c = O.sincos(x)
    assert np.array_equal(g[:, 0], np.sqrt(np.abs(x)))
    assert np.array_equal(g[:, 1], x / y)
    assert np.array_equal(g[:, 2], s) and np.array_equal(g[:, 3], c)


def test_tree_probe_exact():
    from mgs.core import engine as E
    from oracle import oracle as O
    rng = np.random.default_rng(2)
    for n in [1, 2, 3, 5, 8, 9, 16, 17, 20, 31, 32, 33, 50, 64]:
        a, c = rng.standard_normal((16, 64)), rng.standard_normal((16, 64))
        dev = E.tree_probe(a, c, n)
        ref = np.array([O.tree_dot(a[i], c[i], n) for i in range(16)])
        assert np.array_equal(dev, ref), n


@pytest.mark.parametrize("predicate", ["any", "partition"])
def test_collision_mask_parity(env, eng, candidates, oracle_model, predicate):
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    assert np.array_equal(eng.collision_free(q, mp, mq, predicate=predicate),
                          oracle_model.collision_free(q, mp, mq, predicate=predicate, nthreads=8))


def test_collision_mask_api(env, candidates, oracle_model):
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    assert np.array_equal(env.grasp_collision_mask(poses, J), oracle_model.collision_free(q, mp, mq, nthreads=8))


@pytest.mark.parametrize("solver", ["Newton", "PGS"])
def test_rollout_parity_h200(env, candidates, solver):
    from conftest import plan_for
    from oracle import oracle as O
    e2 = _variant(env, solver=solver)
    om = O.OracleModel(e2.model, ncon_max=e2.ncon_max, nefc_max=e2.nefc_max)
    poses, J = candidates
    q, mp, mq, _ = e2.initial_state(poses, J)
    idx = np.nonzero(om.collision_free(q, mp, mq, nthreads=8))[0]
    plan = plan_for(e2, poses[idx], J[idx])
    _assert_same(e2.engine.rollout(plan), om.rollout(plan, nthreads=8), solver)


def test_rollout_parity_reference_horizon(env, eng, candidates, oracle_model):
    """The reference's own 8000-step schedule (close 3000, lift 3000 checked
    every 100, shake 500/500/1000) on a few candidates."""
    from conftest import plan_for
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    idx = np.nonzero(oracle_model.collision_free(q, mp, mq, nthreads=8))[0][:3]
    plan = plan_for(env, poses[idx], J[idx], horizon="ref8000")
    _assert_same(eng.rollout(plan), oracle_model.rollout(plan, nthreads=8), "ref8000")


def test_rollout_parity_unfiltered_with_overflow(env, candidates):
    """Colliding candidates too (deep initial penetration, many contacts) with a
    small contact cap: overflow handling must match as well."""
    from conftest import plan_for
    from mgs.core.engine import Engine
    from oracle import oracle as O
    poses, J = candidates
    plan = plan_for(env, poses[:48], J[:48])
    e = Engine(env.model, ncon_max=6)
    om = O.OracleModel(env.model, ncon_max=6)
    rg, ro = e.rollout(plan), om.rollout(plan, nthreads=8)
    _assert_same(rg, ro, "ncon_max=6")
    assert (rg["stats"][:, 2] != 0).any()


def test_stability_api_and_enough_stable(env, candidates, oracle_model):
    from conftest import plan_for
    from mgs.env.gravityless_object_grasping import HORIZONS, apply_enough_stable
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    idx = np.nonzero(oracle_model.collision_free(q, mp, mq, nthreads=8))[0][:16]
    h = HORIZONS["h200"]
    lab = env.grasp_stability_evaluation_from_joints(poses[idx], J[idx], nstep_lift=h["nstep_lift"],
                                                     shake_steps=h["shake_steps"], close_steps=h["close_steps"],
                                                     lift_check_every=h["lift_check_every"], enough_stable=2)
    ro = oracle_model.rollout(plan_for(env, poses[idx], J[idx]), nthreads=8)
    assert np.array_equal(lab, apply_enough_stable(ro["label"], 2))


def test_empty_and_single(env, eng, candidates):
    from conftest import plan_for
    from mgs.util.geo.transforms import SE3Pose
    poses, J = candidates
    empty = SE3Pose(np.zeros((0, 3), np.float32), np.zeros((0, 4), np.float32), "wxyz")
    assert env.grasp_collision_mask(empty, np.zeros((0, 8))).shape == (0,)
    assert env.grasp_stability_evaluation_from_joints(empty, np.zeros((0, 8))).shape == (0,)
    r1 = eng.rollout(plan_for(env, poses[:1], J[:1]))
    assert r1["label"].shape == (1,)


def test_device_entry_with_active_mask(env, eng, candidates, oracle_model):
    """mgs_collision_free_device + mgs_rollout_device(active) (the bench path)
    equal the host entry points; masked candidates are reported unevaluated."""
    import torch
    from conftest import plan_for
    from mgs.core import abi
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    plan = plan_for(env, poses, J)
    sched = abi.make_schedule(plan.nsteps, plan.check_every, plan.check_at_end, plan.ctrl, plan.obj_qposadr,
                                  check_offset=getattr(plan, "check_offset", None))
    n = len(q)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
    dq, dmp, dmq, dps, dpt = t(q), t(mp), t(mq), t(plan.phase_start), t(plan.phase_target)
    free = torch.zeros(n, dtype=torch.uint8, device=dev)
    lab = torch.zeros(n, dtype=torch.uint8, device=dev)
    fail = torch.zeros(n, dtype=torch.int32, device=dev)
    objq = torch.zeros((n, 7), dtype=torch.float64, device=dev)
    st = torch.zeros((n, abi.MGS["MGS_NSTATS"]), dtype=torch.int32, device=dev)
    eng.collision_free_device(n, dq.data_ptr(), dmp.data_ptr(), dmq.data_ptr(), free.data_ptr())
    eng.rollout_device(sched, n, dq.data_ptr(), dmq.data_ptr(), dps.data_ptr(), dpt.data_ptr(), lab.data_ptr(),
                       fail.data_ptr(), objq.data_ptr(), st.data_ptr(), d_active=free.data_ptr())
    torch.cuda.synchronize()
    mask = free.cpu().numpy().astype(bool)
    assert np.array_equal(mask, oracle_model.collision_free(q, mp, mq, nthreads=8))
    idx = np.nonzero(mask)[0]
    ro = oracle_model.rollout(plan_for(env, poses[idx], J[idx]), nthreads=8)
    assert np.array_equal(lab.cpu().numpy().astype(bool)[idx], ro["label"])
    assert np.array_equal(fail.cpu().numpy()[idx], ro["fail_step"])
    assert np.array_equal(objq.cpu().numpy()[idx], ro["obj_qpos"])
    rej = np.nonzero(~mask)[0]
    assert np.all(lab.cpu().numpy()[rej] == 0) and np.all(fail.cpu().numpy()[rej] == -2)
    assert np.array_equal(objq.cpu().numpy()[rej], q[rej][:, plan.obj_qposadr:plan.obj_qposadr + 7])


def test_fused_mask_rollout_equals_separate_launches(env, eng, candidates):
    """mgs_mask_rollout_device (the bench path) = mgs_collision_free_device then
    mgs_rollout_resumable_device over its mask, bit for bit: mask, labels, fail
    steps, object poses, statistics and resume records"""
    import torch
    from conftest import plan_for
    from mgs.core import abi
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    plan = plan_for(env, poses, J)
    sched = abi.make_schedule(plan.nsteps, plan.check_every, plan.check_at_end, plan.ctrl, plan.obj_qposadr,
                              check_offset=getattr(plan, "check_offset", None))
    n = len(q)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
    dq, dmp, dmq, dps, dpt = t(q), t(mp), t(mq), t(plan.phase_start), t(plan.phase_target)
    rw = eng.resume_width()
    outs = []
    for fused in (False, True):
        o = dict(free=torch.zeros(n, dtype=torch.uint8, device=dev), lab=torch.zeros(n, dtype=torch.uint8, device=dev),
                 fail=torch.zeros(n, dtype=torch.int32, device=dev),
                 objq=torch.zeros((n, 7), dtype=torch.float64, device=dev),
                 st=torch.zeros((n, abi.MGS["MGS_NSTATS"]), dtype=torch.int32, device=dev),
                 rec=torch.zeros((n, rw), dtype=torch.float64, device=dev))
        if fused:
            eng.mask_rollout_device(sched, n, dq.data_ptr(), dmp.data_ptr(), dmq.data_ptr(), dps.data_ptr(),
                                    dpt.data_ptr(), o["free"].data_ptr(), o["lab"].data_ptr(), o["fail"].data_ptr(),
                                    o["objq"].data_ptr(), o["st"].data_ptr(), d_resume_out=o["rec"].data_ptr())
        else:
            eng.collision_free_device(n, dq.data_ptr(), dmp.data_ptr(), dmq.data_ptr(), o["free"].data_ptr())
            eng.rollout_resumable_device(sched, n, dq.data_ptr(), dmq.data_ptr(), dps.data_ptr(), dpt.data_ptr(),
                                         o["lab"].data_ptr(), o["fail"].data_ptr(), o["objq"].data_ptr(),
                                         o["st"].data_ptr(), o["rec"].data_ptr(), d_active=o["free"].data_ptr())
        torch.cuda.synchronize()
        outs.append({k: v.cpu().numpy() for k, v in o.items()})
    for k in outs[0]:
        assert np.array_equal(outs[0][k], outs[1][k]), k
    assert 0 < outs[1]["free"].sum() < n


def test_work_queue_equals_one_workgroup_per_candidate(env, eng, candidates, oracle_model):
    """The work-queue launch (mgs_rollout_queue: a grid of k workgroups pulling
    candidate indices from a counter) gives every output of one workgroup per
    candidate bit for bit -- fused mask, labels, fail steps, object poses,
    statistics, resume records -- whatever the grid (k = 1, 5, 64 here; the
    default grid is the device's resident capacity), and equals the oracle."""
    import torch
    from conftest import plan_for
    from mgs.core import abi
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    plan = plan_for(env, poses, J)
    sched = abi.make_schedule(plan.nsteps, plan.check_every, plan.check_at_end, plan.ctrl, plan.obj_qposadr,
                              check_offset=getattr(plan, "check_offset", None))
    n = len(q)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
    dq, dmp, dmq, dps, dpt = t(q), t(mp), t(mq), t(plan.phase_start), t(plan.phase_target)
    rw = eng.resume_width()
    L = eng.lib
    prev = L.mgs_rollout_queue(-1)
    outs = {}
    try:
        for mode in (0, 1, 5, 64):
            L.mgs_rollout_queue(mode)
            assert eng.rollout_grid(n) == (n if mode <= 1 else mode)
            o = dict(free=torch.zeros(n, dtype=torch.uint8, device=dev),
                     lab=torch.zeros(n, dtype=torch.uint8, device=dev),
                     fail=torch.zeros(n, dtype=torch.int32, device=dev),
                     objq=torch.zeros((n, 7), dtype=torch.float64, device=dev),
                     st=torch.zeros((n, abi.MGS["MGS_NSTATS"]), dtype=torch.int32, device=dev),
                     rec=torch.zeros((n, rw), dtype=torch.float64, device=dev))
            for _ in range(2):      # two launches in a row: each leaves its counter pair zeroed
                if mode > 0:
                    # a call refused before its launch (bad predicate) leaves no trace
                    import ctypes
                    rc = L.mgs_mask_rollout_device(eng.batch(1), ctypes.byref(sched), n, dq.data_ptr(),
                                                   dmp.data_ptr(), dmq.data_ptr(), dps.data_ptr(), dpt.data_ptr(),
                                                   99, o["free"].data_ptr(), o["lab"].data_ptr(),
                                                   o["fail"].data_ptr(), o["objq"].data_ptr(), o["st"].data_ptr(),
                                                   None, None, None)
                    assert rc != 0
                eng.mask_rollout_device(sched, n, dq.data_ptr(), dmp.data_ptr(), dmq.data_ptr(), dps.data_ptr(),
                                        dpt.data_ptr(), o["free"].data_ptr(), o["lab"].data_ptr(),
                                        o["fail"].data_ptr(), o["objq"].data_ptr(), o["st"].data_ptr(),
                                        d_resume_out=o["rec"].data_ptr())
            torch.cuda.synchronize()
            outs[mode] = {k: v.cpu().numpy() for k, v in o.items()}
    finally:
        L.mgs_rollout_queue(prev)
    for mode in (1, 5, 64):
        for k in outs[0]:
            assert np.array_equal(outs[0][k], outs[mode][k]), (mode, k)
    free = outs[5]["free"].astype(bool)
    assert np.array_equal(free, oracle_model.collision_free(q, mp, mq, nthreads=8))
    idx = np.nonzero(free)[0]
    ro = oracle_model.rollout(plan_for(env, poses[idx], J[idx]), nthreads=8)
    # candidates over the capacity stop there with a resume record (fail step
    # -3, the escalation's input); the oracle at that capacity runs on capped
    fit = (outs[5]["st"][idx, 2] & abi.MGS["MGS_FLAG_CAPACITY"]) == 0
    assert fit.sum() > len(idx) // 2 and np.all(outs[5]["fail"][idx][~fit] == -3)
    assert np.array_equal(outs[5]["lab"].astype(bool)[idx][fit], ro["label"][fit])
    assert np.array_equal(outs[5]["fail"][idx][fit], ro["fail_step"][fit])
    assert np.array_equal(outs[5]["objq"][idx][fit], ro["obj_qpos"][fit])


@pytest.mark.parametrize("grid,yield_every", [(5, 1), (5, 7), (64, 7), (16, 32)])
def test_rotation_equals_one_workgroup_per_candidate(env, eng, candidates, grid, yield_every):
    """In-launch rotation (mgs_schedule.yield_every, ABI 19): on a work-queue
    grid smaller than the batch, a candidate that has run yield_every steps
    hands its slot to a waiting one (its record to the launch's ring, another
    workgroup continues it).  Every output -- fused mask, labels, fail steps,
    object poses, statistics -- equals one workgroup per candidate without
    rotation bit for bit, for two launches in a row on the same queue slot
    ring (each leaves its counters and ring zeroed); yield_every 1 rotates at
    every step."""
    import torch
    from conftest import plan_for
    from mgs.core import abi
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    plan = plan_for(env, poses, J)
    n = len(q)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
    dq, dmp, dmq, dps, dpt = t(q), t(mp), t(mq), t(plan.phase_start), t(plan.phase_target)
    rw = eng.resume_width()
    L = eng.lib
    prev = L.mgs_rollout_queue(-1)
    outs = {}
    yields, spins = [], []
    try:
        for mode, ye in ((0, 0), (grid, yield_every)):
            y0, s0 = eng.queue_stats()
            yields.append(y0)
            spins.append(s0)
            L.mgs_rollout_queue(mode)
            sched = abi.make_schedule(plan.nsteps, plan.check_every, plan.check_at_end, plan.ctrl,
                                      plan.obj_qposadr, check_offset=getattr(plan, "check_offset", None))
            sched.yield_every = ye
            for rep in range(2):
                o = dict(free=torch.zeros(n, dtype=torch.uint8, device=dev),
                         lab=torch.zeros(n, dtype=torch.uint8, device=dev),
                         fail=torch.zeros(n, dtype=torch.int32, device=dev),
                         objq=torch.zeros((n, 7), dtype=torch.float64, device=dev),
                         st=torch.zeros((n, abi.MGS["MGS_NSTATS"]), dtype=torch.int32, device=dev),
                         rec=torch.zeros((n, rw), dtype=torch.float64, device=dev))
                eng.mask_rollout_device(sched, n, dq.data_ptr(), dmp.data_ptr(), dmq.data_ptr(), dps.data_ptr(),
                                        dpt.data_ptr(), o["free"].data_ptr(), o["lab"].data_ptr(),
                                        o["fail"].data_ptr(), o["objq"].data_ptr(), o["st"].data_ptr(),
                                        d_resume_out=o["rec"].data_ptr())
                torch.cuda.synchronize()
                outs[(mode, rep)] = {k: v.cpu().numpy() for k, v in o.items() if k != "rec"}
        y1, s1 = eng.queue_stats()
        yields.append(y1)
        spins.append(s1)
        yields, spins = yields[1:], spins[1:]
    finally:
        L.mgs_rollout_queue(prev)
    ref = outs[(0, 0)]
    assert 0 < ref["free"].sum() < n
    for rep in range(2):
        for k in ref:
            assert np.array_equal(ref[k], outs[(grid, rep)][k]), (grid, yield_every, rep, k)
    # the rotation ran (candidates yielded: every grid here is smaller than the
    # batch's rollouts) and its ring protocol never timed out
    assert yields[1] > yields[0] and spins[1] == spins[0] == 0, (yields, spins)


def test_env_rotation_equals_one_launch(env, candidates, oracle_model):
    """GravitylessObjectGrasping.rollout with its default in-launch rotation
    on a small queue grid equals the same call without rotation, and the
    oracle (h200 and ref8000)."""
    from conftest import plan_for
    from oracle import oracle as O
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    idx = np.nonzero(oracle_model.collision_free(q, mp, mq, nthreads=8))[0]
    L = env.engine.lib
    prev = L.mgs_rollout_queue(-1)
    try:
        for horizon, sub in (("h200", idx[:128]), ("ref8000", idx[:6])):
            plan = plan_for(env, poses[sub], J[sub], horizon)
            L.mgs_rollout_queue(0)
            one = env.rollout(plan, yield_every=0)
            L.mgs_rollout_queue(4 if horizon == "ref8000" else 16)
            rot = env.rollout(plan, yield_every=64 if horizon == "ref8000" else 16)
            _assert_same(rot, one, f"rotation {horizon}")
            if horizon == "h200":
                # the env escalates past its capacity: the full-capacity oracle's results
                full = O.OracleModel(env.model, ncon_max=128, nefc_max=256).rollout(plan, nthreads=8)
                for k in ("label", "fail_step", "obj_qpos"):
                    assert np.array_equal(one[k], full[k]), k
    finally:
        L.mgs_rollout_queue(prev)


def test_device_overflow_list_and_list_rollout(env, eng, candidates):
    """mgs_overflow_list_device picks the flagged candidates; mgs_rollout_list_device
    with a grid smaller than the list (workgroups loop over it) reproduces
    mgs_rollout_device's outputs at the listed indices and touches nothing else."""
    import torch
    from conftest import plan_for
    from mgs.core import abi
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    plan = plan_for(env, poses, J)
    sched = abi.make_schedule(plan.nsteps, plan.check_every, plan.check_at_end, plan.ctrl, plan.obj_qposadr,
                              check_offset=getattr(plan, "check_offset", None))
    n = len(q)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
    dq, dmq, dps, dpt = t(q), t(mq), t(plan.phase_start), t(plan.phase_target)

    def outs(fill):
        return (torch.full((n,), fill, dtype=torch.uint8, device=dev), torch.full((n,), -7, dtype=torch.int32, device=dev),
                torch.full((n, 7), 9.0, dtype=torch.float64, device=dev),
                torch.full((n, abi.MGS["MGS_NSTATS"]), -1, dtype=torch.int32, device=dev))
    full = outs(0)
    eng.rollout_device(sched, n, dq.data_ptr(), dmq.data_ptr(), dps.data_ptr(), dpt.data_ptr(),
                       *[x.data_ptr() for x in full])
    # synthetic flags: every 7th candidate overflowed
    flags = torch.zeros((n, abi.MGS["MGS_NSTATS"]), dtype=torch.int32, device=dev)
    pick = np.arange(3, n, 7)
    flags[torch.as_tensor(pick, device=dev), 2] = abi.MGS["MGS_FLAG_CONTACTS"]
    cnt = torch.zeros(abi.MGS["MGS_LIST_HEADER"], dtype=torch.int32, device=dev)
    lst = torch.zeros(n, dtype=torch.int32, device=dev)
    eng.overflow_list_device(n, flags.data_ptr(), cnt.data_ptr(), lst.data_ptr())
    sub = outs(5)
    eng.rollout_list_device(sched, n, cnt.data_ptr(), lst.data_ptr(), 3, dq.data_ptr(), dmq.data_ptr(),
                            dps.data_ptr(), dpt.data_ptr(), *[x.data_ptr() for x in sub])
    torch.cuda.synchronize()
    # the list run records the count it ran (word 2) and leaves count / exits zeroed
    hdr = cnt.cpu().numpy()
    k = int(hdr[2])
    assert hdr[0] == 0 and hdr[1] == 0
    assert k == len(pick) and sorted(lst.cpu().numpy()[:k]) == list(pick)
    for a, b in zip(full, sub):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        assert np.array_equal(a[pick], b[pick])
    rest = np.setdiff1d(np.arange(n), pick)
    assert np.all(sub[0].cpu().numpy()[rest] == 5) and np.all(sub[1].cpu().numpy()[rest] == -7)
    # an empty list launches and changes nothing
    eng.rollout_list_device(sched, n, cnt.data_ptr(), lst.data_ptr(), 3, dq.data_ptr(), dmq.data_ptr(),
                            dps.data_ptr(), dpt.data_ptr(), *[x.data_ptr() for x in sub])
    torch.cuda.synchronize()
    assert np.all(sub[0].cpu().numpy()[rest] == 5)
    assert cnt.cpu().numpy().tolist()[:3] == [0, 0, 0]


def test_full_size_properties(env, eng, oracle_model):
    """8192 candidates (the benchmark size): determinism, permutation
    invariance and sub-batch consistency, tied to the oracle on a slice."""
    from conftest import plan_for
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose
    H, J, _ = robotiq_candidates(env.obj, 8192, seed=5)
    poses = SE3Pose.from_mat(H)
    J = np.asarray(J, np.float64)
    q, mp, mq, _ = env.initial_state(poses, J)
    mask = eng.collision_free(q, mp, mq)
    assert np.array_equal(mask, eng.collision_free(q, mp, mq))
    idx = np.nonzero(mask)[0]
    plan = plan_for(env, poses[idx], J[idx])
    r1 = eng.rollout(plan)
    r2 = eng.rollout(plan)
    _assert_same(r1, r2, "rerun")
    perm = np.random.default_rng(0).permutation(len(idx))
    rp = eng.rollout(plan_for(env, poses[idx[perm]], J[idx[perm]]))
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(rp[k], r1[k][perm]), k
    k = min(24, len(idx))
    ro = oracle_model.rollout(plan_for(env, poses[idx[:k]], J[idx[:k]]), nthreads=8)
    for key in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(r1[key][:k], ro[key]), key


def test_contact_capacity_escalation(env):
    """Candidates whose contacts exceed ncon_max=16 (7 of the seed-0 8192 block)
    are re-run at ncon_max=32 by GravitylessObjectGrasping.rollout; every result
    then equals the oracle run at the capacity that held it, and none stays capped."""
    from conftest import plan_for
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose
    from oracle import oracle as O
    e16 = GravitylessObjectGrasping(env.gripper, env.obj, ncon_max=16)
    H, J, _ = robotiq_candidates(env.obj, 8192, seed=0)
    P = SE3Pose.from_mat(H)
    q, mp, mq, _ = e16.initial_state(P, J)
    idx = np.nonzero(e16.engine.collision_free(q, mp, mq))[0]
    plan = plan_for(e16, P[idx], J[idx])
    capped = e16.engine.rollout(plan)
    ov = np.nonzero(capped["stats"][:, 2])[0]
    assert len(ov) > 0
    res = e16.rollout(plan)
    assert res["overflow"] == 0
    keep = np.setdiff1d(np.arange(len(idx)), ov)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(res[k][keep], capped[k][keep]), k
    # the escalation's stages (32, 64, 128 contacts) end where each one fits:
    # equal to the oracle at full capacity
    ro = O.OracleModel(env.model, ncon_max=128, nefc_max=256).rollout(plan.subset(ov), nthreads=8)
    for k in ("label", "fail_step", "obj_qpos"):
        assert np.array_equal(res[k][ov], ro[k]), k
    assert not (res["stats"][ov, 2] & 3).any()


def test_capped_contact_set_raises_never_labels(env):
    """a call whose escalation cannot hold a candidate's contacts
    (max_ncon below them) raises CapacityError -- no label from a capped
    contact set -- and with the default escalation the same call returns the
    full-capacity oracle's results"""
    from conftest import plan_for
    from mgs.env.gravityless_object_grasping import CapacityError, GravitylessObjectGrasping
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose
    from oracle import oracle as O
    e4 = GravitylessObjectGrasping(env.gripper, env.obj, ncon_max=4)
    H, J, _ = robotiq_candidates(env.obj, 2048, seed=0)
    P = SE3Pose.from_mat(H)
    q, mp, mq, _ = e4.initial_state(P, J)
    idx = np.nonzero(e4.engine.collision_free(q, mp, mq))[0][:64]
    plan = plan_for(e4, P[idx], J[idx])
    ro = O.OracleModel(env.model, ncon_max=128, nefc_max=256).rollout(plan, nthreads=8)
    over8 = np.nonzero(ro["stats"][:, 0] > 8)[0]
    assert len(over8) > 0
    with pytest.raises(CapacityError) as ei:
        e4.rollout(plan, max_ncon=8)
    assert set(ei.value.candidates.tolist()) <= set(range(len(idx)))
    assert set(over8.tolist()) & set(ei.value.candidates.tolist())
    res = e4.rollout(plan)            # 4 -> 8 -> ... -> 128
    for k in ("label", "fail_step", "obj_qpos"):
        assert np.array_equal(res[k], ro[k]), k
    assert res["overflow"] == 0


def test_resumed_escalation_equals_wide_run(env, candidates):
    """Capacity 4 overflows most candidates: each stops at its overflowing step
    and is continued from the state entering it at 8, 16, 32 and 40 contacts
    (mgs_rollout_resume, chained).  Every output equals one run at 40 from the
    start, bit for bit; so does the device path (resumable rollout -> overflow
    list -> list rollout continuing from the records)."""
    import torch
    from conftest import plan_for
    from mgs.core import abi
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    e4 = GravitylessObjectGrasping(env.gripper, env.obj, ncon_max=4)
    poses, J = candidates
    q, mp, mq, _ = e4.initial_state(poses, J)
    idx = np.nonzero(e4.engine.collision_free(q, mp, mq))[0][:96]
    plan = plan_for(e4, poses[idx], J[idx])
    n = len(idx)
    ref = e4.engine_for(40).rollout(plan)
    capped = e4.engine.rollout(plan, resumable=True)
    stopped = np.nonzero(capped["stats"][:, 2] & abi.MGS["MGS_FLAG_CAPACITY"])[0]
    assert len(stopped) > n // 4
    assert np.all(capped["fail_step"][stopped] == -3) and not capped["label"][stopped].any()
    res = e4.rollout(plan, max_ncon=40)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(res[k], ref[k]), k
    assert res["overflow"] == int((ref["stats"][:, 2] & abi.MGS["MGS_FLAG_CAPACITY"] != 0).sum())
    # device path, one stage 4 -> 40
    sched = abi.make_schedule(plan.nsteps, plan.check_every, plan.check_at_end, plan.ctrl, plan.obj_qposadr,
                              check_offset=getattr(plan, "check_offset", None))
    dev = torch.device("cuda", 0)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
    dq, dmq, dps, dpt = t(plan.qpos_init), t(plan.mocap_quat), t(plan.phase_start), t(plan.phase_target)
    NS = abi.MGS["MGS_NSTATS"]
    outs = lambda: (torch.zeros(n, dtype=torch.uint8, device=dev), torch.zeros(n, dtype=torch.int32, device=dev),  # noqa
                    torch.zeros((n, 7), dtype=torch.float64, device=dev),
                    torch.zeros((n, NS), dtype=torch.int32, device=dev))
    main, esc = outs(), outs()
    rec = torch.zeros((n, e4.engine.resume_width()), dtype=torch.float64, device=dev)
    e4.engine.rollout_resumable_device(sched, n, dq.data_ptr(), dmq.data_ptr(), dps.data_ptr(), dpt.data_ptr(),
                                       *[x.data_ptr() for x in main], rec.data_ptr())
    cnt = torch.zeros(abi.MGS["MGS_LIST_HEADER"], dtype=torch.int32, device=dev)
    lst = torch.zeros(n, dtype=torch.int32, device=dev)
    e4.engine.overflow_list_device(n, main[3].data_ptr(), cnt.data_ptr(), lst.data_ptr())
    e4.engine_for(40).rollout_list_device(sched, n, cnt.data_ptr(), lst.data_ptr(), 5, dq.data_ptr(),
                                          dmq.data_ptr(), dps.data_ptr(), dpt.data_ptr(),
                                          *[x.data_ptr() for x in esc], d_resume_in=rec.data_ptr())
    torch.cuda.synchronize()
    k = int(cnt[2].item())
    lo = np.sort(lst.cpu().numpy()[:k])
    assert np.array_equal(lo, stopped)
    # ABI 17: the capped launch appends its overflowing candidates to a list
    # itself (no list kernel); the list re-run over it gives the same outputs,
    # twice in a row on the same header (left zeroed by each re-run)
    H = abi.MGS["MGS_LIST_HEADER"]
    ovf = torch.zeros(H + n, dtype=torch.int32, device=dev)
    for _ in range(2):
        main2, esc2 = outs(), outs()
        rec2 = torch.zeros_like(rec)
        e4.engine.rollout_resumable_device(sched, n, dq.data_ptr(), dmq.data_ptr(), dps.data_ptr(), dpt.data_ptr(),
                                           *[x.data_ptr() for x in main2], rec2.data_ptr(), d_ovf=ovf.data_ptr())
        e4.engine_for(40).rollout_list_device(sched, n, ovf.data_ptr(), ovf.data_ptr() + 4 * H, 5, dq.data_ptr(),
                                              dmq.data_ptr(), dps.data_ptr(), dpt.data_ptr(),
                                              *[x.data_ptr() for x in esc2], d_resume_in=rec2.data_ptr())
        torch.cuda.synchronize()
        o = ovf.cpu().numpy()
        assert o[0] == 0 and o[1] == 0 and o[2] == k
        assert np.array_equal(np.sort(o[H:H + k]), stopped)
        for a, b in zip(main, main2):
            assert torch.equal(a, b)
        for a, b in zip(esc, esc2):
            a, b = a.cpu().numpy(), b.cpu().numpy()
            assert np.array_equal(a[lo], b[lo])
    got = [x.cpu().numpy() for x in main]
    for a, e in zip(got, [x.cpu().numpy() for x in esc]):
        a[lo] = e[lo]
    for key, a in zip(("label", "fail_step", "obj_qpos", "stats"), got):
        assert np.array_equal(a.astype(ref[key].dtype), ref[key]), key


def test_divergence_guard_parity(env, eng, candidates, oracle_model):
    """injected NaN / beyond-mjMAXVAL states: the GPU stops and flags exactly the
    candidates the oracle does (obj_qpos compared with NaN == NaN)."""
    from test_oracle import _guard_plan
    plan = _guard_plan(env, candidates, oracle_model)
    rg = eng.rollout(plan)
    ro = oracle_model.rollout(plan)
    for k in ("label", "fail_step", "stats"):
        assert np.array_equal(rg[k], ro[k]), k
    assert np.array_equal(rg["obj_qpos"], ro["obj_qpos"], equal_nan=True)


def test_specialised_kernels_match_runtime_layout(env, eng, candidates):
    """The headline engine runs its model-specialised code object (constant
    layout and description); an engine of the same model and capacity without
    it runs the library's runtime-offset kernels: every output is identical."""
    from conftest import plan_for
    from mgs.core.engine import Engine
    assert eng.specialized()
    other = Engine(env.model, ncon_max=env.ncon_max, nefc_max=env.nefc_max, specialize=False)
    assert not other.specialized()
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    assert np.array_equal(eng.collision_free(q, mp, mq), other.collision_free(q, mp, mq))
    idx = np.nonzero(eng.collision_free(q, mp, mq))[0][:64]
    plan = plan_for(env, poses[idx], J[idx])
    a, b = eng.rollout(plan), other.rollout(plan)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(a[k], b[k]), k


def test_specialised_object_of_another_model_is_refused(env, eng):
    """mgs_model_attach_special reads the object's baked description and layout
    back and refuses an object made for another capacity"""
    import ctypes
    from mgs.core import abi, special
    from mgs.core.engine import Engine, EngineError
    path = special.code_object(eng.lib, eng.desc, compile=False)
    assert path is not None
    other = Engine(env.model, ncon_max=env.ncon_max, nefc_max=env.nefc_max - 1, specialize=False)
    with pytest.raises(EngineError):
        other._ck(other.lib.mgs_model_attach_special(other._model, path.encode()), "mgs_model_attach_special")
    assert not other.specialized()


@pytest.mark.parametrize("nefc_max", [10, 16, 40])
def test_row_capacity_overflow_parity(env, candidates, nefc_max):
    """Constraint-row capacities below the equality rows (10 < 13), just above
    them (16) and mid-range (40): which equality / friction / limit / contact
    rows are kept, the overflow flags, and everything downstream match the
    oracle at the same capacity (the kernel places equality and contact rows for
    all of them at once; the oracle appends them one by one)."""
    from conftest import plan_for
    from mgs.core.engine import Engine
    from oracle import oracle as O
    poses, J = candidates
    plan = plan_for(env, poses[:40], J[:40])
    e = Engine(env.model, ncon_max=8, nefc_max=nefc_max)
    om = O.OracleModel(env.model, ncon_max=8, nefc_max=nefc_max)
    rg, ro = e.rollout(plan), om.rollout(plan, nthreads=8)
    _assert_same(rg, ro, f"nefc_max={nefc_max}")
    assert (rg["stats"][:, 2] & 2).any()


@pytest.mark.parametrize("horizon,n,slices", [("h200", 256, [2, 3, 7]), ("ref8000", 4, [5])])
def test_time_slices_equal_one_launch(env, candidates, oracle_model, horizon, n, slices):
    """GravitylessObjectGrasping.rollout in time slices (mgs_schedule.pause_step:
    every unfinished candidate stops at the slice boundary with its resume
    record, MGS_FLAG_PAUSED, and the next launch continues the survivors) gives
    every output of one launch bit for bit, and equals the oracle; a pause
    right at a phase boundary and inside the lift's check cadence included
    (h200: phases end at 76 / 152 / 164 / 176)"""
    from conftest import plan_for
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    idx = np.nonzero(oracle_model.collision_free(q, mp, mq, nthreads=8))[0][:n]
    plan = plan_for(env, poses[idx], J[idx], horizon)
    one = env.rollout(plan, slices=1)
    assert one["overflow"] == 0
    for k in slices:
        r = env.rollout(plan, slices=k)
        _assert_same(r, one, f"{k} slices")
    # a boundary on a phase end (76) and one on a lift check (76 + 25), on the
    # main engine: the candidates its capacity holds (the others stop at -3
    # for the escalation, which one launch continues wider)
    e = env.engine
    fit = (e.rollout(plan)["stats"][:, 2] & abi_flag("MGS_FLAG_CAPACITY")) == 0
    assert fit.sum() > len(idx) // 2
    for b in (76, 101):
        a = e.rollout(plan, resumable=True, pause_step=b)
        live = np.nonzero(a["stats"][:, 2] & abi_flag("MGS_FLAG_PAUSED"))[0]
        assert np.all(a["fail_step"][live] == -4)
        if len(live):
            sub = e.rollout(plan.subset(live), resumable=True, resume_from=a["resume"][live])
            for k in ("label", "fail_step", "obj_qpos", "stats"):
                a[k][live] = sub[k]
        keys = ("label", "fail_step", "obj_qpos", "stats")
        _assert_same({k: a[k][fit] for k in keys}, {k: one[k][fit] for k in keys}, f"pause at {b}")
    from oracle import oracle as O
    ro = O.OracleModel(env.model, ncon_max=128, nefc_max=256).rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos"):
        assert np.array_equal(one[k], ro[k]), k


def abi_flag(name):
    from mgs.core.abi import MGS
    return MGS[name]


def test_time_slices_keep_capacity_flags(env, candidates):
    """with the last escalation stage from the first launch
    (ncon_max = max_ncon = 4, capped_continue), a capped candidate that pauses
    at a slice boundary keeps its capacity flag in the relaunch (the record
    carries MGS_FLAG_PAUSED and the resumed run restores its flags without it),
    so slices equal one launch in every output, res['overflow'] included"""
    from conftest import plan_for
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    e4 = GravitylessObjectGrasping(env.gripper, env.obj, ncon_max=4)
    poses, J = candidates
    q, mp, mq, _ = e4.initial_state(poses, J)
    idx = np.nonzero(e4.engine.collision_free(q, mp, mq))[0][:96]
    plan = plan_for(e4, poses[idx], J[idx])
    one = e4.rollout(plan, max_ncon=4, slices=1, on_capacity="capped")
    assert one["overflow"] > 0
    for k in (2, 3, 7):
        r = e4.rollout(plan, max_ncon=4, slices=k, on_capacity="capped")
        _assert_same(r, one, f"{k} slices, capped")
        assert r["overflow"] == one["overflow"]


def _device_run(eng, plan, q, mp, n, sched, dev):
    import torch
    from mgs.core import abi
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
    o = dict(free=torch.zeros(n, dtype=torch.uint8, device=dev), lab=torch.zeros(n, dtype=torch.uint8, device=dev),
             fail=torch.zeros(n, dtype=torch.int32, device=dev),
             objq=torch.zeros((n, 7), dtype=torch.float64, device=dev),
             st=torch.zeros((n, abi.MGS["MGS_NSTATS"]), dtype=torch.int32, device=dev))
    rec = torch.zeros((n, eng.resume_width()), dtype=torch.float64, device=dev)
    ins = [t(a) for a in (q, mp, plan.mocap_quat, plan.phase_start, plan.phase_target)]
    eng.mask_rollout_device(sched, n, *[x.data_ptr() for x in ins], o["free"].data_ptr(), o["lab"].data_ptr(),
                            o["fail"].data_ptr(), o["objq"].data_ptr(), o["st"].data_ptr(),
                            d_resume_out=rec.data_ptr())
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in o.items()}


def test_rotation_rings_sized_by_launch_n(env):
    """a fresh engine's batch holds 256 candidates, but a
    device launch over n = 1024 rotates through rings indexed modulo 2n; the
    rings are sized for the launch's n (grown on demand), so a rotating launch
    over more candidates than the batch capacity equals one workgroup per
    candidate bit for bit with no expired spin"""
    import torch
    from conftest import plan_for
    from mgs.core import abi
    from mgs.core.engine import Engine, check_no_lost_candidates
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose
    n = 1024
    H, J, _ = robotiq_candidates(env.obj, n, seed=3)
    P = SE3Pose.from_mat(H)
    q, mp, mq, _ = env.initial_state(P, J)
    plan = plan_for(env, P, J)
    fresh = Engine(env.model, ncon_max=env.ncon_max, nefc_max=env.nefc_max)
    assert fresh.specialized()
    sched = abi.make_schedule(plan.nsteps, plan.check_every, plan.check_at_end, plan.ctrl, plan.obj_qposadr)
    dev = torch.device("cuda", 0)
    L = fresh.lib
    prev = L.mgs_rollout_queue(-1)
    try:
        L.mgs_rollout_queue(0)
        ref = _device_run(fresh, plan, q, mp, n, sched, dev)
        sched.yield_every = 5
        L.mgs_rollout_queue(48)
        for _ in range(2):
            got = _device_run(fresh, plan, q, mp, n, sched, dev)
            for k in ref:
                assert np.array_equal(ref[k], got[k]), k
    finally:
        L.mgs_rollout_queue(prev)
    y, s = fresh.queue_stats()
    assert y > 0 and s == 0
    check_no_lost_candidates(got["fail"], s)
    fresh.close()


def test_lost_rotation_candidate_raises(env, candidates):
    """verdict r4 item 3: a rotation that loses a candidate must not return
    stale labels.  A fault-injection object (role "fault", -DMGS_TEST_DROP_POP:
    every ring pop expires and drops the candidate it took) makes the env's
    rollout raise EngineError (mgs_rollout fails with MGS_EQUEUE), and on the
    device path the lost candidates keep the MGS_FAIL_YIELDED sentinel that
    check_no_lost_candidates reports; the same engine runs correctly after
    the reset (rotation off)"""
    import torch
    from conftest import plan_for
    from mgs.core import abi, special
    from mgs.core.engine import Engine, EngineError, check_no_lost_candidates
    from mgs.env.gravityless_object_grasping import sliced_rollout
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    idx = np.nonzero(env.engine.collision_free(q, mp, mq))[0][:64]
    plan = plan_for(env, poses[idx], J[idx])
    bad = Engine(env.model, ncon_max=env.ncon_max, nefc_max=env.nefc_max, specialize=False)
    path = special.code_object(bad.lib, bad.desc, compile=False, role="fault")
    assert path is not None, "the fault-injection object is built by __graft_entry__.build()"
    bad._ck(bad.lib.mgs_model_attach_special(bad._model, path.encode()), "mgs_model_attach_special")
    L = bad.lib
    prev = L.mgs_rollout_queue(-1)
    try:
        L.mgs_rollout_queue(8)
        with pytest.raises(EngineError, match="rotation"):
            sliced_rollout(plan, bad, lambda c: bad, env.ncon_max, env.ncon_max, 1, yield_every=7)
        # device path: the sentinel marks the lost candidates
        n = len(q)
        plan_all = plan_for(env, poses, J)
        sched = abi.make_schedule(plan_all.nsteps, plan_all.check_every, plan_all.check_at_end, plan_all.ctrl,
                                  plan_all.obj_qposadr)
        sched.yield_every = 7
        y0, s0 = bad.queue_stats()
        got = _device_run(bad, plan_all, q, mp, n, sched, torch.device("cuda", 0))
        y1, s1 = bad.queue_stats()
        assert s1 > s0 and (got["fail"] == abi.MGS["MGS_FAIL_YIELDED"]).any()
        with pytest.raises(EngineError, match="lost"):
            check_no_lost_candidates(got["fail"], s1 - s0)
        # rotation off: the same engine (rings reset) gives the oracle-checked outputs
        r = bad.rollout(plan, resumable=True)
        _assert_same(r, env.engine.rollout(plan, resumable=True), "after the fault")
    finally:
        L.mgs_rollout_queue(prev)
        bad.close()


@pytest.mark.gpu
def test_queue_spans_device_clock(env, candidates):
    """mgs_queue_spans: a work-queue rollout launch leaves its execution span
    on the device's real-time counter (bench.py's launch_ms); the call
    returns each completed launch once, then clears it"""
    from conftest import plan_for
    eng = env.engine
    eng.queue_spans()
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    idx = np.nonzero(eng.collision_free(q, mp, mq))[0]
    prev = eng.lib.mgs_rollout_queue(16)       # the queue on 16 workgroups: a real work queue
    try:
        r = eng.rollout(plan_for(env, poses[idx], J[idx]))
    finally:
        eng.lib.mgs_rollout_queue(prev)
    s = eng.queue_spans()
    assert len(s) == 1 and eng.spans_overwritten == 0
    assert 0.0 < s[0] <= r["kernel_ms"] * 1.05 + 0.05     # inside the HIP events around the launch
    assert eng.queue_spans() == []
    # more than the ring's 64 launches between two calls: the lost ones are counted
    sub = plan_for(env, poses[idx[:20]], J[idx[:20]], horizon="h200")
    sub.nsteps = [2] * len(sub.nsteps)
    prev = eng.lib.mgs_rollout_queue(4)
    try:
        for _ in range(70):
            eng.rollout(sub)
    finally:
        eng.lib.mgs_rollout_queue(prev)
    s = eng.queue_spans()
    assert len(s) == 64 and eng.spans_overwritten == 6


@pytest.mark.gpu
def test_small_rollout_calls_take_the_latency_engine(env, candidates):
    """a rollout call of at most LATENCY_ROUNDS x the G-rows-in-LDS engine's
    resident grid runs on that engine (shorter steps: one round of rollouts
    ends sooner), a larger one on the eight-per-CU main engine; both give the
    oracle's results bit for bit, so the env's answer does not depend on the
    choice"""
    from conftest import plan_for
    from mgs.env.gravityless_object_grasping import sliced_rollout
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    idx = np.nonzero(env.engine.collision_free(q, mp, mq))[0][:48]
    plan = plan_for(env, poses[idx], J[idx])
    le = env.latency_engine
    assert int(env.engine.desc.g_rows_hbm) and le is not None and not int(le.desc.g_rows_hbm)
    assert env.engine_for_rollouts(len(idx)) is le
    big = int(env.LATENCY_ROUNDS * le.rollout_grid(4096)) + 1
    assert env.engine_for_rollouts(big) is env.engine
    r_small = env.rollout(plan)
    r_main = sliced_rollout(plan, env.engine, env.engine_for, env.ncon_max, 40, 1, yield_every=env.YIELD_EVERY)
    _assert_same(r_small, r_main, "latency engine vs main engine")
