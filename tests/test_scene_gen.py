"""Scene generation: the free-simulation entry point
mgs_simulate behind ClutterTableEnv.gen_clutter / is_stable / settle
(clutter_table.py:155-222), the object-set selector (obj/selector.py:54-246)
and the gen_scene CLI (cli/gen_scene.py:15-212).

CPU: get_objects' parked layout, the config interpolation, and the oracle's
free simulation (checks off, vstate, vclip).  GPU: mgs_simulate bit-exact
against oracle.simulate_batch, and a batch of gen_clutter piles plus the
is_stable test bit-exact against the same sequence run on the oracle; the
gen_scene CLI end to end."""
import os
import random
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
SCENE = os.path.join(HERE, "golden", "clutter_scene.npz")


def _gpu():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass


@pytest.fixture(scope="module")
def senv():
    from make_clutter_scene import make_env
    env = make_env()
    env.set_state(np.load(SCENE)["state"])
    return env


def test_get_objects_parked_layout():
    from mgs.obj.selector import get_objects
    from mgs.util.const import ASSET_PATH
    objs = get_objects({"name": "Fast_Data_Subset", "num_objects": 12}, random.Random(0))
    xy = np.array([o.pos[:2] for o in objs])
    assert len(objs) == 12 and len({o.name for o in objs}) == 12
    assert np.allclose(xy[:10, 0], -8.0) and np.allclose(xy[10:, 0], -7.5)
    assert np.allclose(xy[:10, 1], -8.0 + 0.5 * np.arange(10)) and np.allclose(xy[10:, 1], [-8.0, -7.5])
    fast = open(os.path.join(ASSET_PATH, "mj-objects", "fast_eta_objects.txt")).read().splitlines()
    assert all(o.object_id in fast for o in objs)
    ids = lambda s: [o.object_id for o in get_objects({"name": "Fast_Data_Subset", "num_objects": 5}, s)]
    assert ids(4) == ids(4)
    ycb = [o.object_id for o in get_objects({"name": "YCB"})]
    assert ycb == sorted(ycb) and len(ycb) > 0
    sub = get_objects({"name": "Full_Data_Subset", "num_objects_min": 2, "num_objects_max": 3}, 1)
    assert 2 <= len(sub) <= 3
    with pytest.raises(ValueError):
        get_objects({"name": "nope"})


def test_gen_scene_config():
    from mgs.cli._hydra import compose
    cfg = compose("gen_scene", ["num_objects=3", "gripper=robotiq_2f_85"])
    assert cfg.object.name == "Fast_Data_Subset" and cfg.object.num_objects == 3
    assert cfg.env.name == "ClutterTable" and cfg.gripper.name == "Robotiq2f85Gripper"
    assert cfg.only_collision_free is False and cfg.scene_batch == 1


class _FakeEnv:
    """host-logic stand-in for filter_grasps: object 0 at the origin, object 1
    shifted; every other grasp collides, every third collision-free one holds."""
    object_names, object_ids = ["a", "b"], ["id_a", "id_b"]

    def get_obj_pose(self, name):
        from mgs.util.geo.transforms import SE3Pose
        return SE3Pose(np.array([0.0, 0.0, 0.0] if name == "a" else [1.0, 0.0, 0.0]), np.array([1.0, 0, 0, 0]),
                       "wxyz")

    def grasp_collision_mask(self, poses, joints):
        return np.arange(len(poses)) % 2 == 0

    def grasp_stable_mask(self, poses, joints, state, enough_stable=None, **kw):
        from mgs.env.gravityless_object_grasping import apply_enough_stable
        return apply_enough_stable(np.arange(len(poses)) % 3 == 0, enough_stable)


def test_gen_scene_filter_grasps_host_logic(monkeypatch):
    """gen_scene.py:48-159 host rules: object-frame grasps posed by the object
    pose, collision split, enough_stable = min(128, 32 * num_objects), and the
    reference's unshuffled object indices (fixed by fix_shuffle)."""
    from mgs.cli import gen_scene
    from mgs.cli._hydra import compose
    eye = np.tile(np.eye(4, dtype=np.float32), (6, 1, 1))
    eye[:, 2, 3] = np.arange(6)
    monkeypatch.setattr(gen_scene, "get_env_from_dict", lambda cfg, sd: _FakeEnv())
    monkeypatch.setattr(gen_scene, "get_grasps", lambda g, oid: (eye, np.zeros((6, 1))))
    scene = {"env_state": {"state": np.zeros(3)}}
    # 12 grasps, 6 collision-free (3 per object), 2 of them stable: the default
    # enough_stable = min(128, 32 * 2) = 64 and an explicit 3 both fail
    cfg = compose("gen_scene", ["num_objects=2", "enough_collision_free=6"])
    assert cfg.get("enough_stable") is None
    with pytest.raises(ValueError, match="Not enough stable"):
        gen_scene.filter_grasps(cfg, scene, rng=0)
    with pytest.raises(ValueError, match="Not enough stable"):
        gen_scene.filter_grasps(compose("gen_scene", ["num_objects=2", "enough_collision_free=6",
                                                      "enough_stable=3"]), scene, rng=0)
    cfg = compose("gen_scene", ["num_objects=2", "enough_collision_free=6", "enough_stable=1",
                                "save_collision_grasps=true", "only_collision_free=true"])
    res, neg = gen_scene.filter_grasps(cfg, scene, rng=0)
    assert [r["object_id"] for r in res] == ["id_a", "id_b"] and [len(r["pose"]) for r in res] == [3, 3]
    assert np.allclose(res[1]["pose"][:, 0, 3], 1.0) and np.allclose(res[1]["pose"][:, 2, 3], [0, 2, 4])
    assert [len(r["pose"]) for r in neg] == [3, 3]
    with pytest.raises(ValueError, match="Not enough collision free"):
        gen_scene.filter_grasps(compose("gen_scene", ["enough_collision_free=7"]), scene, rng=0)
    # the stable pass keeps the reference's unshuffled indices unless fix_shuffle
    from mgs.env.gravityless_object_grasping import apply_enough_stable
    base = ["num_objects=2", "enough_collision_free=6", "enough_stable=2"]
    quirk, _ = gen_scene.filter_grasps(compose("gen_scene", base), scene, rng=0)
    fixed, _ = gen_scene.filter_grasps(compose("gen_scene", base + ["fix_shuffle=true"]), scene, rng=0)
    perm = np.random.default_rng(0).permutation(6)
    idx = np.array([0, 0, 0, 1, 1, 1])
    stable = apply_enough_stable(np.arange(6) % 3 == 0, 2)
    assert [r["object_id"] for r in quirk] == [["id_a", "id_b"][i] for i in np.unique(idx[stable])]
    assert [r["object_id"] for r in fixed] == [["id_a", "id_b"][i] for i in np.unique(idx[perm][stable])]


def test_oracle_free_simulation(senv):
    """simulate_batch is the rollout loop with its checks off: vstate = the model's
    qvel0 / qacc_ws0 equals vstate=None, identical states stay identical, vclip
    bounds qvel, and the settled fixture pile barely moves."""
    from oracle import oracle as O
    st = np.tile(senv.get_state(), (2, 1))
    plan, vs = senv.free_plan(st, 20)
    plan.check_every = [1]           # ignored by a free simulation
    om = O.OracleModel(senv.model_for(st[0]), ncon_max=senv.ncon_max, nefc_max=256)
    a = om.simulate_batch(plan, vstate=vs, nthreads=2)
    b = om.simulate_batch(plan, vstate=None, nthreads=2)
    for k in ("qpos", "qvel", "qacc_warmstart"):
        assert np.array_equal(a[k], b[k]) and np.array_equal(a[k][0], a[k][1]), k
    assert np.abs(a["qpos"][0] - plan.qpos_init[0]).max() < 1e-3
    c = om.simulate_batch(plan, vstate=vs, vclip=1e-6, nthreads=2)
    assert np.abs(c["qvel"]).max() <= 1e-6
    out = senv.apply_free(st, a, 20)
    assert out[0, 0] == pytest.approx(st[0, 0] + 0.02)
    assert np.array_equal(senv.split_state(out[0])["qpos"][senv._gripper_nq:senv._gripper_nq + 7],
                          senv.split_state(st[0])["qpos"][senv._gripper_nq:senv._gripper_nq + 7])


def _oracle_simulate_states(env, states, nsteps, vclip=0.0, max_ncon=128, ncon_max=None):
    """ClutterTableEnv.simulate_states with the oracle in place of mgs_simulate
    (same capacity escalation)."""
    from oracle import oracle as O
    states = np.atleast_2d(states)
    plan, vs = env.free_plan(states, nsteps)

    def run(nc, p, v, first=False):
        eng = env._sim_engine(states[0], nc) if first else env.engine_for_state(states[0], ncon_max=nc)
        om = O.OracleModel(env.model_for(states[0]), ncon_max=nc, nefc_max=eng.desc.nefc_max)
        return om.simulate_batch(p, vstate=v, vclip=vclip, nthreads=8)

    cap = env.ncon_max if ncon_max is None else ncon_max
    res = run(cap, plan, vs, first=True)
    ov = np.nonzero(res["stats"][:, 2])[0]
    while len(ov) and cap < max_ncon:
        cap = min(2 * cap, max_ncon)
        sub = run(cap, plan.subset(ov), vs[ov])
        for k in res:
            res[k][ov] = sub[k]
        ov = ov[np.nonzero(sub["stats"][:, 2])[0]]
    return env.apply_free(states, res, nsteps)


@pytest.mark.gpu
def test_simulate_gpu_parity(senv):
    _gpu()
    from oracle import oracle as O
    rng = np.random.default_rng(5)
    st = np.tile(senv.get_state(), (6, 1))
    v0 = 1 + senv.ref_nq
    for i, (_, qs, vs) in enumerate(senv._obj_slices()):
        st[i, 1 + qs.start + 2] += 0.05                           # lift one object per state ...
        st[i, v0 + vs.start + 3:v0 + vs.start + 6] = rng.normal(size=3)   # ... and spin it
    plan, vs = senv.free_plan(st, 150)
    eng = senv.engine_for_state(st[0])
    g = eng.simulate(plan, vstate=vs, vclip=50.0)
    om = O.OracleModel(senv.model_for(st[0]), ncon_max=senv.ncon_max, nefc_max=eng.desc.nefc_max)
    o = om.simulate_batch(plan, vstate=vs, vclip=50.0, nthreads=8)
    for k in ("qpos", "qvel", "qacc_warmstart", "stats"):
        assert np.array_equal(g[k], o[k]), k
    assert np.abs(g["qpos"][:5] - plan.qpos_init[:5]).max() > 1e-3      # the perturbed piles moved


@pytest.mark.gpu
def test_gen_clutter_and_is_stable_gpu_vs_oracle():
    _gpu()
    from make_clutter_scene import make_env
    env = make_env()
    got = env.gen_clutter_states(2, np.random.default_rng(11), steps_each=80, steps_final=160)
    ref_env = make_env()
    ref_env.simulate_states = lambda s, n, vclip=0.0, ncon_max=None: \
        _oracle_simulate_states(env, s, n, vclip, ncon_max=ncon_max)
    ref = ref_env.gen_clutter_states(2, np.random.default_rng(11), steps_each=80, steps_final=160)
    assert np.array_equal(got, ref)
    # a smaller starting capacity (auto-sized rows, escalation on overflow) is exact too
    got24 = env.gen_clutter_states(2, np.random.default_rng(11), steps_each=80, steps_final=160, ncon_max=24)
    ref24 = ref_env.gen_clutter_states(2, np.random.default_rng(11), steps_each=80, steps_final=160, ncon_max=24)
    assert np.array_equal(got24, ref24)
    ok, mx, adv = env.is_stable_states(got, rounds=2, steps=40)
    ok2, mx2, adv2 = ref_env.is_stable_states(ref, rounds=2, steps=40)
    assert np.array_equal(mx, mx2) and np.array_equal(adv, adv2) and np.array_equal(ok, ok2)


@pytest.mark.gpu
def test_gen_scene_cli(tmp_path, monkeypatch):
    """gen_scene.py end to end: a 4-object pile of the fast subset settled on the
    GPU (4 candidate piles at once), grasps filtered, files written."""
    _gpu()
    from mgs.cli import gen_scene
    from mgs.env.selector import load_scene
    from mgs.obj.selector import get_object
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.const import ASSET_PATH
    fast = open(os.path.join(ASSET_PATH, "mj-objects", "fast_eta_objects.txt")).read().splitlines()
    for k, oid in enumerate(fast):
        h, j, _ = robotiq_candidates(get_object(oid), 256, seed=k)
        d = tmp_path / "in" / "Robotiq2f85Gripper" / oid
        d.mkdir(parents=True)
        np.savez(d / "stable_grasps.npz", pose=np.asarray(h, np.float32), joints=j)
    monkeypatch.setenv("MGS_INPUT_DIR", str(tmp_path / "in"))
    monkeypatch.setenv("MGS_OUTPUT_DIR", str(tmp_path / "out"))
    out = gen_scene.run(["gripper=robotiq_2f_85", "seed=3", "num_objects=4", "scene_batch=4", "steps_each=300",
                         "steps_final=2000", "lift_steps=300", "enough_collision_free=4", "enough_stable=1",
                         "save_collision_grasps=true"])
    assert out is not None
    sd = load_scene(os.path.join(out, "scene.npz"))
    assert len(sd["objects"]) == 4
    files = [f for f in os.listdir(out) if f != "scene.npz"]
    assert any(not f.endswith("_collision.npz") for f in files)
    for f in files:
        z = np.load(os.path.join(out, f))
        assert z["pose"].shape[1:] == (4, 4) and len(z["pose"]) == len(z["joints"])


def test_gen_scene_refuses_oversized_pile_before_any_compile(monkeypatch):
    """the reference draws pile sizes at random (mgs/obj/selector.py:124-130;
    num_objects overrides it, cli/config/gen_scene.yaml:10); the kernels hold
    at most 128 dofs, so gen_scene refuses a Shadow pile of 17 with the limit in
    the message, from the model sizes alone: no code object is compiled and
    nothing is simulated"""
    from mgs.cli import gen_scene
    from mgs.cli._hydra import compose
    from mgs.core import special

    def no_compile(*a, **k):
        raise AssertionError("a code object was compiled")
    monkeypatch.setattr(special, "compile_object", no_compile)
    cfg = compose("gen_scene", ["num_objects=17", "gripper=shadow"])
    with pytest.raises(ValueError, match=r"nv=\d+; the kernels hold at most 128 dofs, i.e. piles of at most 16 free"):
        gen_scene.gen_stable_scene(cfg, rng=0)
