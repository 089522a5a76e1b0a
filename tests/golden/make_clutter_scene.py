"""Generate tests/golden/clutter_scene.npz: a settled 5-object pile for the
ClutterTableEnv tests.

TEST INFRASTRUCTURE ONLY.  The reference's scenes come from
ClutterTableEnv.gen_clutter (mgs/env/clutter_table.py:197-222) under MuJoCo,
which is not installed; this script restates gen_clutter on the CPU oracle:
the gripper parked at (5, 5, 1) (gen_scene.py:31-34), one random drop pose at
(0, 0, 0.8) shared by all objects, each object placed there in turn with qvel
zeroed and 900 steps, then 9000 steps to settle, qvel clipped to +-50 after
every step; is_stable's criterion (:155-195) is checked on 1000 more steps.
The scene is seeded (numpy default_rng(0)) and the object names are fixed, so
the fixture is reproducible.  Output: the mjSTATE_INTEGRATION vector of the
reference model layout, the object ids and names.

    python tests/golden/make_clutter_scene.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "mj-grasp-sim_amd")):
    sys.path.insert(0, p)

OBJECT_IDS = ["010_potted_meat_can", "061_foam_brick", "005_tomato_soup_can", "017_orange", "061_foam_brick"]
GRIPPER = "Robotiq2f85Gripper"
OUT = os.path.join(HERE, "clutter_scene.npz")
# `python make_clutter_scene.py ShadowHand` -> clutter_scene_shadow.npz (config C5's gripper)
OUTS = {"Robotiq2f85Gripper": OUT, "ShadowHand": os.path.join(HERE, "clutter_scene_shadow.npz")}


def make_env(gripper_name=GRIPPER, object_ids=OBJECT_IDS):
    from mgs.env.clutter_table import ClutterTableEnv
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_object
    from mgs.util.geo.transforms import SE3Pose
    grip = get_gripper({"name": gripper_name},
                       default_pose=SE3Pose(np.array([5.0, 5.0, 1.0]), np.array([1.0, 0, 0, 0]), "wxyz"))
    objs = [get_object(oid, name=f"obj{i}") for i, oid in enumerate(object_ids)]
    return ClutterTableEnv(grip, objs, scene_randomization=False)


def settle(env, rng, steps_each=900, steps_final=9000, vclip=50.0):
    from scipy.spatial.transform import Rotation
    from oracle import oracle as O
    st = env.split_state(env.get_state())
    qpos = st["qpos"].copy()
    qvel = np.zeros(env.ref_nv)
    ws = np.zeros(env.ref_nv)
    xyzw = Rotation.random(random_state=rng.integers(1 << 31)).as_quat()
    drop = np.concatenate([[0.0, 0.0, 0.8], [xyzw[3], xyzw[0], xyzw[1], xyzw[2]]])
    t = 0.0

    def run(q, v, w, n):
        parts = dict(st, qpos=q, qvel=v, qacc_warmstart=w)
        state = env.join_state(parts)
        cm = env.model_for(state)
        om = O.OracleModel(cm, ncon_max=64, nefc_max=256)
        qr = env._reduce(q, "q")
        qn, vn, wn = om.simulate(qr, st["mocap_pos"], st["mocap_quat"], np.zeros(max(cm.nu, 1)), n, vclip)
        return env_expand(env, q, qn, "q"), env_expand(env, v, vn, "v"), env_expand(env, w, wn, "v")

    for name, qs, vs in env._obj_slices():
        qpos[qs] = drop
        qvel[:] = 0.0
        qpos, qvel, ws = run(qpos, qvel, ws, steps_each)
        t += steps_each * 1e-3
    qpos, qvel, ws = run(qpos, qvel, ws, steps_final)
    t += steps_final * 1e-3
    st = dict(st, time=np.array([t]), qpos=qpos, qvel=qvel, qacc_warmstart=ws)
    return env.join_state(st)


def env_expand(env, ref_vec, reduced, which):
    """write a compiled-model vector back into the reference layout."""
    out = np.array(ref_vec, dtype=np.float64).copy()
    gq, gv = env._gripper_nq, env._gripper_nv
    h = gq if which == "q" else gv
    out[:h] = reduced[:h]
    o = h
    for name, qs, vs in env._obj_slices():
        if name in env.removed:
            continue
        sl = qs if which == "q" else vs
        w = sl.stop - sl.start
        out[sl] = reduced[o:o + w]
        o += w
    return out


def main():
    gname = sys.argv[1] if len(sys.argv) > 1 else GRIPPER
    env = make_env(gname)
    rng = np.random.default_rng(0)
    state = settle(env, rng)
    env.set_state(state)
    # is_stable (:155-195): summed |displacement| of every object over 10 x 100 steps < 5e-3
    s2 = settle_more(env, state, 1000)
    q0, q1 = env.split_state(state)["qpos"], env.split_state(s2)["qpos"]
    drift = max(np.abs(q1[qs][:3] - q0[qs][:3]).sum() for _, qs, _ in env._obj_slices())
    print("object z:", [round(float(q0[qs][2]), 4) for _, qs, _ in env._obj_slices()], "drift", drift)
    np.savez(OUTS[gname], state=state, object_ids=np.array(OBJECT_IDS), gripper=np.array(gname), drift=drift)
    print("wrote", OUTS[gname], state.shape)


def settle_more(env, state, n):
    from oracle import oracle as O
    st = env.split_state(state)
    cm = env.model_for(state)
    om = O.OracleModel(cm, ncon_max=64, nefc_max=256)
    qn, vn, wn = om.simulate(env._reduce(st["qpos"], "q"), st["mocap_pos"], st["mocap_quat"],
                             np.zeros(max(cm.nu, 1)), n, 50.0)
    return env.join_state(dict(st, qpos=env_expand(env, st["qpos"], qn, "q")))


if __name__ == "__main__":
    main()
