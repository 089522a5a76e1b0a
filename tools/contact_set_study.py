"""Label sensitivity to the contact set.

Runs the CPU oracle (test infrastructure: the checker, never the product) on
the same candidate blocks under three contact models (mgs_model_desc.ccd_mode):

  r5        round 5's contract: MPR + face clipping (<= 4 points per convex
            pair), spheres / capsules as hull (+) ball through MPR
  multiccd  MuJoCo 3.2.2 restated: libccd's MPR penetration, multiccd (4
            perturbed MPRs, <= 5 contacts per convex pair), analytic sphere /
            capsule / box / cylinder colliders -- the envs' option set
  single    the same without multiccd (one MPR contact per convex pair)

and reports, for every pair of models, how many collision-mask entries,
labels and fail steps differ, with the contact / row statistics.  Blocks:
the bench's 8192-candidate headline block (Robotiq x 003_cracker_box, seed 0)
at h200 and at ref8000 (every collision-free candidate), and Allegro x the
GSO-format mug (config C4's pair).  Full capacity (64 contacts, 256 rows), so
no capacity escalation is involved.

  python tools/contact_set_study.py [--n 8192] [--threads 8] [--out profiles/r06_contact_set_study.json]
"""
import argparse
import copy
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mj-grasp-sim_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

MODES = ["r5", "multiccd", "single"]


def model_variant(cm, mode):
    v = copy.copy(cm)
    v.options = dict(cm.options)
    if mode == "r5":
        v.options["contact_model"] = "r5"
    else:
        v.options["contact_model"] = "mujoco"
        v.options["multiccd"] = mode == "multiccd"
    return v


def run_block(name, env, poses, joints, horizons, threads, ncon=64, nefc=256):
    from mgs.env.gravityless_object_grasping import HORIZONS
    from oracle import oracle as O
    out = {"block": name, "n": int(len(poses))}
    q, mp, mq, _ = env.initial_state(poses, joints)
    masks, res = {}, {}
    for mode in MODES:
        om = O.OracleModel(model_variant(env.model, mode), ncon_max=ncon, nefc_max=nefc)
        t0 = time.time()
        masks[mode] = om.collision_free(q, mp, mq, nthreads=threads)
        out.setdefault("mask_s", {})[mode] = round(time.time() - t0, 2)
    free = masks["multiccd"]
    idx = np.nonzero(free)[0]
    out["collision_free"] = {m: int(masks[m].sum()) for m in MODES}
    out["mask_differs"] = {f"{a}/{b}": int((masks[a] != masks[b]).sum())
                           for i, a in enumerate(MODES) for b in MODES[i + 1:]}
    for hz in horizons:
        h = HORIZONS[hz]
        plan = env.rollout_plan(poses[idx], joints[idx], nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                                close_steps=h["close_steps"], lift_check_every=h["lift_check_every"])
        r = {}
        for mode in MODES:
            om = O.OracleModel(model_variant(env.model, mode), ncon_max=ncon, nefc_max=nefc)
            t0 = time.time()
            r[mode] = om.rollout(plan, nthreads=threads)
            el = time.time() - t0
            st = r[mode]["stats"]
            steps = np.maximum(1, st[:, 4] * 0 + 1)
            out.setdefault(hz, {}).setdefault("per_model", {})[mode] = {
                "seconds": round(el, 2), "stable": int(r[mode]["label"].sum()),
                "max_ncon": int(st[:, 0].max()) if len(st) else 0,
                "max_nefc": int(st[:, 1].max()) if len(st) else 0,
                "capacity_flagged": int(((st[:, 2] & 3) != 0).sum()),
                "sum_ncon": int(st[:, 4].sum()), "sum_nefc": int(st[:, 5].sum()),
                "solver_iters": int(st[:, 3].sum())}
            del steps
        cmp = {}
        for i, a in enumerate(MODES):
            for b in MODES[i + 1:]:
                la, lb = r[a]["label"], r[b]["label"]
                fa, fb = r[a]["fail_step"], r[b]["fail_step"]
                dq = np.abs(r[a]["obj_qpos"][:, :3] - r[b]["obj_qpos"][:, :3]).max(1) if len(idx) else np.zeros(0)
                cmp[f"{a}/{b}"] = {"labels_differ": int((la != lb).sum()),
                                   "stable_to_unstable": int((la & ~lb).sum()),
                                   "unstable_to_stable": int((~la & lb).sum()),
                                   "fail_steps_differ": int((fa != fb).sum()),
                                   "obj_pos_diff_median_m": float(np.median(dq)) if len(dq) else 0.0,
                                   "obj_pos_diff_p90_m": float(np.percentile(dq, 90)) if len(dq) else 0.0}
        out[hz]["compare"] = cmp
        out[hz]["rollouts"] = int(len(idx))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--n-allegro", type=int, default=2048)
    ap.add_argument("--threads", type=int, default=min(8, len(os.sched_getaffinity(0))))
    ap.add_argument("--horizons", default="h200,ref8000")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_contact_set_study.json"))
    ap.add_argument("--skip-allegro", action="store_true")
    a = ap.parse_args()
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_object
    from mgs.sampler.antipodal import hand_candidates, robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose
    hz = a.horizons.split(",")
    recs = []
    env = GravitylessObjectGrasping(GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz")),
                                    get_object("003_cracker_box"))
    H, J, _ = robotiq_candidates(env.obj, a.n, seed=0)
    recs.append(run_block("robotiq_x_003_cracker_box (bench block, seed 0)", env, SE3Pose.from_mat(H),
                          np.asarray(J, np.float64), hz, a.threads))
    print(json.dumps(recs[-1]), flush=True)
    if not a.skip_allegro:
        aenv = GravitylessObjectGrasping(get_gripper({"name": "AllegroGripper"}), get_object("Synthetic_Mug_Body"))
        H, J, _ = hand_candidates(aenv.obj, a.n_allegro, aenv.gripper, seed=0)
        recs.append(run_block("allegro_x_Synthetic_Mug_Body (GSO-format stand-in, seed 0)", aenv, SE3Pose.from_mat(H), J, ["h200"], a.threads))
        print(json.dumps(recs[-1]), flush=True)
    meta = {"what": "label sensitivity to the contact set (oracle, full capacity)", "modes": MODES,
            "date": time.strftime("%Y-%m-%d"), "threads": a.threads}
    with open(a.out, "w") as f:
        json.dump({"meta": meta, "blocks": recs}, f, indent=1)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
